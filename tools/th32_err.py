#!/usr/bin/env python3
"""The compact phase rows' precision (sdr_nco.h "compact phase rows"): the pilot loop's
phases (a Python restatement of fmPll on the oracle's pilot-BPF rows of a synthetic FM stream)
cut into 32-row lines, each row's f32 residual against its line, and the angle error that
rounding makes (x ncoScale 2): a flat line (the line's start) against a straight one (start +
slope), at acquisition and once locked.  Test infrastructure: reads oracle/.
usage: python3 tools/th32_err.py [seed]"""
import math
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "real-time-software-defined-radio_amd"))
from oracle import fm_oracle as O  # noqa: E402
import synth  # noqa: E402

iq = synth.fm_iq(153600 * 5, seed=int(sys.argv[1]) if len(sys.argv) > 1 else 0)
blocks = O.mono_stereo_blocks(iq, 153600, nblocks=4)
x = np.concatenate([b["bpf_recovery"] for b in blocks])
def pll_phases(x, freq, Fs, bw, scale):
    Kp = bw * 2.666; Ki = bw * bw * 3.555
    integ, phase, fI, fQ, off = 0.0, 0.0, 1.0, 0.0, 0.0
    w = 2 * math.pi * freq / Fs
    ph = np.empty(len(x))
    for k in range(len(x)):
        e = math.atan2(x[k] * (-fQ), x[k] * fI)
        integ += Ki * e; phase += Kp * e + integ
        arg = w * (off + k + 1) + phase
        fI = math.cos(arg); fQ = math.sin(arg)
        ph[k] = phase
    return ph
ph = pll_phases(x, 19e3, 240e3, 0.01, 2)
n = len(ph) // 32 * 32
P = ph[:n].reshape(-1, 32)
o = np.arange(32)
prev = np.concatenate([[0.0], P[:-1, -1]])
for name, A, S in (("flat (A = chunk start)", P[:, :1], 0 * P[:, :1]),
                   ("linear, slope of the chunk", prev[:, None] + (P[:, -1:] - prev[:, None]) / 32, (P[:, -1:] - prev[:, None]) / 32)):
    base = A + S * o
    r = P - base
    err = np.abs(r.astype(np.float32).astype(np.float64) - r) * 2   # x scale 2
    w = np.argmax(err.max(1))
    print(f"{name}: max|r| {np.abs(r).max():.3g} rad, max angle err {err.max():.3g} (chunk {w}, step {32*w}), "
          f"after 1000 steps {err[1000//32:].max():.3g}, after 5000 {err[5000//32:].max():.3g}")
