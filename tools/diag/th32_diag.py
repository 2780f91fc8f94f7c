#!/usr/bin/env python3
"""Diagnostic (GPU): one span of the receiver (stereo + RDS, u8, K blocks of 153 600) with the
library SDR_LIB points at; saves the stereo NCO, stereo, bpf_recovery rows to OUT.npz.  Two runs
(the compact phase rows and a -DSDR_NO_TH32 build, tools/build_dbg.sh) and `compare` locate
where their outputs part.
usage: python3 tools/diag/th32_diag.py run OUT.npz [K] | compare A.npz B.npz"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
B5 = 153_600
NAMES = ["nco", "stereo", "bpf_recovery", "left"]


def run(out, K):
    import rtsdr as sdr
    iq = sdr.synth.fm_iq(K * B5 + 1, seed=70, dtype=np.uint8)[None, :]
    rx = sdr.Receiver(1, K * B5, stereo=True, rds=True, iq_dtype=np.uint8)
    got = rx.process(iq[:, :2 * K * B5], fetch=NAMES)
    np.savez(out, **{k: np.asarray(got[k][0]) for k in NAMES}, stats=str(rx.pll_stats()))
    print("saved", out, rx.pll_stats())


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for k in NAMES:
        x, y = A[k].astype(np.float64), B[k].astype(np.float64)
        d = np.abs(x - y)
        bad = np.flatnonzero(~(d <= 1e-5))
        print(f"{k}: n {len(x)}, max diff {np.nanmax(d):.3g}, nan a/b {np.isnan(x).sum()}/{np.isnan(y).sum()}, "
              f"bad {len(bad)}" + (f", first {bad[:8]}, last {bad[-4:]}" if len(bad) else ""))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 4)
    else:
        compare(sys.argv[2], sys.argv[3])
