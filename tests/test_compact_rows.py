"""The compact phase rows (csrc/sdr_nco.h "compact phase rows") on the CPU: the
pilot loop's phaseEst (model/fmPll.py:22-37, restated per step) on the oracle's pilot-BPF rows
of a synthetic FM stream, cut into 32-row lines, and the angle error the f32 residual's
rounding makes (x ncoScale 2, model/fmMonoBlock.py:119):

  * sloped lines (start + slope over the line, as the solve sets them from its previous pass
    over a chunk -- here the exact trajectory, what a round-0 solve's guess follows): the bound
    the NCO replay tolerance of tests/test_span.py counts on, at acquisition and once locked;
  * flat lines at a chunk's start (the solve's AF check form, middle pseudo-blocks only, i.e.
    after the first 14 336 steps of a stream): locked-loop rounding;
  * the acquisition is why the first pseudo-block keeps the slopes: a flat line there rounds
    ~5x worse.

And the matrix-core mixers' folded angle (sdr_nco.h nco4_eval_w<TH32>) against the direct
form, in f64 on the host: the same angle to rounding."""
import math

import numpy as np
import pytest

B5 = 153_600
LINE = 32
PB = 14_336           # pll.hip LONG_PB: the first pseudo-block of a stream


@pytest.fixture(scope="module")
def pilot_phases(oracle):
    import rtsdr
    iq = rtsdr.synth.fm_iq(3 * B5 + 1, seed=0)
    x = np.concatenate([b["bpf_recovery"] for b in oracle.mono_stereo_blocks(iq, B5, nblocks=3)])
    kp, ki = 0.01 * 2.666, 0.01 * 0.01 * 3.555        # model/fmPll.py:4-10, normBandwidth 0.01
    w = 2 * math.pi * 19e3 / 240e3
    integ = phase = 0.0
    fi, fq = 1.0, 0.0
    ph = np.empty(len(x))
    for k in range(len(x)):
        e = math.atan2(x[k] * (-fq), x[k] * fi)
        integ += ki * e
        phase += kp * e + integ
        arg = w * (k + 1) + phase
        fi, fq = math.cos(arg), math.sin(arg)
        ph[k] = phase
    n = len(ph) // LINE * LINE
    return ph[:n].reshape(-1, LINE)


def _angle_err(r):
    return np.abs(r.astype(np.float32).astype(np.float64) - r) * 2.0       # x ncoScale


def test_sloped_lines_round_below_the_replay_tolerance(pilot_phases):
    P = pilot_phases
    prev = np.concatenate([[0.0], P[:-1, -1]])        # the phase before each line's first row
    s = (P[:, -1] - prev) / LINE
    a = prev + s
    r = P - (a[:, None] + s[:, None] * np.arange(LINE))
    e = _angle_err(r)
    print(f"sloped lines: max angle error {e.max():.2e} rad (after 2 000 steps {e[2000 // LINE:].max():.2e}), "
          f"max |r| {np.abs(r).max():.3f} rad")
    assert e.max() < 4e-8                              # measured 2.3e-8 (acquisition)
    assert e[2000 // LINE:].max() < 1.5e-8             # measured 7.5e-9 (locked)


def test_flat_lines_after_the_first_pseudo_block(pilot_phases):
    P = pilot_phases
    prev = np.concatenate([[0.0], P[:-1, -1]])
    r = P - prev[:, None]
    e = _angle_err(r)
    af = e[PB // LINE:]
    print(f"flat lines: max angle error {af.max():.2e} rad past step {PB}, {e.max():.2e} over the stream, "
          f"max |r| past step {PB} {np.abs(r[PB // LINE:]).max():.3f} rad")
    assert af.max() < 3e-8                             # measured 1.5e-8
    assert e.max() > 4e-8                              # at acquisition a flat line would not do (1.1e-7)


def test_folded_mixer_angle_equals_the_direct_form():
    rng = np.random.default_rng(7)
    ws = 2 * math.pi * 19e3 / 240e3 * 2.0             # w scale
    scale = 2.0
    worst = 0.0
    for _ in range(2000):
        base = rng.uniform(-math.pi, math.pi)
        a = rng.uniform(-50.0, 50.0)
        s = rng.uniform(-1e-3, 1e-3)
        o = int(rng.integers(0, 29)) & ~3            # a group's first row within its line
        dk = int(rng.integers(-4, 1500))             # output index relative to the window's reference
        r = rng.uniform(-0.3, 0.3, 4).astype(np.float32).astype(np.float64)
        w2 = scale * s + ws
        g = scale * (s * (o - dk) + a) + base
        for e in range(4):
            folded = r[e] * scale + (w2 * (dk + e) + g)
            direct = (a + s * (o + e) + r[e]) * scale + (ws * (dk + e) + base)
            worst = max(worst, abs(folded - direct))
    print(f"folded vs direct angle: {worst:.2e} rad")
    assert worst < 1e-11
