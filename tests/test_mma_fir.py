"""The matrix-core FIR's arithmetic (csrc/rx.hip rx_mma_kernel): f16 hi/lo operand splits
(v = hi + lo / 2048), three f16 products per tap accumulated in f32, the lo x lo product
dropped.  A numpy emulation of that arithmetic against f64 lfilter, next to the f32 direct
form the VALU tiles compute: the split form must be as accurate (the receiver's parity
tolerances were set on the f32 form).  CPU only; the GPU kernel itself is checked through the
span tests (tests/test_span.py: the same outputs against the per-block VALU path and the
oracle)."""
import numpy as np
import pytest
from scipy.signal import firwin, lfilter

LO = np.float32(2048.0)


def split(v):
    v = v.astype(np.float32)
    hi = v.astype(np.float16).astype(np.float32)
    lo = ((v - hi) * LO).astype(np.float16).astype(np.float32)
    return hi, lo


def fir_f32(h, x):
    acc = np.zeros(len(x), np.float32)
    for k, hk in enumerate(h.astype(np.float32)):
        acc = (acc + hk * np.concatenate([np.zeros(k, np.float32), x[:len(x) - k]])).astype(np.float32)
    return acc


def fir_split(h, x):
    (xh, xl), (hh, hl) = split(x), split(h)
    acc_h = np.zeros(len(x), np.float32)
    acc_c = np.zeros(len(x), np.float32)
    for k in range(len(h)):
        sh = np.concatenate([np.zeros(k, np.float32), xh[:len(x) - k]])
        sl = np.concatenate([np.zeros(k, np.float32), xl[:len(x) - k]])
        acc_h = (acc_h + hh[k] * sh).astype(np.float32)
        acc_c = (acc_c + (hh[k] * sl + hl[k] * sh)).astype(np.float32)
    return acc_c / LO + acc_h


@pytest.mark.parametrize("band,taps", [((18.5e3, 19.5e3), 151), ((54e3, 60e3), 151), ((22e3, 54e3), 151), (None, 101)])
def test_split_fir_matches_f32_direct_accuracy(band, taps):
    fs = 240e3
    rng = np.random.default_rng(5)
    n = 12_000
    t = np.arange(n) / fs
    # a demod-like input: pilot + stereo + RDS bands, noise, and rare +-pi spikes
    x = (0.1 * np.sin(2 * np.pi * 19e3 * t) + 0.3 * np.sin(2 * np.pi * 1e3 * t) * np.cos(2 * np.pi * 38e3 * t)
         + 0.05 * np.sin(2 * np.pi * 57e3 * t + 0.3) + 0.02 * rng.standard_normal(n))
    x[rng.integers(0, n, 20)] = np.pi
    x = x.astype(np.float32)
    h = firwin(taps, [band[0] / (fs / 2), band[1] / (fs / 2)], pass_zero=False) if band else firwin(taps, 3e3 / (fs / 2))
    ref = lfilter(h, 1.0, x.astype(np.float64))
    peak = np.max(np.abs(ref))
    e32 = np.max(np.abs(fir_f32(h, x) - ref)) / peak
    esp = np.max(np.abs(fir_split(h, x) - ref)) / peak
    assert esp < 1.5 * e32 + 1e-7, (esp, e32)
    assert esp < 2e-6, esp
