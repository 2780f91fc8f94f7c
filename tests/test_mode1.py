"""Mode-1 audio resampler: 250 kS/s IF -> 48 kHz by 24/125 through a
3 623-tap filter at 6 MHz (src/fm_radio.cpp:174-180, :228; src/filter.cpp:222-298).

The pin is tests/golden/mode1.npz, written by make_mode1_golden.py with the reference's own
convolveWithDecimMode1 compiled from its sources.  Parity bar:
  * block 0 (zero history): every output the reference writes (floor(n*24/125));
  * later blocks: outputs 29.. (those whose 151 terms are all inside the block).  The
    reference's first 28 outputs read its raw history at zi[(Z-1-count)/up]
    (src/filter.cpp:249), not the previous block's tail; this build carries the stream
    continuously (lfilter state on the zero-stuffed stream) -- DESIGN.md §8.
The reference's y has no up-gain (it multiplies by 24 at the int16 write, :297), so it is
compared with y / 24.  Tolerance 2e-6 (f32 accumulation of 151 terms; |y| <= 0.06).
"""
import numpy as np
import pytest

TOL = 2e-6


def _blocks(z):
    B, up, down = int(z["block"]), int(z["up"]), int(z["down"])
    nb = len(z["x"]) // B
    ny = B * up // down
    first = -(-(len(z["taps"]) - 1) // down)      # 29: first output without history terms
    return B, up, down, nb, ny, first


def _check(y_blocks, z):
    B, up, down, nb, ny, first = _blocks(z)
    ref = z["y"].reshape(nb, ny)
    for b, y in enumerate(y_blocks):
        lo = 0 if b == 0 else first
        assert np.max(np.abs(y[lo:ny] / up - ref[b, lo:])) < TOL, b


def test_oracle_resampler_matches_reference(oracle, golden):
    z = golden("mode1.npz")
    B, up, down, nb, ny, first = _blocks(z)
    h = z["taps"].astype(np.float64)
    zi = np.zeros(len(h) - 1)
    out = []
    for b in range(nb):
        y, zi = oracle.resample(z["x"][b * B:(b + 1) * B].astype(np.float64), h, zi, up, down)
        assert len(y) == ny + 1                  # ceil(n*up/down): one more than the reference
        out.append(y)
    _check(out, z)


@pytest.mark.gpu
def test_gpu_mode1_resampler(sdr, gpu_ctx, golden, oracle):
    z = golden("mode1.npz")
    B, up, down, nb, ny, first = _blocks(z)
    h = z["taps"].astype(np.float64)
    zi = np.zeros(len(h) - 1)
    zo = zi.copy()
    out = []
    for b in range(nb):
        x = z["x"][b * B:(b + 1) * B]
        y, zi = sdr.resample(x, h, zi, up, down)
        yo, zo = oracle.resample(x.astype(np.float64), h, zo, up, down)
        assert y.shape == yo.shape
        assert np.max(np.abs(y - yo)) < up * TOL and np.max(np.abs(zi - zo)) < 1e-9
        out.append(y)
    _check(out, z)


@pytest.mark.gpu
def test_gpu_resampler_tap_limit(sdr, gpu_ctx):
    x = np.ones(1000, np.float32)
    with pytest.raises(ValueError):
        sdr.resample(x, np.ones(4097) / 4097, np.zeros(4096), 24, 125)
    y, _ = sdr.resample(x, np.ones(4096) / 4096, np.zeros(4095), 24, 125)
    assert np.all(np.isfinite(y))
