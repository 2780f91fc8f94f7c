"""A/B of the parallel PLL solve: run with SDR_PLL_SPEC=0 and =1 (read once per process).
Prints the NCO error against the oracle and the time per sdr_pll call (host buffers)."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import rtsdr
import fm_oracle as oracle

FS = 240e3
for B, df in ((5120, 3.0), (15360, 0.0), (15360, 3.0), (15360, 10.0)):
    rng = np.random.default_rng(1)
    t = np.arange(40 * B)
    x = (np.cos(2 * np.pi * (19e3 + df) / FS * t + 0.3) + 0.05 * rng.standard_normal(t.size)).astype(np.float32)
    st = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]; sr = list(st); err = 0.0
    for k in range(4):
        nco, _, st = rtsdr.fmPll(x[k * B:(k + 1) * B], 19e3, FS, st, 2.0)
        nr, _, sr = oracle.fm_pll(x[k * B:(k + 1) * B].astype(np.float64), 19e3, FS, sr, 2.0)
        err = max(err, float(np.abs(nco[1:] - nr[1:]).max()))
    t0 = time.perf_counter()
    for k in range(4, 40):
        rtsdr.fmPll(x[k * B:(k + 1) * B], 19e3, FS, st, 2.0)
    dt = (time.perf_counter() - t0) / 36
    print(f"SDR_PLL_SPEC={os.environ.get('SDR_PLL_SPEC', '1')} block {B}, pilot offset {df:g} Hz: max NCO err {err:.2e}, {dt * 1e6:.1f} us per sdr_pll call", flush=True)
