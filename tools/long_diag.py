"""Diagnostic: the span receiver on bench.py's seamless synthetic span, solver counters per
span and the time of each call (run with SDR_LIB=.../libsdr_dbg.so for the chain's prints)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rtsdr  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
spans = int(sys.argv[3]) if len(sys.argv) > 3 else 4
pipe = int(sys.argv[4]) if len(sys.argv) > 4 else 1
from importlib import import_module  # noqa: E402
_lib = import_module("real-time-software-defined-radio_amd._lib")
ctx = rtsdr.get_context()
B = 153_600
n = K * B
base = rtsdr.synth.fm_iq(n, seed=0, dtype=np.uint8)
rows = np.stack([np.roll(base, 2 * ((s * n // S) // 50 * 50)) for s in range(S)])
d = _lib.DeviceBuffer.from_array(ctx, rows)
rf_b, au_b = rtsdr.design.mono_coeffs(151, 151)
rx = rtsdr.Receiver(S, n, stereo=True, rds=True, iq_dtype=np.uint8, rf_coeff=rf_b, audio_coeff=au_b,
                    pipeline=bool(pipe), ctx=ctx)
for sp in range(spans):
    rx.pll_stats(reset=True)
    t = time.perf_counter()
    rx.process_dev(d.ptr, n)
    st = rx.pll_stats()
    print(f"span {sp}: {1e3 * (time.perf_counter() - t):.2f} ms", st, flush=True)
