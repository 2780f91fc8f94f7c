"""Diagnostic: fe_mfma_mono_kernel time per sample against the work split -- one u8 stream whose
audio-block count is k x the wave count (every wave the same run) or the bench's 10 240.
usage: python3 tools/diag/u8_balance.py [audio_blocks ...]   (SDR_FE_MFMA_WPC= for waves per CU)"""
import json
import os
import sys
import time

import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import rtsdr
from importlib import import_module

_lib = import_module("real-time-software-defined-radio_amd._lib")
ctx = rtsdr.get_context()
lib, h = ctx.lib, ctx.handle
rf_b, au_b = rtsdr.design.mono_coeffs(101, 151)
rfp, aup = _lib.f64p(rf_b), _lib.f64p(au_b)
out = []
for ab in [int(a) for a in sys.argv[1:]] or [9216, 10240, 12288]:
    n = ab * 12800
    M = (n + 9) // 10
    A = (M + 4) // 5
    d_iq = _lib.DeviceBuffer.from_array(ctx, rtsdr.synth.fm_iq(n, seed=1, dtype=np.uint8))
    d_au = _lib.DeviceBuffer(ctx, 4 * A)

    def launch():
        _lib.check(lib.sdr_fe_mono_dev(h, d_iq.ptr, _lib.SDR_IQ_U8, n, n, 1, rfp, 101, 10, aup, 151, 5, d_au.ptr, A), "u8")

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for _ in range(16):
            launch()
        ctx.synchronize()
    tm = _lib.Timer(ctx)
    e0, e1 = tm.event(), tm.event()
    tm.record(e0)
    for _ in range(50):
        launch()
    tm.record(e1)
    ms = tm.elapsed_ms(e0, e1) / 50
    tm.close()
    d_iq.free()
    d_au.free()
    r = {"audio_blocks": ab, "samples": n, "us": round(ms * 1e3, 2), "us_per_131M": round(ms * 1e3 * 131072000 / n, 2),
         "wpc": os.environ.get("SDR_FE_MFMA_WPC", "default")}
    print(json.dumps(r), flush=True)
    out.append(r)
