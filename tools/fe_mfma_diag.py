"""Diagnostic: the u8 FE on the MFMA path vs the vector path (SDR_FE_MFMA=0 in a child), first
mismatching demod outputs per stream (tile = 256 outputs)."""
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1:                     # child: write the demod to the given file
    import rtsdr
    iq = rtsdr.synth.fm_iq(200 * 2560 + 777, seed=3, dtype=np.uint8)
    b, _ = rtsdr.design.mono_coeffs(151, 151)
    d, *_ = rtsdr.rf_frontend_block(iq, b, None, None, 0.0)
    np.save(sys.argv[1], np.asarray(d))
    sys.exit(0)
out = {}
for mode in ("1", "0"):
    f = f"/tmp/fe_diag_{mode}.npy"
    subprocess.run([sys.executable, __file__, f], check=True, env=dict(os.environ, SDR_FE_MFMA=mode))
    out[mode] = np.load(f)
a, b = out["1"], out["0"]
err = np.abs(a - b)
bad = np.nonzero(err > 1e-4)[0]
print("n", len(a), "max err", err.max(), "bad", len(bad))
if len(bad):
    print("first bad", bad[:20], "tiles", sorted(set((bad // 256).tolist()))[:40])
