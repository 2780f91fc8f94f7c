"""Diagnostic (GPU box): where does the K = 256 bench-shape span leave the per-block loop?
Prints, for the RDS PLL input (pre_pll) and NCO (nco_i), the first blocks whose outputs
differ beyond rounding, and every pre_pll sample whose sign differs between the two paths.
usage: python tools/diag/span_flip.py [seed]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import rtsdr as sdr  # noqa: E402

B5, K, spans = 153_600, 256, 2
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 7
names = ["pre_pll", "nco_i", "extract"]
iq = sdr.synth.fm_iq(K * spans * B5 + 1, seed=seed, dtype=np.uint8)[None, :]
kw = dict(stereo=True, rds=True, iq_dtype=np.uint8)
span_rx = sdr.Receiver(1, K * B5, **kw)
got = [span_rx.process(iq[:, 2 * sp * K * B5:2 * (sp + 1) * K * B5], fetch=names) for sp in range(spans)]
per_rx = sdr.Receiver(1, B5, **kw)
M = B5 // 10
shown = 0
flips = []
for k in range(K * spans):
    p = per_rx.process(iq[:, 2 * k * B5:2 * (k + 1) * B5], fetch=names)
    sp, kk = divmod(k, K)
    w = p["pre_pll"][0]
    g = got[sp]["pre_pll"][0][kk * M:(kk + 1) * M]
    d = np.nonzero(np.sign(w) != np.sign(g))[0]
    for i in d:
        flips.append((k, int(i), float(w[i]), float(g[i])))
    wn = p["nco_i"][0]
    gn = got[sp]["nco_i"][0][kk * M:kk * M + M + 1]
    e = float(np.max(np.abs(wn - gn)))
    if e > 1e-5 and shown < 6:
        j = int(np.argmax(np.abs(wn - gn) > 1e-5))
        print(f"block {k}: nco_i max diff {e:.3e}, first at offset {j}; pre_pll diff there "
              f"{float(np.max(np.abs(w - g))):.3e}", flush=True)
        shown += 1
print("pre_pll sign flips (block, offset, per-block, span):", flips[:20], "total", len(flips))
peak = max(float(np.max(np.abs(got[sp]["pre_pll"][0]))) for sp in range(spans))
print("pre_pll peak", peak)
