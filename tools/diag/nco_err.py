"""Diagnostic: where the RDS NCO of the block receiver departs from the oracle (one u8 stream,
3 blocks), with the PLL solver counters (the r04 split A/B switch it was run under is removed)."""
import os, sys
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
import rtsdr
from conftest import _load_oracle
oracle = _load_oracle()
B5 = 153600
nb = 3
iq = rtsdr.synth.fm_iq(nb * B5 + 1, seed=0, dtype=np.uint8)
ctx = rtsdr.get_context()
for stereo in (False, True):
    rx = rtsdr.Receiver(1, B5, stereo=stereo, rds=True, iq_dtype=np.uint8)
    rds = oracle.rds_blocks(iq, 2 * B5, taps=151, nblocks=nb, pll_fn=oracle.fm_pll_c)
    for k in range(nb):
        ctx.pll_stats(reset=True)
        g = rx.process(iq[None, 2 * k * B5:2 * (k + 1) * B5], fetch=["nco_i", "nco_q", "pre_pll"])
        st = rx.pll_stats()
        for key in ("pre_pll", "nco_i", "nco_q"):
            e = np.abs(g[key][0].astype(np.float64) - rds[k][key])
            bad = np.nonzero(e > 1e-6)[0]
            print(f"stereo={stereo} block {k} {key}: max {e.max():.2e} at {int(e.argmax())}, {len(bad)} > 1e-6"
                  + (f" first {bad[:6]} last {bad[-3:]}" if len(bad) else ""))
        print("   counters", {k2: v for k2, v in st.items() if v})
    rx.close()
