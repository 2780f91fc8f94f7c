#!/usr/bin/env python3
"""Diagnostic (GPU): the span receiver (S streams x K blocks of 153 600, stereo + RDS, u8) against
the per-block receiver on the same input (tests/test_span.py's first case): per stream and
output, the largest difference and where it is (block, index).  Run with each library
(SDR_LIB) to see which build parts from the block loop.
usage: python3 tools/diag/th32_vs_blocks.py [S] [K] [spans]"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
B5 = 153_600
NAMES = ["nco", "stereo", "left", "bpf_recovery", "nco_i", "lpf_i"]


def main():
    import rtsdr as sdr
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    spans = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    nblk = K * spans
    iq = np.stack([sdr.synth.fm_iq(nblk * B5 + 1, seed=70 + s, dtype=np.uint8) for s in range(S)])
    kw = dict(stereo=True, rds=True, iq_dtype=np.uint8)
    per_rx = sdr.Receiver(S, B5, **kw)
    per = [per_rx.process(iq[:, 2 * k * B5:2 * (k + 1) * B5], fetch=NAMES) for k in range(nblk)]
    span_rx = sdr.Receiver(S, K * B5, **kw)
    got = []
    for sp in range(spans):
        got.append(span_rx.process(iq[:, 2 * sp * K * B5:2 * (sp + 1) * K * B5], fetch=NAMES))
        print("stats", span_rx.pll_stats())
    for s in range(S):
        for name in NAMES:
            worst = (0.0, -1, -1)
            for k in range(nblk):
                sp, kk = divmod(k, K)
                w = np.asarray(per[k][name][s], dtype=np.float64)
                n = len(w) - 1 if name in ("nco", "nco_i") else len(w)
                g = np.asarray(got[sp][name][s][kk * n:kk * n + len(w)], dtype=np.float64)
                d = np.abs(g - w)
                d[np.isnan(d)] = np.inf
                i = int(np.argmax(d))
                if d[i] > worst[0]:
                    worst = (float(d[i]), k, i)
            print(f"stream {s} {name}: max diff {worst[0]:.3g} at block {worst[1]} index {worst[2]}")


if __name__ == "__main__":
    main()
