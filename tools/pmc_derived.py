#!/usr/bin/env python3
"""Derived per-kernel metrics from a closing set's SQ / TCC passes (tools/gpu_round.sh pmc steps).

usage: python3 tools/pmc_derived.py DIR TAG [TAG ...] > profiles/rNN/pmc_derived.md
Reads DIR/pmc_<tag>_{a,b,c,fetch,write}/pmc_counter_collection.csv and prints, per kernel
(means over its dispatches): the disjoint split of wave time into issuing / parked on
s_waitcnt / issue-stalled (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
~= WAVE_CYCLES), instructions per wave, LDS bank-conflict share, matrix-pipe busy cycles and
HBM bytes (FETCH_SIZE x 2, the gfx950 wide-read correction; WRITE_SIZE as measured)."""
import csv
import os
import sys
from collections import defaultdict


def load(path):
    agg = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return agg
    for row in csv.DictReader(open(path)):
        agg[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return agg


def short(k):
    return k.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0]


def main():
    d = sys.argv[1]
    for tag in sys.argv[2:]:
        merged = defaultdict(dict)
        for part in ("a", "b", "c", "fetch", "write"):
            for k, cs in load(os.path.join(d, f"pmc_{tag}_{part}", "pmc_counter_collection.csv")).items():
                for c, v in cs.items():
                    merged[k][c] = sum(v) / len(v)
        print(f"\n### {tag}\n")
        print("| kernel | dispatches' waves | issuing | parked (waitcnt) | issue-stalled | VALU / wave | SALU / wave "
              "| LDS / wave | LDS bank-conflict / LDS active | MFMA busy / wave-cycle | HBM read MB | HBM write MB |")
        print("|---|---|---|---|---|---|---|---|---|---|---|---|")
        for k, m in merged.items():
            if "rocclr" in k or "probe" in k:
                continue
            wc = m.get("SQ_WAVE_CYCLES", 0.0)
            w = m.get("SQ_WAVES", 0.0) or 1.0
            f = lambda c: m.get(c, float("nan"))
            frac = lambda c: f"{f(c) / wc:.2f}" if wc else "-"
            conf = (f"{f('SQ_LDS_BANK_CONFLICT') / f('SQ_LDS_IDX_ACTIVE'):.2f}"
                    if m.get("SQ_LDS_IDX_ACTIVE") else "-")
            mfma = (f"{f('SQ_VALU_MFMA_BUSY_CYCLES') / (4 * wc):.3f}" if wc and "SQ_VALU_MFMA_BUSY_CYCLES" in m
                    else "-")
            rd = f"{2 * 1024 * f('FETCH_SIZE') / 1e6:.1f}" if "FETCH_SIZE" in m else "-"
            wr = f"{1024 * f('WRITE_SIZE') / 1e6:.1f}" if "WRITE_SIZE" in m else "-"
            print(f"| `{short(k)}` | {w:.0f} | {frac('SQ_ACTIVE_INST_ANY')} | {frac('SQ_WAIT_ANY')} | "
                  f"{frac('SQ_WAIT_INST_ANY')} | {f('SQ_INSTS_VALU') / w:.0f} | {f('SQ_INSTS_SALU') / w:.0f} | "
                  f"{f('SQ_INSTS_LDS') / w:.0f} | {conf} | {mfma} | {rd} | {wr} |")


if __name__ == "__main__":
    main()
