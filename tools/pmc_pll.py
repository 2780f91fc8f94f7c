#!/usr/bin/env python3
"""Per-kernel SQ instruction counts of the PLL kernels, for bench.py's `pll_roofline`.

usage: python3 tools/pmc_pll.py OUT.json CONFIG_JSON DIR [DIR ...]
  DIR: rocprofv3 --pmc output dirs (tools/gpu_round.sh pmc:<name>:<counters>:<bench args>),
       each holding pmc_counter_collection.csv; counters from several passes are merged.
  CONFIG_JSON: the bench configuration the passes ran, e.g. '{"streams": 8, "span": 256}'
Writes {"config": ..., "kernels": {name: {counter: mean per dispatch}}, "dispatches": {...}}.
SQ_INSTS_* count wave-instructions summed over a dispatch's waves."""
import csv
import json
import os
import sys
from collections import defaultdict


def short(k):
    return k.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0]


def main():
    out, cfg, dirs = sys.argv[1], json.loads(sys.argv[2]), sys.argv[3:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        path = os.path.join(d, "pmc_counter_collection.csv")
        if not os.path.exists(path):
            for root, _, files in os.walk(d):
                for f in files:
                    if f.endswith("counter_collection.csv"):
                        path = os.path.join(root, f)
        with open(path) as fh:
            for row in csv.DictReader(fh):
                name = short(row["Kernel_Name"])
                if "pll" not in name and "nco" not in name:
                    continue
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    kernels = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    disp = {k: max(len(v) for v in cs.values()) for k, cs in acc.items()}
    with open(out, "w") as fh:
        json.dump({"config": cfg, "kernels": kernels, "dispatches": disp, "sources": dirs}, fh, indent=1)
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
