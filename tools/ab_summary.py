#!/usr/bin/env python3
"""Summarise tools/ab_bench.sh output: per variant, the median over reps of the line's value,
ms/step, the dominant kernel's launch time and frac, and (receiver workloads) the stage times.
usage: ab_summary.py <dir> [<dir> ...]"""
import glob
import json
import os
import statistics
import sys

for d in sys.argv[1:]:
    runs = {}
    for f in sorted(glob.glob(os.path.join(d, "ab_*_*.json"))):
        name = os.path.basename(f)[3:-5].rsplit("_", 1)[0]
        try:
            line = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        runs.setdefault(name, []).append(line)
    print(d)
    for name, ls in runs.items():
        med = lambda xs: statistics.median(xs) if xs else None
        v = med([l["value"] for l in ls])
        ms = med([l["ms_per_step"] for l in ls])
        r = [l.get("roofline", {}) for l in ls]
        k = med([x["avg_launch_ms"] for x in r if x.get("avg_launch_ms")])
        fr = med([x["frac"] for x in r if x.get("frac") is not None])
        st = {}
        for l in ls:
            for key, val in (l.get("stage_ms") or {}).items():
                st.setdefault(key, []).append(val)
        sts = " ".join(f"{key}={med(v_):.4f}" for key, v_ in st.items())
        print(f"  {name:>14} n={len(ls)} value={v:.1f} ms/step={ms} kernel_ms={k} frac={fr} {sts}")
