#!/usr/bin/env python3
"""Per-kernel table of rocprofv3 --pmc counters (mean over dispatches), one column per
counter, from one or more pmc_counter_collection.csv files (tuning aid).
usage: pmc_table.py CSV [CSV ...] [--per-wave]"""
import csv
import sys
from collections import OrderedDict, defaultdict

files = [a for a in sys.argv[1:] if not a.startswith("--")]
per_wave = "--per-wave" in sys.argv
agg = OrderedDict()
for f in files:
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        agg.setdefault(k, defaultdict(list))[row["Counter_Name"]].append(float(row["Counter_Value"]))
cols = []
for cs in agg.values():
    for c in cs:
        if c not in cols:
            cols.append(c)
short = lambda c: c.replace("SQ_", "").replace("INST", "I").replace("ACTIVE", "ACT")[:13]
print(f"{'kernel':58s}" + "".join(f"{short(c):>14s}" for c in cols))
for k, cs in agg.items():
    waves = (sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"])) if per_wave and "SQ_WAVES" in cs else 1.0
    name = k.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0][-58:]
    print(f"{name:58s}" + "".join(
        f"{(sum(cs[c]) / len(cs[c]) / (waves if per_wave else 1.0)) if c in cs else float('nan'):14.4g}" for c in cols))
