#!/usr/bin/env python3
"""Per-kernel VALU / LDS utilisation of a c5 profile set (tuning aid).
usage: pmc_util.py DIR TAG   (DIR/prof_TAG/prof_kernel_trace.csv, DIR/pmc_TAG_{a,b}/...)
VALU util = SQ_ACTIVE_INST_VALU quad-cycles x 4 / (kernel time x 1024 SIMDs x 2.4 GHz);
LDS util = SQ_LDS_IDX_ACTIVE / (kernel time x 256 CUs x 2.4 GHz) (both vs the trace's mean
duration of that kernel, so at the peak clock: a lower bound when the clock runs lower)."""
import collections
import csv
import re
import sys


def short(k):
    k = k.replace("(anonymous namespace)::", "").removeprefix("void ")
    return re.sub(r"\(.*", "", k)


def load(p):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(p)):
        per[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Kernel_Name"]].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in per.items()}


d, tag = sys.argv[1], sys.argv[2]
a = load(f"{d}/pmc_{tag}_a/pmc_counter_collection.csv")
b = load(f"{d}/pmc_{tag}_b/pmc_counter_collection.csv")
dur = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/prof_{tag}/prof_kernel_trace.csv")):
    dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("| kernel | us (mean) | VALU util | LDS util | VALU insts / wave | waves |")
print("|---|---|---|---|---|---|")
for k in sorted(b, key=lambda k: -sum(dur.get(k, [0]))):
    if k not in dur or "rocclr" in k:
        continue
    us = sum(dur[k]) / len(dur[k])
    v = b[k].get("SQ_ACTIVE_INST_VALU", a[k].get("SQ_ACTIVE_INST_VALU", 0)) * 4 / (us * 2400 * 1024)   # (either pass)
    l = b[k].get("SQ_LDS_IDX_ACTIVE", 0) / (us * 2400 * 256)
    w = a[k].get("SQ_WAVES", 1)
    print(f"| `{short(k)}` | {us:.1f} | {v:.2f} | {l:.2f} | {a[k].get('SQ_INSTS_VALU', 0) / w:.0f} | {w:.0f} |")
