#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel (first 40 chars of name + template args).
usage: python3 tools/pmc_summary.py <counter_collection.csv> [...] [--filter substr]"""
import csv
import sys
from collections import defaultdict

args = sys.argv[1:]
flt_i = args.index("--filter") if "--filter" in args else -1
files = [a for i, a in enumerate(args) if not a.startswith("--") and i != flt_i + 1]
flt = ""
if "--filter" in sys.argv:
    flt = sys.argv[sys.argv.index("--filter") + 1]
agg = defaultdict(lambda: defaultdict(list))
meta = {}
for f in files:
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if flt and flt not in k:
            continue
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        meta[k] = (row["VGPR_Count"], row["SGPR_Count"], row["LDS_Block_Size"], row["Grid_Size"], row["Workgroup_Size"])
for k, cs in agg.items():
    v, s, l, g, w = meta[k]
    print(f"== {k[:120]}  vgpr={v} sgpr={s} lds={l} grid={g} wg={w}")
    for c in sorted(cs):
        vals = cs[c]
        print(f"   {c:28s} {sum(vals) / len(vals):16.1f}   (n={len(vals)})")
