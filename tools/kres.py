#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per kernel.
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python3 tools/kres.py [filter]"""
import re
import subprocess
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0]] = m.group(2)
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
except OSError:
    dem = names
for r, d in zip(rows, dem):
    if flt in d:
        print(f"{d[:110]:110s} v{r.get('VGPRs','?'):>4} s{r.get('TotalSGPRs','?'):>4} lds{r.get('LDS','?'):>6} "
              f"scr{r.get('ScratchSize','?'):>4} occ{r.get('Occupancy','?')}")
