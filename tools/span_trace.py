#!/usr/bin/env python3
"""The last kernels of a rocprofv3 kernel trace as a small CSV (tool, not product):
kernel, queue, start / end / duration in us from the first of them, grid and workgroup size.
  python3 tools/span_trace.py <prof_dir>/prof_kernel_trace.csv [n] > trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ev = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))[-n:]
t0 = int(ev[0]["Start_Timestamp"])
print("kernel,queue,start_us,end_us,dur_us,grid_x,wg_x")
for r in ev:
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f'"{name}",{r["Queue_Id"]},{s / 1e3:.3f},{e / 1e3:.3f},{(e - s) / 1e3:.3f},{r["Grid_Size_X"]},{r["Workgroup_Size_X"]}')
