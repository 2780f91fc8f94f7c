"""Per-block timeline from a rocprofv3 --kernel-trace --memory-copy-trace CSV pair (tool, not
product): prints the last blocks' kernels / copies with durations and the gaps between them.
  python tools/timeline.py <dir> <prefix> [n_events]"""
import csv
import sys

d, pre = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")[:60])
      for r in csv.DictReader(open(f"{d}/{pre}_kernel_trace.csv"))]
try:
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"][12:])
           for r in csv.DictReader(open(f"{d}/{pre}_memory_copy_trace.csv"))]
except FileNotFoundError:
    pass
ev.sort()
base, prev = ev[-n][0], None
for s, e, name in ev[-n:]:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - base) / 1e3:9.2f}  dur {(e - s) / 1e3:7.2f}  gap {gap:6.2f}  {name}")
    prev = e
