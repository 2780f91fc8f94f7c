#!/usr/bin/env python3
"""Per-kernel HBM traffic of the C5 span workload from a FETCH_SIZE and a WRITE_SIZE
rocprofv3 --pmc pass (tools/gpu_round.sh pmc:c5_fetch:FETCH_SIZE:--workload,c5,...):
medians per dispatch, bytes = FETCH_SIZE x 2 (gfx950 wide-read correction,
MI355X_MICROARCH.md) and WRITE_SIZE as measured, both KiB.
  python3 tools/pmc_c5_traffic.py <fetch_dir> <write_dir> > c5_pmc_traffic.json"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def per_kernel(d, counter):
    v = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/pmc_counter_collection.csv")):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            v[name].append(float(r["Counter_Value"]))
    return v


f, w = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
S, K, B = 8, 256, 153_600
out = {"config": {"workload": "c5", "streams": S, "span": K, "block_complex": B},
       "note": ("per dispatch (one dispatch = one 8-stream span call per kernel launch); FETCH_SIZE and WRITE_SIZE "
                "medians in KiB from separate rocprofv3 --pmc passes; bytes = FETCH_SIZE x 2 (gfx950 wide-read "
                "correction, MI355X_MICROARCH.md) and WRITE_SIZE as measured"),
       "kernels": {}}
for k in sorted(set(f) | set(w)):
    fe, wr = statistics.median(f.get(k, [0.0])), statistics.median(w.get(k, [0.0]))
    e = {"dispatches": len(f.get(k, [])), "fetch_size_kib_median": fe, "write_size_kib_median": wr,
         "hbm_read_bytes": fe * 1024 * 2, "hbm_write_bytes": wr * 1024}
    if k.startswith("fe_mfma_demod_kernel"):          # u8 IQ in, f32 demod out
        ar, aw = S * K * B * 2, S * K * (B // 10) * 4
        e.update(algorithmic_read_bytes=ar, algorithmic_write_bytes=aw,
                 read_over_algorithmic=round(e["hbm_read_bytes"] / ar, 4),
                 write_over_algorithmic=round(e["hbm_write_bytes"] / aw, 4))
    out["kernels"][k] = e
print(json.dumps(out, indent=1))
