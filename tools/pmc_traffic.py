#!/usr/bin/env python3
"""HBM traffic per launch of the bench's dominant kernel from rocprofv3 --pmc CSVs.

usage: python3 tools/pmc_traffic.py <tag> [--blocks 64 --taps 101] [--dir D]
Reads gpurun_out/pmc_<tag>_<path>_{fetch,write}/pmc_counter_collection.csv, or with --dir D
(relative to the repo) the closing set's D/pmc_<path>_{fetch,write}/ -- one counter per
rocprofv3 pass, tools/gpu_round.sh pmc:<path>_fetch:FETCH_SIZE:<bench args> and
pmc:<path>_write:WRITE_SIZE:<bench args>, paths fused / u8 / split -- and writes
profiles/fe_pmc_traffic.json.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE is in KiB and on gfx950 counts half
the bytes of a wide (16 B/lane) coalesced streaming read -> x2; WRITE_SIZE (KiB) is
exact for 16-B-per-lane streaming stores.  Our stores are 8-B (float2) per lane; the
write figure is reported as measured (uncalibrated for that width).
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"split": "fe_ring_kernel<101, false", "fused": "fe_ring_kernel<101, true", "u8": "fe_mfma_mono_kernel"}


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1]
    blocks = int(sys.argv[sys.argv.index("--blocks") + 1]) if "--blocks" in sys.argv else 128
    taps = int(sys.argv[sys.argv.index("--taps") + 1]) if "--taps" in sys.argv else 101
    n = blocks * 1_024_000
    d = sys.argv[sys.argv.index("--dir") + 1] if "--dir" in sys.argv else None
    entries = []
    for path, key in KERNELS.items():
        pre = os.path.join(ROOT, d, f"pmc_{path}") if d else os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_{path}")
        fdir = os.path.join(pre + "_fetch", "pmc_counter_collection.csv")
        wdir = os.path.join(pre + "_write", "pmc_counter_collection.csv")
        if not (os.path.exists(fdir) and os.path.exists(wdir)):
            continue
        fetch = [v for k, v in per_kernel(fdir, "FETCH_SIZE").items() if key in k]
        write = [v for k, v in per_kernel(wdir, "WRITE_SIZE").items() if key in k]
        if not fetch or not write:
            continue
        f_kib = sorted(fetch[0])[len(fetch[0]) // 2]
        w_kib = sorted(write[0])[len(write[0]) // 2]
        rd = 2.0 * f_kib * 1024
        wr = w_kib * 1024
        alg_rd = n * (2 if path == "u8" else 8)
        alg_wr = n // 10 * 4 if path == "split" else n // 50 * 4
        entries.append({"path": "u8_mfma" if path == "u8" else path, "kernel": key, "taps": taps, "n_complex": n,
                        "fetch_size_kib_median": f_kib, "write_size_kib_median": w_kib,
                        "hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                        "algorithmic_read_bytes": alg_rd, "algorithmic_write_bytes": alg_wr,
                        "read_over_algorithmic": round(rd / alg_rd, 4),
                        "samples": {"fetch": len(fetch[0]), "write": len(write[0])},
                        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), tag {tag}; "
                                  f"FETCH_SIZE x2 (gfx950 wide-read correction)"})
    out = os.path.join(ROOT, "profiles", "fe_pmc_traffic.json")
    if os.path.exists(out):                 # paths this run did not measure keep their entries
        with open(out) as f:
            have = {e["path"] for e in entries}
            entries = [e for e in json.load(f)["entries"] if e["path"] not in have] + entries
    with open(out, "w") as f:
        json.dump({"entries": entries}, f, indent=1)
    print(json.dumps(entries, indent=1))


if __name__ == "__main__":
    main()
