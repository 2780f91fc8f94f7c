#!/usr/bin/env python3
"""Per-STAGE hardware counts of the C5 span workload (bench.py --workload c5), for bench.py's
`c5.stage_roofline`: each receiver stage's HBM bytes, executed matrix-core operations and f64
VALU instructions per span call, from rocprofv3 --pmc passes of the same command
(tools/gpu_round.sh pmc:<name>:<counters>:--workload,c5,...).

usage: python3 tools/pmc_c5.py OUT.json DIR [DIR ...]
  DIR: a pass's output dir (holding pmc_counter_collection.csv); the passes are merged.
Counters used when present: FETCH_SIZE (x 2: the gfx950 wide-read correction,
MI355X_MICROARCH.md), WRITE_SIZE, SQ_INSTS_VALU_MFMA_MOPS_F16 / _I8 (x 512 = executed
matrix-core ops), SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64, SQ_INSTS_VALU, SQ_WAVES,
SQ_ACTIVE_INST_VALU (quad-cycles of vector issue), SQ_VALU_MFMA_BUSY_CYCLES (matrix-pipe cycles).

The stages are the receiver's timing stages (csrc/rx.hip, sdr_rx_stage_ms):
  fe                fe_mfma_demod_kernel<151>
  filters_of_demod  rx_mma_kernel<151, 3> (pilot, stereo, RDS-extract BPFs) + rx_decmm_kernel<false, false> (audio LPF)
  rds_square        the first rx_mma_kernel<151, 1> dispatch of a span call (x^2 + BPF)
  pll               pll_spec_kernel<512, true> + pll_long_fix_kernel
  mix_lpf           rx_decmm_kernel<true, true> (stereo mixer + LPF + L/R, its NCO formed from the PLL's compact phase rows)
  resample          rx_cresmm_kernel<true> (RDS I/Q mixers + LPF + x19/80 resampler, composite; compact rows)
(round-6 closing passes before the compact rows: rx_decmm_kernel<false> / <true>, rx_cresmm_kernel --
the names are matched by ALIASES)
  rrc               the second rx_mma_kernel<151, 1> dispatch of a span call (RRC I/Q)
Values are medians over the dispatches of a kernel (its span calls), summed over a stage's kernels."""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

STAGES = {
    "fe": ["fe_mfma_demod_kernel<151>"],
    "filters_of_demod": ["rx_mma_kernel<151, 3>", "rx_decmm_kernel<false, false>"],
    "rds_square": ["rx_mma_kernel<151, 1>#0"],
    "pll": ["pll_spec_kernel<512, true>", "pll_long_fix_kernel"],
    "mix_lpf": ["rx_decmm_kernel<true, true>"],
    "resample": ["rx_cresmm_kernel<true>"],
    "rrc": ["rx_mma_kernel<151, 1>#1"],
}
ALIASES = {"rx_decmm_kernel<false>": "rx_decmm_kernel<false, false>", "rx_decmm_kernel<true>": "rx_decmm_kernel<true, true>",
           "rx_cresmm_kernel": "rx_cresmm_kernel<true>"}
TWO_PER_CALL = "rx_mma_kernel<151, 1>"      # rds_square, then rrc, in every span call's launch order


def short(k):
    return k.replace("(anonymous namespace)::", "").removeprefix("void ").split("(")[0]


def load(d):
    path = os.path.join(d, "pmc_counter_collection.csv")
    if not os.path.exists(path):
        for root, _, files in os.walk(d):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    path = os.path.join(root, f)
    rows = defaultdict(dict)             # dispatch id -> {"name": ..., counter: value}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            e = rows[int(r["Dispatch_Id"])]
            e["name"] = ALIASES.get(short(r["Kernel_Name"]), short(r["Kernel_Name"]))
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return rows


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    per = defaultdict(lambda: defaultdict(list))   # kernel (with #i for the shared one) -> counter -> values
    for d in dirs:
        rows = load(d)
        nth = 0
        for did in sorted(rows):
            e = rows[did]
            name = e["name"]
            if name == TWO_PER_CALL:
                name = f"{name}#{nth % 2}"
                nth += 1
            for c, v in e.items():
                if c != "name":
                    per[name][c].append(v)
    kernels = {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in per.items()}
    stages = {}
    for st, ks in STAGES.items():
        acc = defaultdict(float)
        for k in ks:
            for c, v in kernels.get(k, {}).items():
                acc[c] += v
        s = {"kernels": ks}
        if "FETCH_SIZE" in acc:
            s["hbm_read_bytes"] = 2 * 1024 * acc["FETCH_SIZE"]
        if "WRITE_SIZE" in acc:
            s["hbm_write_bytes"] = 1024 * acc["WRITE_SIZE"]
        for c in ("SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_INSTS_VALU_MFMA_MOPS_I8"):
            if c in acc:
                s[c.replace("SQ_INSTS_VALU_MFMA_MOPS_", "mfma_ops_").lower()] = 512 * acc[c]
        f64 = [acc[c] for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                "SQ_INSTS_VALU_TRANS_F64") if c in acc]
        if f64:
            s["f64_wave_instr"] = sum(f64)
        for c, key in (("SQ_INSTS_VALU", "valu_wave_instr"), ("SQ_WAVES", "waves"),
                       ("SQ_ACTIVE_INST_VALU", "valu_active_quad_cycles"),
                       ("SQ_VALU_MFMA_BUSY_CYCLES", "mfma_busy_cycles")):
            if c in acc:
                s[key] = acc[c]
        stages[st] = s
    res = {"config": {"workload": "c5", "streams": 8, "span": 256, "block_complex": 153_600},
           "note": ("per span call (medians over a kernel's dispatches, summed over the stage's kernels): HBM bytes "
                    "(FETCH_SIZE x 2, WRITE_SIZE), executed matrix-core ops (MOPS x 512), f64 VALU wave-instructions, "
                    "vector-issue quad-cycles (SQ_ACTIVE_INST_VALU), matrix-pipe busy cycles; tools/pmc_c5.py"),
           "stages": stages, "kernels": kernels, "sources": [os.path.relpath(d) for d in dirs]}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(stages, indent=1))


if __name__ == "__main__":
    main()
