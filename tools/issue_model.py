#!/usr/bin/env python3
"""Issue-bound model of one kernel from its SQ counter passes: how many
cycles each SIMD must spend issuing the kernel's instruction stream, against its measured time
and the HBM floor of its algorithmic bytes.

usage: python3 tools/issue_model.py KERNEL_SUBSTR TIME_US ALG_BYTES CLOCK_GHZ DIR [DIR ...]
  DIR: rocprofv3 --pmc pass dirs holding pmc_counter_collection.csv (merged; means per dispatch)
Needs SQ_WAVES, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_INSTS_SALU, SQ_INSTS_LDS,
SQ_VALU_MFMA_BUSY_CYCLES, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY
(optional: SQ_INSTS_VALU_MFMA_MOPS_I8 / _F16, SQ_INSTS_SMEM, SQ_INSTS_BRANCH, SQ_INSTS_VMEM).

Model (MI355X_MICROARCH.md): a wave64 VALU instruction holds its SIMD's vector issue for
SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU quad-cycles (measured: ~1 = 4 cycles); an MFMA holds it for
half the matrix pipe's busy cycles (8 of the 16 of a 16x16xK step); scalar, LDS and memory
instructions issue from their own units beside the vector issue.  The vector-issue demand per
SIMD is the floor of the kernel's time at 100 % issue, whatever the occupancy hides."""
import csv
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def load(dirs, sub):
    acc = defaultdict(list)
    for d in dirs:
        path = os.path.join(d, "pmc_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            if sub in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    sub, t_us, alg, ghz, dirs = sys.argv[1], float(sys.argv[2]), float(sys.argv[3]), float(sys.argv[4]), sys.argv[5:]
    c = load(dirs, sub)
    waves = c["SQ_WAVES"]
    cyc = t_us * 1e-6 * ghz * 1e9                               # kernel cycles at CLOCK_GHZ
    valu_q = c["SQ_ACTIVE_INST_VALU"] / c["SQ_INSTS_VALU"]      # quad-cycles per VALU instruction
    valu_cyc = 4 * c["SQ_ACTIVE_INST_VALU"] / SIMDS             # per SIMD
    mfma_cyc = c["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS
    hold = 0.5 * mfma_cyc
    issue = valu_cyc + hold
    hbm_us = alg / 8e12 * 1e6
    wc = c["SQ_WAVE_CYCLES"]
    per = lambda k: c.get(k, float("nan")) / waves               # noqa: E731
    rows = [
        ("waves per dispatch", f"{waves:.0f} ({waves / SIMDS:.1f} per SIMD)"),
        ("VALU / SALU / LDS / SMEM / branch / VMEM instructions per wave",
         f"{per('SQ_INSTS_VALU'):.0f} / {per('SQ_INSTS_SALU'):.0f} / {per('SQ_INSTS_LDS'):.0f} / "
         f"{per('SQ_INSTS_SMEM'):.0f} / {per('SQ_INSTS_BRANCH'):.0f} / {per('SQ_INSTS_VMEM'):.0f}"),
        ("vector issue per VALU instruction", f"{valu_q:.2f} quad-cycles = {4 * valu_q:.1f} cycles"),
        ("matrix-pipe busy per SIMD", f"{mfma_cyc / 1e3:.1f} k cycles"
         + (f" ({c['SQ_INSTS_VALU_MFMA_MOPS_I8'] * 512 / 32768 / waves:.0f} int8 16x16x64 MFMAs per wave)"
            if "SQ_INSTS_VALU_MFMA_MOPS_I8" in c else "")),
        ("vector-issue demand per SIMD (VALU + half the MFMA busy)",
         f"{valu_cyc / 1e3:.1f} k + {hold / 1e3:.1f} k = {issue / 1e3:.1f} k cycles = {issue / ghz / 1e3:.1f} us at {ghz} GHz"),
        ("HBM floor of the algorithmic bytes (8 TB/s)", f"{hbm_us:.1f} us"),
        ("measured", f"{t_us:.1f} us = {cyc / 1e3:.1f} k cycles: vector issue busy {issue / cyc:.2f} of the kernel, "
                     f"HBM {hbm_us / t_us:.2f}"),
        ("wave time: issuing / parked on s_waitcnt / issue-stalled",
         f"{c['SQ_ACTIVE_INST_ANY'] / wc:.2f} / {c['SQ_WAIT_ANY'] / wc:.2f} / {c['SQ_WAIT_INST_ANY'] / wc:.2f}"),
        ("ceiling: max(issue demand, HBM floor)", f"{max(issue / ghz / 1e3, hbm_us):.1f} us "
                                                  f"(the kernel at {max(issue / ghz / 1e3, hbm_us) / t_us:.2f} of it)"),
    ]
    print(f"### issue model: `{sub}`\n")
    print("| quantity | value |\n|---|---|")
    for k, v in rows:
        print(f"| {k} | {v} |")


if __name__ == "__main__":
    main()
