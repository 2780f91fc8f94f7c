#!/usr/bin/env python3
"""Per-config throughput of the block processors on one GPU (not the headline bench).

C3: MonoBlockProcessor at fmMonoBlock.py block sizes (51 200 complex, f32 IQ), host block in,
    audio out per call (the drop-in per-block path: H2D + kernels + D2H each block).
C4: StereoBlockProcessor, same blocks (+ pilot BPF, PLL, band BPF, mixer+LPF, combiner).
C5: RdsBlockProcessor at fm_radio.cpp blocks (153 600 complex, u8 IQ) to the RRC output,
    and StereoBlockProcessor on the same u8 blocks (one stream; configs[4] runs one per GPU).
Prints one JSON object: per config MS/s (complex input samples), ms per block, blocks timed.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import rtsdr  # noqa: E402


def timeit(proc, blocks, reps):
    for b in blocks[:2]:
        proc.process(b)
    t0 = time.perf_counter()
    for _ in range(reps):
        for b in blocks:
            proc.process(b)
    dt = time.perf_counter() - t0
    return dt, reps * len(blocks)


def main():
    out = {}
    B3 = 51_200
    iq = rtsdr.synth.fm_iq(B3 * 20, seed=0)
    blocks = [np.ascontiguousarray(iq[2 * k * B3:2 * (k + 1) * B3]) for k in range(20)]
    rf_b, au_b = rtsdr.design.mono_coeffs(101, 151)
    for name, proc in (("C3_mono_51200_f32", rtsdr.MonoBlockProcessor(B3, rf_b, au_b)),
                       ("C4_stereo_51200_f32", rtsdr.StereoBlockProcessor(B3, rf_b, au_b))):
        dt, nb = timeit(proc, blocks, 5)
        out[name] = {"MS_per_s": round(nb * B3 / dt / 1e6, 2), "ms_per_block": round(dt / nb * 1e3, 4),
                     "blocks": nb}
    B5 = 153_600
    u8 = rtsdr.synth.fm_iq(B5 * 12, seed=1, dtype=np.uint8)
    ublocks = [np.ascontiguousarray(u8[2 * k * B5:2 * (k + 1) * B5]) for k in range(12)]
    rf151, au151 = rtsdr.design.mono_coeffs(151, 151)
    for name, proc in (("C5_rds_153600_u8", rtsdr.RdsBlockProcessor(B5)),
                       ("C5_stereo_153600_u8", rtsdr.StereoBlockProcessor(B5, rf151, au151, iq_dtype=np.uint8))):
        dt, nb = timeit(proc, ublocks, 3)
        out[name] = {"MS_per_s": round(nb * B5 / dt / 1e6, 2), "ms_per_block": round(dt / nb * 1e3, 4),
                     "blocks": nb}
    out["note"] = ("per-block drop-in path: each call uploads one host IQ block, runs the block's kernels "
                   "on the context stream and downloads its outputs; real time is 2.4 MS/s")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
