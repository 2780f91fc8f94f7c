#!/usr/bin/env python3
"""Benchmark of the FM-SDR hot path on MI355X (BASELINE.json metric).

One step = one pass of RF front end (101-tap IQ LPF, decimate by 10, atan2 demod;
configs[1]) + mono (151-tap audio LPF, decimate by 5; configs[2]) over a batch of
`--blocks` (default 128) x 1 024 000-complex-sample blocks of one synthetic 2.4 MS/s stream, input
resident in HBM (block boundaries are carried-state continuations, so the batch is
one continuous stream; SURVEY §5 "long-context").  Kernel: libsdr.so's fused
FE + mono kernel (sdr_fe_mono_dev: the demodulated signal never leaves the CU);
`--path split` runs the FE kernel + FIR kernel pair instead.  Launched through the
C-ABI (no torch in the data path).

Multi-GPU (`torchrun --nproc-per-node N bench.py --gpus N`): one process per GPU,
each rank processes its own independent stream (seed = rank): weak scaling, no
data-path collective.  torch.distributed (gloo, CPU) only provides the barrier and
the max-over-ranks of the timed region.

Other workloads (`--workload`, one JSON line each; BASELINE.json configs):
  c5  configs[4]: `--streams` (default 8) independent u8 streams per GPU, 153 600-sample
      blocks (src/fm_radio.cpp:23), mono + stereo + RDS to the RRC output through the
      multi-stream receiver (sdr_rx), inputs resident in HBM, one step = one block of every
      stream (>= 256 blocks per stream by default); per-stage GPU times from HIP events.
  c3 / c4  configs[2] / [3]: the per-block drop-in path at fmMonoBlock.py's 51 200-sample
      blocks, host buffers in and out (PCIe-inclusive by nature), one stream: mono (c3) or
      mono + stereo (c4).  Blocks are submitted as a live receiver feeds them (sdr_rx_submit:
      block k runs while block k-1's outputs are delivered; the reference's rf / audio
      thread overlap); the synchronous one-block call (sdr_rx_run) is timed beside it
      ("sync", "block_latency_ms").  --no-pipeline: sdr_rx_run only.
  CPU baselines for these: the reference's own C++ receiver (src/filter.cpp, helper.cpp,
  rf_module.cpp compiled from its sources, oracle/ref_driver.cpp ref_rx_streams).

Prints ONE JSON line (rank 0).  `value` = complex IQ samples processed by all ranks
per second (MS/s); `roofline` is for the step's dominant kernel (HIP events on the libsdr stream);
`cpu_baseline` = the C restatement of the Python model (oracle/fm_oracle.c) on the
host cores (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "IQ MSamples/s through RF front-end+mono path; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
BLOCK = 1_024_000              # complex samples per block (SURVEY §7 hard part 7)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["mono", "c3", "c4", "c5", "live"], default="mono",
                    help="mono: configs[1]+[2] batched (the headline); c3/c4: per-block drop-in path; "
                         "c5: multi-stream mono+stereo+RDS; live: fm_radio_gpu end to end (u8 stdin -> int16 "
                         "stdout) beside the reference's own fm_radio")
    ap.add_argument("--streams", type=int, default=8, help="c5: independent streams per GPU")
    ap.add_argument("--span", type=int, default=256,
                    help="c5: 153 600-sample blocks of every stream processed per receiver call (device-resident "
                         "spans, time-parallel: FE and filters as one pass, PLLs as long calls); 1 = the per-block "
                         "receiver, one block of every stream per call")
    ap.add_argument("--no-extras", action="store_true",
                    help="mono: skip the c5 (8 and 1 streams) and u8 blocks appended to the headline line")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 50; c5: 256 blocks)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--settle-ms", type=float, default=250.0,
                    help="untimed warm-up continues past --warmup steps until this much GPU time has "
                         "run, so the clocks have ramped before the timed region (DESIGN.md §5)")
    ap.add_argument("--blocks", type=int, default=128,
                    help="1 024 000-sample blocks per step (>= 64, SURVEY §8d; the launch has ~6 us of fixed cost, "
                         "DESIGN.md §5)")
    ap.add_argument("--taps", type=int, default=101)
    ap.add_argument("--audio-taps", type=int, default=151)
    ap.add_argument("--iq", choices=["f32", "u8"], default="f32")
    ap.add_argument("--path", choices=["fused", "split"], default="fused",
                    help="fused: one fe_mono_kernel (demod stays on chip); split: FE kernel + FIR kernel")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--depth", type=int, default=2,
                    help="c3 / c4: sdr_rx_submit depth (blocks in flight; sdr_rx_set_depth)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="c3/c4/c5: one block at a time (c3/c4: sdr_rx_run; c5: one stream of launches)")
    ap.add_argument("--split-stream", action="store_true",
                    help="mono: ONE stream of --blocks blocks split over the ranks, each range with a read-only "
                         "halo (SURVEY §8e; strong scaling) instead of one stream per rank")
    ap.add_argument("--live-repeat", type=int, default=8,
                    help="live: passes of the --span-block stream in the long run (the short run is one pass)")
    ap.add_argument("--allow-wrap", action="store_true",
                    help="more ranks than visible GPUs: wrap them onto the devices (one-GPU rehearsals only; the "
                         "line's n_gpus then counts distinct devices)")
    ap.add_argument("--cpu-samples", type=int, default=4_096_000, help="complex samples per CPU stream")
    ap.add_argument("--cpu-seconds", type=float, default=1.5, help="wall time per CPU leg")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="mono with extras: the full record (every field of every configuration) is written here; "
                         "the printed line is its compact form ('' prints the full record instead)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "fe_pmc_traffic.json"),
                    help="PMC-derived HBM bytes per FE launch (written by tools/pmc_traffic.py)")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = ((256 if a.span == 1 else 10) if a.workload == "c5" else
                   (200 if a.workload in ("c3", "c4") else 50))
    return a


def dist_setup(args):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints its connection messages on fd 1: keep stdout for the one JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=ws)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    return ws, rank, local


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(ws, value: float) -> float:
    if ws == 1:
        return value
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(args, rf_b, au_b):
    """Oracle C port (f64, model semantics) + reference C++ FE, one stream per thread."""
    import subprocess
    lib_path = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    lib = ctypes.CDLL(lib_path)
    P = np.ctypeslib.ndpointer
    lib.orc_fe_mono_streams.argtypes = [P(np.float32), ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                        P(np.float64), ctypes.c_int, P(np.float64), ctypes.c_int,
                                        P(np.float64), ctypes.c_int64, ctypes.c_int]
    threads = cpu_threads()
    visible, model = cpu_cores()
    import rtsdr
    n = args.cpu_samples
    # one synthetic stream shared read-only by all threads (bounded memory); each thread
    # writes its own output; repeated until ~args.cpu_seconds of wall time (~16x that of CPU work)
    iq = rtsdr.synth.fm_iq(n, seed=100)
    A = ((n + 9) // 10 + 4) // 5
    out = np.empty(A * threads)

    def run_port():
        lib.orc_fe_mono_streams(iq, n, 0, threads, np.ascontiguousarray(rf_b), len(rf_b),
                                np.ascontiguousarray(au_b), len(au_b), out, A, threads)

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter() - t0
        reps = max(1, int(np.ceil(args.cpu_seconds / max(t1, 1e-6))))
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return reps, time.perf_counter() - t0

    reps, dt = timed(run_port)
    res = {"value": round(n * threads * reps / dt / 1e6, 3), "unit": "MS/s", "cores": threads, "kind": "port",
           "cpu": model, "cores_visible": visible,
           "sample": f"{threads} threads x {reps} x {n} complex samples (one stream each), "
                     f"FE({len(rf_b)} taps)+mono({len(au_b)} taps), f64 C restatement of the Python model "
                     f"(oracle/fm_oracle.c, -O3 -march=x86-64-v3, OpenMP), {dt:.2f} s wall"}
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_fe.so")
    if os.path.exists(ref):
        rl = ctypes.CDLL(ref)
        rl.ref_fe_streams.argtypes = [P(np.float32), ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int64,
                                      P(np.float32), ctypes.c_int, ctypes.c_int, P(np.float32), ctypes.c_int64,
                                      ctypes.c_int]
        blk = 153_600
        nn = (n // blk) * blk
        dm = np.empty((nn // 10) * threads, dtype=np.float32)
        h32 = np.ascontiguousarray(rf_b, dtype=np.float32)

        def run_ref():
            rl.ref_fe_streams(iq, nn, 0, threads, blk, h32, len(rf_b), 10, dm, nn // 10, threads)

        reps, dt = timed(run_ref)
        res["reference_cpp_fe"] = {"value": round(nn * threads * reps / dt / 1e6, 3), "unit": "MS/s",
                                   "cores": threads, "kind": "reference",
                                   "sample": f"{threads} threads x {reps} x {nn} complex, src/filter.cpp "
                                             f"convolveWithDecimIQ + src/rf_module.cpp fmDemodArctan (FE only, "
                                             f"f32, reference -O3 flags), {dt:.2f} s wall; {ref_provenance()}"}
    else:
        res["reference_cpp_fe"] = {"value": None, "kind": "reference",
                                   "sample": "not run: oracle/_ref/libref_fe.so absent (built only where "
                                             "/root/reference exists; make -C oracle ref)"}
    return res


def ref_provenance():
    """Which reference sources oracle/_ref was compiled from (sha256, oracle/Makefile)."""
    try:
        with open(os.path.join(ROOT, "oracle", "_ref", "sources.sha256")) as f:
            got = f.read()
        with open(os.path.join(ROOT, "oracle", "ref_sources.sha256")) as f:
            want = f.read()
        return "sources match oracle/ref_sources.sha256" if got == want else "sources DIFFER from oracle/ref_sources.sha256"
    except OSError:
        return "source hashes unavailable"


def cpu_threads():
    """Worker threads for the CPU legs: the lease's CPU share.  OMP_NUM_THREADS when the
    environment sets it (the GPU box sets it to its per-GPU share), else every core this
    process may run on."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env if env > 0 else cpu_cores()[0]


def copy_bandwidth(lib, handle, nbytes: int = 2 << 30, reps: int = 10, read_only: bool = False):
    """the achieved fraction beside a measured stream kernel on the same box --
    libsdr's 16-B-per-lane nontemporal copy (sdr_copy_bandwidth, GB/s counting read + write) or
    read-only stream (sdr_read_bandwidth), best of `reps`.  (torch's own copy kernel cannot be
    used here: torch bundles its own HIP runtime, which does not initialise in a process that
    already runs libsdr's.)"""
    g = ctypes.c_double()
    fn = lib.sdr_read_bandwidth if read_only else lib.sdr_copy_bandwidth
    rc = fn(handle, nbytes, reps, ctypes.byref(g))
    if rc != 0:
        print(f"bench: stream bandwidth not measured: {lib.sdr_last_error().decode()}", file=sys.stderr)
        return None
    return round(g.value, 1)


def load_traffic(path, taps, blocks, kpath):
    """HBM bytes per launch of the dominant kernel, from tools/pmc_traffic.py's PMC summary."""
    try:
        with open(path) as f:
            t = json.load(f)
        for e in t.get("entries", []):
            if e.get("taps") == taps and e.get("n_complex") == blocks * BLOCK and e.get("path") == kpath:
                return e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def split_range(n_total: int, ws: int, rank: int, halo: int, step: int = 50):
    """--split-stream: rank r's range [s0, s1) of ONE stream of n_total complex
    samples (boundaries on whole audio samples, `step` = rf_decim x audio_decim IQ samples)
    and the start w0 = s0 - halo of the read-only halo it reads before it.  Returns
    (w0, s0, s1); its audio outputs are those of IQ positions [s0, s1)."""
    s0 = (rank * n_total // ws) // step * step
    s1 = n_total if rank == ws - 1 else ((rank + 1) * n_total // ws) // step * step
    return max(0, s0 - halo), s0, s1


def device_for(local: int, allow_wrap: bool = False, count: int | None = None) -> int:
    """GPU of this rank: LOCAL_RANK (one process per GPU).  More ranks than visible devices is
    refused (a line must not claim N GPUs that did not run) unless --allow-wrap, which wraps
    the ranks onto the devices for a multi-process rehearsal on a one-GPU box."""
    if count is None:
        import rtsdr
        count = rtsdr.device_count()
    if count <= 0:
        raise SystemExit("bench: no GPU visible (sdr_device_count = 0)")
    if local >= count and not allow_wrap:
        raise SystemExit(f"bench: LOCAL_RANK {local} but only {count} device(s) visible; refusing to wrap ranks "
                         "onto shared devices (--allow-wrap for a one-GPU rehearsal)")
    return local % count


def device_map(ws: int, rank: int, mine: dict) -> list:
    """Every rank's device (index and PCI bus id), gathered over gloo (rank order)."""
    mine = dict(mine, rank=rank)
    if ws == 1:
        return [mine]
    import torch.distributed as dist
    out = [None] * ws
    dist.all_gather_object(out, mine)
    return out


def check_devices(dmap: list, allow_wrap: bool) -> int:
    """Distinct physical devices among the ranks (by PCI bus id); refuses a run whose ranks
    share a device unless allow_wrap."""
    distinct = len({d["pci_bus_id"] for d in dmap})
    if distinct < len(dmap) and not allow_wrap:
        raise SystemExit(f"bench: {len(dmap)} ranks ran on {distinct} distinct device(s) "
                         f"({[d['pci_bus_id'] for d in dmap]}); refusing (--allow-wrap for a rehearsal)")
    return distinct


def main():
    args = parse()
    ws, rank, local = dist_setup(args)
    local = device_for(local, args.allow_wrap)
    os.environ["SDR_DEVICE"] = str(local)
    import rtsdr
    dmap = device_map(ws, rank, rtsdr.device_info(local))
    args.devices = {"distinct": check_devices(dmap, args.allow_wrap), "ranks": ws,
                    "map": [{"rank": d["rank"], "device": d["device"], "pci_bus_id": d["pci_bus_id"]} for d in dmap]}
    if args.workload == "live":
        return run_live(args, ws, rank, local)
    if args.workload == "c5" and args.span > 1:
        return run_c5_span(args, ws, rank, local)
    if args.workload != "mono":
        return run_rx(args, ws, rank, local)
    import rtsdr
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")

    ctx = _lib.Context(local)
    lib, h = ctx.lib, ctx.handle
    rf_b, au_b = rtsdr.design.mono_coeffs(args.taps, args.audio_taps)
    n_total = args.blocks * BLOCK
    n = n_total
    dt = np.uint8 if args.iq == "u8" else np.float32
    if args.split_stream:
        # rank r: IQ [s0, s1) of the one stream plus the halo before s0 (no exchange)
        w0, s0, s1 = split_range(n_total, ws, rank, rtsdr.split_halo(len(rf_b), len(au_b)))
        iq = rtsdr.synth.fm_iq(n_total, seed=0, dtype=dt)[2 * w0:2 * s1].copy()
        n = s1 - w0
    else:
        iq = rtsdr.synth.fm_iq(n, seed=rank, dtype=dt)
    M = (n + 9) // 10
    A = (M + 4) // 5
    dtype_code = _lib.SDR_IQ_U8 if args.iq == "u8" else _lib.SDR_IQ_F32
    d_iq = _lib.DeviceBuffer.from_array(ctx, iq)
    del iq
    d_dm = _lib.DeviceBuffer(ctx, 4 * M)
    d_au = _lib.DeviceBuffer(ctx, 4 * A)
    rfp, aup = _lib.f64p(rf_b), _lib.f64p(au_b)
    T, TA = len(rf_b), len(au_b)

    def fused():
        _lib.check(lib.sdr_fe_mono_dev(h, d_iq.ptr, dtype_code, n, n, 1, rfp, T, 10, aup, TA, 5, d_au.ptr, A),
                   "fe_mono")

    def fe():
        _lib.check(lib.sdr_rf_frontend_dev(h, d_iq.ptr, dtype_code, n, n, 0, 1, rfp, T, 10, None, None, 0, None,
                                           None, None, d_dm.ptr, M, None, None), "fe")

    def mono():
        _lib.check(lib.sdr_fir_dev(h, d_dm.ptr, None, 1.0, 0, M, M, 0, 1, aup, TA, 5, None, 0, None, d_au.ptr, A),
                   "mono")

    # fused: fe_ring_kernel for f32 IQ, fe_mfma_mono_kernel (RF FIR on the int8 matrix cores) for u8
    stages = [fused] if args.path == "fused" else [fe, mono]
    tm = _lib.Timer(ctx)
    # fused: one kernel per step -> one event pair around the whole timed region (per-step
    # events would add ~10 us of event processing between launches); split: events
    # between the two kernels of every step to separate them
    per_step = len(stages) > 1
    ev = [[tm.event() for _ in range(len(stages) + 1)] for _ in range(args.steps if per_step else 1)]
    for _ in range(args.warmup):
        for f in stages:
            f()
    ctx.synchronize()
    # clock ramp: the GPU reaches its sustained clocks only after tens of ms of load; a
    # 10-step warm-up is ~1 ms (measured: 121 us per launch at 50 cold steps, 97-104 us settled)
    settle_steps = 0
    t_set = time.perf_counter()
    while (time.perf_counter() - t_set) * 1e3 < args.settle_ms:
        for _ in range(50):
            for f in stages:
                f()
        settle_steps += 50
        ctx.synchronize()
    barrier(ws)
    ctx.synchronize()
    t0 = time.perf_counter()
    if per_step:
        for e in ev:
            tm.record(e[0])
            for k, f in enumerate(stages):
                f()
                tm.record(e[k + 1])
    else:
        tm.record(ev[0][0])
        for _ in range(args.steps):
            stages[0]()
        tm.record(ev[0][1])
    t_enq = time.perf_counter() - t0                 # host enqueue time (async launches)
    ctx.synchronize()
    barrier(ws)
    elapsed = max_over_ranks(ws, time.perf_counter() - t0)
    if per_step:
        stage_ms = [float(np.mean([tm.elapsed_ms(e[k], e[k + 1]) for e in ev])) for k in range(len(stages))]
    else:
        stage_ms = [tm.elapsed_ms(ev[0][0], ev[0][1]) / args.steps]
    k_avg = stage_ms[0]                              # the dominant (first) kernel of the step
    bpc = 2 if args.iq == "u8" else 8
    if args.path == "fused" and lib.sdr_fe_mono_fused(T, 10, TA, 5):
        # compulsory HBM bytes of the fused kernel: IQ in + audio out
        k_bytes = n * bpc + A * 4
        # u8: the int8-MFMA kernel takes 16-B aligned stream bases (every stride here is)
        kname = ("fe_mfma_mono_kernel (RF FIR on v_mfma_i32_16x16x64_i8)" if args.iq == "u8"
                 else f"fe_ring_kernel<{args.taps},fused>") + \
            f" (sdr_fe_mono_dev: FE {args.taps} taps + audio {args.audio_taps} taps)"
        kernels = {"fe_mono": round(k_avg, 5)}
    elif args.path == "fused":
        # sdr_fe_mono_dev runs its two-kernel path here (sdr_fe_mono_fused == 0): the timed
        # launch pair moves the demod through HBM too
        k_bytes = n * bpc + 2 * M * 4 + A * 4
        kname = f"sdr_fe_mono_dev two-kernel path (FE {args.taps} taps -> demod in HBM -> audio {args.audio_taps} taps)"
        kernels = {"fe_mono_pair": round(k_avg, 5)}
    else:
        k_bytes = n * bpc + M * 4                    # IQ in + demod out
        kname = (f"fe_slot_kernel<{args.taps},u8>" if args.iq == "u8" else f"fe_ring_kernel<{args.taps}>") + \
            " (sdr_rf_frontend_dev)"
        mono_bytes = M * 4 + A * 4
        kernels = {"fe": round(k_avg, 5), "mono": round(stage_ms[1], 5),
                   "mono_gbs": round(mono_bytes / (stage_ms[1] * 1e-3) / 1e9, 1)}
    achieved = k_bytes / (k_avg * 1e-3) / 1e9
    traffic = load_traffic(args.traffic, args.taps, args.blocks, args.path if args.iq == "f32" else "u8_mfma")

    result = None
    if rank == 0:
        total = n_total * args.steps * (1 if args.split_stream else ws)
        result = {
            "metric": METRIC,
            "value": round(total / elapsed / 1e6, 1),
            "unit": "MS/s",
            "n_gpus": args.devices["distinct"],
            "devices": args.devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.split_stream else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic FM IQ ({'one stream split over the ranks with halos' if args.split_stream else 'seed=rank'})"
                    f", interleaved {args.iq}, device-resident",
            "config": {"workload": f"RF front end ({args.taps}-tap LPF, decim 10, atan2 demod) + mono "
                                   f"({args.audio_taps}-tap LPF, decim 5): configs[1]+[2], one stream per GPU",
                       "block_complex": BLOCK, "blocks_per_step": args.blocks, "complex_per_step": n_total,
                       "taps": args.taps,
                       "iq": args.iq, "path": args.path,
                       "parallelism": f"one stream in {ws} ranges + halo" if args.split_stream else
                       f"independent streams x{ws}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": kname, "algorithmic_bytes_per_launch": k_bytes,
                         "avg_launch_ms": round(k_avg, 5)},
            "kernels_ms": kernels,
            "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 4),
            "settle": {"untimed_steps": settle_steps, "min_ms": args.settle_ms},
        }
    if rank == 0:
        # the measured ceilings beside the kernel: a copy (read + write) and a read-only stream
        # (the FE reads 8 B per complex sample and writes 0.04 B).  frac_of_copy_kernel: against
        # the copy (rounds 1-2's field, comparable across rounds); frac_of_stream_ceiling:
        # against the higher of the two (the practical ceiling of a read-mostly kernel)
        cbw = copy_bandwidth(lib, h)
        rbw = copy_bandwidth(lib, h, read_only=True)
        ceil = max([v for v in (cbw, rbw) if v] or [0.0])
        result["roofline"]["copy_kernel_gbs"] = cbw
        result["roofline"]["read_stream_gbs"] = rbw
        result["roofline"]["frac_of_copy_kernel"] = round(achieved / cbw, 4) if cbw else None
        result["roofline"]["frac_of_stream_ceiling"] = round(achieved / ceil, 4) if ceil else None
    if ws == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args, rf_b, au_b)
    elif rank == 0:
        result["cpu_baseline"] = None
    tm.close()
    if not args.no_extras and not args.split_stream and args.iq == "f32" and args.path == "fused":
        # the other configurations, measured in the same run (same box, same clock): C5 at its
        # per-GPU shapes (8 streams and 1 stream, >= 256 blocks per stream) and the u8 FE + mono
        del d_iq, d_dm, d_au
        cpu = ws == 1 and not args.no_cpu and rank == 0
        extras = {
            # (the standalone --workload c5 line's 10 timed spans after 10 warm-up spans: the
            # same measurement; r06 ran 5 after 2, ~8 % below the standalone line on one box)
            "c5": c5_measure(ctx, 8, 256, 10, 10, rank, ws, cpu=cpu, args=args),
            "c5_1stream": c5_measure(ctx, 1, 256, 10, 2, rank, ws),
            "u8": u8_measure(ctx, 128, 50, 10, rank),
            # configs[2] / [3] at fmMonoBlock.py's 51 200-sample blocks: the per-block drop-in path
            # (host buffers, PCIe-inclusive), and configs[3] as a device-resident span
            "c3": rx_measure(ctx, "c3", args, rank, ws, 200, 10, cpu=cpu),
            "c4": rx_measure(ctx, "c4", args, rank, ws, 200, 10, cpu=cpu),
            "c4_span": c5_measure(ctx, 1, 300, 10, 2, rank, ws, cpu=cpu, args=args, B=51_200, rds=False, u8=False,
                                  rf_taps=args.taps),
        }
        cb = extras["c5"].get("cpu_baseline")
        if cb is not None:                       # the CPU leg runs one stream per host thread either way
            extras["c5_1stream"]["cpu_baseline"] = dict(cb, note="the c5 leg (one stream per host thread)")
        if rank == 0:
            result.update(extras)
    if rank == 0:
        emit(result, args)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def _pick(d, keys):
    return {k: d[k] for k in keys if d is not None and k in d}


def compact_line(result: dict) -> dict:
    """The printed line: every headline key, and each extra configuration by its numbers
    (value, ms, stage times, solver counters, CPU baseline) -- short enough that the driver's
    2 000-character tail of stdout holds all of it, c5 last.  The full
    record (notes, samples, per-run strings) goes to the --detail file."""
    out = {k: result[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data") if k in result}
    dv = result.get("devices") or {}
    out["devices"] = {"distinct": dv.get("distinct"), "ranks": dv.get("ranks")}
    cfg = result.get("config", {})
    out["config"] = _pick(cfg, ("blocks_per_step", "complex_per_step", "iq", "path"))
    out["config"]["workload"] = (f"configs[1]+[2]: FE ({cfg.get('taps', '?')} taps, /10, atan2) + mono (151, /5)"
                                 if "taps" in cfg else cfg.get("workload"))
    rf = result.get("roofline", {})
    out["roofline"] = _pick(rf, ("bound", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_ms",
                                 "algorithmic_bytes_per_launch", "read_stream_gbs", "frac_of_stream_ceiling"))
    out["roofline"]["kernel"] = (rf.get("kernel") or "").split(" (")[0]
    cb = result.get("cpu_baseline")
    if cb is not None:
        c = _pick(cb, ("value", "unit", "cores", "kind"))
        c["sample"] = (cb.get("sample") or "")[:48]
        ref = cb.get("reference_cpp_fe") or {}
        c["reference_cpp_fe"] = ref.get("value")
        out["cpu_baseline"] = c
    else:
        out["cpu_baseline"] = None
    cpu_v = lambda d: (d.get("cpu_baseline") or {}).get("value")   # noqa: E731
    if "u8" in result:
        u = result["u8"]
        out["u8"] = dict(_pick(u, ("value", "avg_launch_ms")), frac=u["roofline"]["frac"])
    for key in ("c3", "c4"):
        if key in result:
            r = result[key]
            out[key] = dict(_pick(r, ("value",)), sync_ms=(r.get("sync") or {}).get("ms_per_block"), cpu=cpu_v(r))
    for key in ("c4_span", "c5_1stream"):
        if key in result:
            out[key] = _pick(result[key], ("value", "ms_per_step"))
    if result.get("detail"):
        out["detail"] = result["detail"]
    if "c5" in result:
        r = result["c5"]
        pl = r.get("pll_solver") or {}
        # (stages by the receiver's names, include/sdr.h SDR_RX_ST_*: fe, A = filters of the demod,
        # B = RDS x^2 + BPF, pll, C = stereo mixer + LPF, D = composite RDS filter, E = RRC)
        sk = {"filters_of_demod": "A", "rds_square": "B", "mix_lpf": "C", "resample": "D", "rrc": "E"}
        c5 = _pick(r, ("value", "ms_per_step"))
        c5["stage_ms"] = {sk.get(k, k): v for k, v in (r.get("stage_ms") or {}).items()}
        c5["pll"] = {k: pl.get(k) for k in ("recurrences", "spec_r0", "sequential", "long_stops", "long_tail")}
        rl = r.get("roofline") or {}
        c5["roofline"] = {"stage": sk.get(rl.get("kernel_stage"), rl.get("kernel_stage")), "bound": rl.get("bound"),
                          "frac": rl.get("frac")}
        sr = (r.get("stage_roofline") or {}).get("stages") or {}
        c5["stage_roofline"] = {sk.get(k, k): [v.get("bound"), round(v["frac"], 3) if v.get("frac") is not None else None]
                                for k, v in sr.items()}
        c5["pll_roofline"] = (r.get("pll_roofline") or {}).get("frac")
        c5["cpu"] = cpu_v(r)
        out["c5"] = c5
    return out


def emit(result: dict, args):
    """Rank 0's one JSON line: compact (compact_line) when the record carries the extra
    configurations, with the whole record in args.detail; otherwise the record itself."""
    line = result
    if any(k in result for k in ("c5", "c3", "u8")) and args.detail:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
            with open(args.detail, "w") as f:
                json.dump(result, f)
            result["detail"] = os.path.relpath(os.path.abspath(args.detail), ROOT)
        except OSError as e:
            result["detail"] = f"not written: {e}"
        line = compact_line(result)
    print(json.dumps(line), flush=True)


def cpu_cores():
    """Host cores this process may use, and the CPU model (all cores)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, model


def ref_rx_baseline(args, iq_blocks, B, u8, stereo, rds, rf_taps):
    """The reference's own C++ receiver (oracle/_ref/libref_fe.so, ref_rx_streams), one stream
    per thread on all host cores, ~args.cpu_seconds of wall time; None when the library was not
    built (it needs /root/reference at build time) -- said so in the line."""
    path = os.path.join(ROOT, "oracle", "_ref", "libref_fe.so")
    visible, model = cpu_cores()
    cores = cpu_threads()
    if not os.path.exists(path):
        return {"value": None, "unit": "MS/s", "cores": cores, "kind": "reference", "cpu": model,
                "sample": "not run: oracle/_ref/libref_fe.so absent (built only where /root/reference exists)"}
    lib = ctypes.CDLL(path)
    lib.ref_rx_streams.restype = ctypes.c_double
    lib.ref_rx_streams.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                   ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    x = np.ascontiguousarray(iq_blocks)                 # one stream's blocks, shared read-only by all threads
    n = x.size // 2
    n = (n // B) * B

    def run(threads):
        return lib.ref_rx_streams(x.ctypes.data, int(u8), n, 0, threads, B, rf_taps, int(stereo), int(rds), threads)

    t0 = time.perf_counter()
    run(1)
    t1 = max(time.perf_counter() - t0, 1e-6)
    reps = max(1, int(np.ceil(args.cpu_seconds / t1)))
    t0 = time.perf_counter()
    for _ in range(reps):
        run(cores)
    dt = time.perf_counter() - t0
    return {"value": round(n * cores * reps / dt / 1e6, 3), "unit": "MS/s", "cores": cores, "kind": "reference",
            "cpu": model, "cores_visible": visible,
            "sample": f"{cores} threads x {reps} x {n // B} blocks of {B} complex (one stream per thread), the "
                      f"reference's rf/mono_stereo/rds thread bodies (src/fm_radio.cpp mode 0, stereo={int(stereo)}, "
                      f"rds={int(rds)}) compiled from its sources -O3, {dt:.2f} s wall; {ref_provenance()}"}


def run_rx(args, ws, rank, local):
    """--workload c3 / c4 / c5 --span 1: one JSON line."""
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    ctx = _lib.Context(local)
    result = rx_measure(ctx, args.workload, args, rank, ws, args.steps, args.warmup,
                        cpu=(ws == 1 and not args.no_cpu and rank == 0))
    if rank == 0:
        print(json.dumps(result), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def rx_measure(ctx, workload, args, rank, ws, steps, warmup, cpu=False):
    """c3 / c4 (per-block drop-in path, host buffers) and c5 (multi-stream, device-resident,
    one block per call): the result dict (rank 0; None elsewhere)."""
    import rtsdr
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    c5 = workload == "c5"
    B = 153_600 if c5 else 51_200
    S = args.streams if c5 else 1
    u8 = c5
    stereo = workload in ("c4", "c5")
    rds = c5
    rf_taps = 151 if c5 else args.taps
    rf_b, au_b = rtsdr.design.mono_coeffs(rf_taps, args.audio_taps)
    pipe = not args.no_pipeline
    # the second stream only pays where there is a back half (PLLs, stereo / RDS stages) to
    # overlap; c3's two launches gain nothing from it but the cross-stream event hops
    two_streams = pipe and (stereo or rds)
    depth = 1 if c5 else max(1, args.depth)
    mk = lambda two, d=1: rtsdr.Receiver(S, B, stereo=stereo, rds=rds, iq_dtype=np.uint8 if u8 else np.float32,
                                         rf_coeff=rf_b, audio_coeff=au_b, pipeline=two, depth=d, keep=LEAN_KEEP,
                                         ctx=ctx)
    rx = mk(two_streams, depth if pipe else 1)
    rx_sync = mk(False) if (pipe and not c5) else rx     # the one-block-at-a-time call
    nres = 16                                           # distinct blocks per stream, cycled
    dt = np.uint8 if u8 else np.float32
    # one synthetic stream per stream index (seed = rank * S + s), nres consecutive blocks
    host = np.stack([rtsdr.synth.fm_iq(nres * B, seed=rank * S + s, dtype=dt).reshape(nres, 2 * B)
                     for s in range(S)], axis=1)        # (nres, S, 2B)
    es = 2 if u8 else 8
    fetch = ["audio", "left", "right"] if stereo else ["audio"]
    if c5:
        d_iq = _lib.DeviceBuffer.from_array(ctx, host)
        blk_bytes = S * B * es

        def step(k):
            rx.process_dev(d_iq.ptr + (k % nres) * blk_bytes, B)
    else:
        def sync_step(k):
            return rx_sync.process(host[k % nres], fetch=fetch)

        def step(k):                         # block k launched, block k-depth delivered
            if not pipe:
                return sync_step(k)
            return rx.submit(host[k % nres], fetch=fetch)
    for k in range(warmup):
        step(k)
    if not c5:
        rx.flush()
    ctx.synchronize()
    t_set = time.perf_counter()
    settle = 0
    while (time.perf_counter() - t_set) * 1e3 < args.settle_ms:
        for _ in range(8):
            step(settle)
            settle += 1
        ctx.synchronize()
    # per-stage GPU times (events between the receiver's launches), a separate pass -- on a
    # receiver past its stream's first blocks (the PLLs' acquisition block runs sequentially)
    if not c5 and rx_sync is not rx:
        for k in range(4):
            sync_step(k)
    (rx if c5 else rx_sync).set_timing(True)
    stages = []
    for k in range(8):
        rx.process_dev(d_iq.ptr + (k % nres) * blk_bytes, B) if c5 else rx_sync.process(host[k % nres], fetch=fetch)
        stages.append((rx if c5 else rx_sync).stage_ms())
    (rx if c5 else rx_sync).set_timing(False)
    sync = None
    if not c5 and pipe:                      # the synchronous drop-in call, for its latency
        sl = []
        for k in range(steps):
            t = time.perf_counter()
            sync_step(k)
            sl.append(time.perf_counter() - t)
        sl = np.array(sl) * 1e3
        sync = {"ms_per_block": round(float(sl.mean()), 4), "p50": round(float(np.median(sl)), 4),
                "p99": round(float(np.percentile(sl, 99)), 4),
                "MS/s": round(S * B / (float(sl.mean()) * 1e-3) / 1e6, 1)}
    stage_ms = {key: round(float(np.mean([st[key] for st in stages])), 5) for key in stages[0]}
    if stereo:
        rx.pll_stats(reset=True)
    barrier(ws)
    ctx.synchronize()
    lat = []
    t0 = time.perf_counter()
    if c5:
        tm = _lib.Timer(ctx)
        e0, e1 = tm.event(), tm.event()
        tm.record(e0)
        for k in range(steps):
            step(k)
        tm.record(e1)
    else:
        for k in range(steps):
            t = time.perf_counter()
            step(k)
            lat.append(time.perf_counter() - t)
        rx.flush()
    ctx.synchronize()
    barrier(ws)
    elapsed = max_over_ranks(ws, time.perf_counter() - t0)
    gpu_ms = tm.elapsed_ms(e0, e1) / steps if c5 else None
    pll = rx.pll_stats() if stereo else None
    result = None
    if rank == 0:
        total = S * B * steps * ws
        M = B // 10
        dom = max(stage_ms, key=stage_ms.get)
        # the front end is the HBM-streaming kernel of the chain: IQ in + demod out per launch
        fe_bytes = S * (B * es + M * 4)
        fe_gbs = fe_bytes / (stage_ms["fe"] * 1e-3) / 1e9
        if dom == "pll" and pll is not None:
            par = pll["spec_r0"] + pll["spec_r1"] + pll["spec_r2"]
            dom_bound = (f"PLL: {par} of {pll['recurrences']} timed recurrences solved in parallel "
                         f"(pll_spec_kernel, one workgroup per recurrence), {pll['sequential']} by the "
                         "sequential kernel")
        elif dom == "fe":
            dom_bound = "FE: IQ in, demod out (see roofline)"
        else:
            dom_bound = "stage FIRs: FP32 VALU multiply-adds"
        result = {
            "metric": f"IQ MSamples/s through the {'multi-stream mono+stereo+RDS receiver' if c5 else 'per-block drop-in path'}"
                      f" ({workload}); achieved HBM GB/s vs peak",
            "value": round(total / elapsed / 1e6, 1), "unit": "MS/s", "n_gpus": args.devices["distinct"],
            "devices": args.devices, "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": (f"synthetic FM IQ (seed = rank*streams + stream), interleaved {'u8' if u8 else 'f32'}, "
                     + ("device-resident, 16 distinct blocks per stream cycled" if c5 else
                        "host buffers: each step uploads one block and downloads its outputs (PCIe-inclusive)")),
            "config": {"workload": {"c3": "configs[2]: FE + mono per block, fmMonoBlock.py block size",
                                    "c4": "configs[3]: FE + mono + stereo per block, fmMonoBlock.py block size",
                                    "c5": "configs[4]: independent streams, mono + stereo + RDS to the RRC output"}
                       [workload],
                       "block_complex": B, "streams_per_gpu": S, "rf_taps": rf_taps, "iq": "u8" if u8 else "f32",
                       "parallelism": f"independent streams x{S * ws}",
                       "pipeline": " + ".join(
                           ([f"sdr_rx_submit: block k launched while block k-{depth} is delivered "
                             f"({depth} block{'s' if depth > 1 else ''} in flight)"] if (not c5 and pipe) else [])
                           + (["front half (FE, stage A) of block k beside the back half of k-1 (two streams)"]
                              if two_streams else [])) or None},
            "roofline": {"bound": "hbm", "achieved": round(fe_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(fe_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": f"FE stage (fe_slot/ring kernel, {rf_taps} taps, + its zf and phase kernels)",
                         "algorithmic_bytes_per_launch": fe_bytes, "avg_launch_ms": stage_ms["fe"]},
            "stage_ms": stage_ms,
            "dominant_stage": {"stage": dom, "ms": stage_ms[dom], "bound": dom_bound},
        }
        if pll is not None:
            result["pll_solver"] = pll
        if c5:
            result["gpu_ms_per_block"] = round(gpu_ms, 5)
            # the chain is FIR work on the FP32 VALU (the FE stage's HBM figure stays beside it)
            fps = chain_flops_per_sample()
            tf = fps * S * B / (gpu_ms * 1e-3) / 1e12
            result["fe_roofline"] = result["roofline"]
            result["roofline"] = {"bound": "valu", "achieved": round(tf, 3), "peak": VALU_PEAK_TFLOPS,
                                  "unit": "TFLOP/s", "frac": round(tf / VALU_PEAK_TFLOPS, 4), "traffic": None,
                                  "flops_per_sample": round(fps, 2),
                                  "note": "FIR flops of the whole chain per input sample x samples / GPU ms per block"}
        else:
            la = np.array(lat) * 1e3
            result["block_latency_ms"] = ({"mean": round(float(la.mean()), 4), "p50": round(float(np.median(la)), 4),
                                           "p99": round(float(np.percentile(la, 99)), 4)} if sync is None else
                                          {"mean": sync["ms_per_block"], "p50": sync["p50"], "p99": sync["p99"],
                                           "note": "sdr_rx_run (one block in flight)"})
            if sync is not None:
                result["sync"] = sync
            result["realtime_factor"] = round((total / elapsed) / 2.4e6, 1)     # x the 2.4 MS/s input rate
    if cpu and rank == 0:
        result["cpu_baseline"] = ref_rx_baseline(args, host[:, 0].reshape(-1), B, u8, stereo, rds, rf_taps)
    elif rank == 0:
        result["cpu_baseline"] = None
    rx.close()
    rx_sync.close()
    return result

C5_B = 153_600                 # complex samples per reference block (src/fm_radio.cpp:23)
# what the receivers materialise on their device-resident path: every output but the NCO rows,
# the RDS LPF rows and (spans) the PLLs' f32 input rows -- intermediates the chain does not need
# (sdr_rx_set_keep): the mixers form the NCO from the PLL phases, the RDS LPF runs inside the
# composite resampler, the PLLs read their inputs as sign codes (the same values either way)
LEAN_KEEP = ("demod", "audio", "bpf_extraction", "stereo", "left", "right", "extract",
             "resample_i", "resample_q", "rrc_i", "rrc_q")
VALU_PEAK_TFLOPS = 157.3       # MI355X FP32 vector peak (MI355X_MICROARCH.md)
# f64 VALU issue: a wave64 f64 instruction holds its SIMD 4 cycles (half the f32 rate: 78.6
# TFLOP/s FMA), 256 CUs x 4 SIMDs x 2.4 GHz / 4 (tools/f64_probe.hip measured a lone wave at
# ~4.5 cycles per f64 op, dependent or not)
F64_WAVE_INSTR_PEAK = 256 * 4 * 2.4e9 / 4


def pll_roofline(stage_ms_pll, S, K, B, steps_per_span, path=None):
    """The PLL stage against the f64 VALU issue rate, from the committed SQ counts of its kernels
    (tools/pmc_c5.py over rocprofv3 --pmc passes of the same configuration: pll_spec_kernel +
    pll_long_fix_kernel) and the stage time measured in this run.  None when no counts for this
    configuration are committed."""
    path = path or C5_PMC
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    cfg = t.get("config", {})
    if cfg.get("streams") != S or cfg.get("span") != K or cfg.get("block_complex") != B:
        return None
    c = t.get("stages", {}).get("pll") or {}
    f64, valu = c.get("f64_wave_instr", 0.0), c.get("valu_wave_instr", 0.0)
    if not f64 or stage_ms_pll <= 0:
        return None
    rate = f64 / (stage_ms_pll * 1e-3)
    return {"bound": "f64 VALU issue", "achieved": round(rate / 1e9, 2), "peak": round(F64_WAVE_INSTR_PEAK / 1e9, 1),
            "unit": "G f64 wave-instr/s", "frac": round(rate / F64_WAVE_INSTR_PEAK, 4),
            "f64_wave_instr_per_span": f64, "valu_wave_instr_per_span": valu,
            "f64_lane_ops_per_step": round(64 * f64 / steps_per_span, 2),
            "valu_lane_ops_per_step": round(64 * valu / steps_per_span, 2),
            "kernels": c.get("kernels"), "stage_ms": stage_ms_pll,
            "source": os.path.relpath(path, ROOT) + " (SQ counts per span call) + this run's PLL stage time"}


SIMDS, CLOCK_HZ = 256 * 4, 2.4e9   # MI355X: 256 CUs x 4 SIMDs; nominal clock (the chip runs lower under load)
MFMA_F16_PEAK_TFLOPS = 2500.0    # dense f16 / bf16 matrix-core peak (MI355X_MICROARCH.md; not the 2:1-sparse figure)
MFMA_I8_PEAK_TOPS = 5000.0       # dense int8 matrix-core peak: 2x the f16 rate per clock (MI355X_MICROARCH.md)
C5_PMC = os.path.join(ROOT, "profiles", "r06", "c5_pmc.json")


def c5_stage_roofline(stage_ms, S, K, B, path=C5_PMC):
    """Each C5 span stage against the ceilings it can hit: HBM bytes / s vs 8 TB/s, executed
    matrix-core ops / s vs the dense f16 (2.5 PF) or int8 (5 POPS) peak, f64 VALU wave-
    instructions / s vs the f64 issue rate -- from committed per-stage counts of the same
    configuration (tools/pmc_c5.py over rocprofv3 --pmc passes of `bench.py --workload c5`) and
    THIS run's per-stage times (solo).  `bound` is the ceiling the stage comes closest to and
    `frac` its fraction.  None when no counts for this configuration are committed."""
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    cfg = t.get("config", {})
    if cfg.get("streams") != S or cfg.get("span") != K or cfg.get("block_complex") != B:
        return None
    out = {}
    for st, c in t["stages"].items():
        ms = stage_ms.get(st, 0.0)
        if ms <= 0:
            continue
        sec = ms * 1e-3
        e = {"ms": ms}
        if "hbm_read_bytes" in c and "hbm_write_bytes" in c:
            gbs = (c["hbm_read_bytes"] + c["hbm_write_bytes"]) / sec / 1e9
            e["hbm"] = {"achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
        if c.get("mfma_ops_f16"):
            tf = c["mfma_ops_f16"] / sec / 1e12
            e["mfma_f16"] = {"achieved_tflops": round(tf, 1), "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4)}
        if c.get("mfma_ops_i8"):
            to = c["mfma_ops_i8"] / sec / 1e12
            e["mfma_i8"] = {"achieved_tops": round(to, 1), "frac": round(to / MFMA_I8_PEAK_TOPS, 4)}
        if c.get("f64_wave_instr"):
            g = c["f64_wave_instr"] / sec
            e["f64_issue"] = {"achieved_g_wave_instr_s": round(g / 1e9, 1), "frac": round(g / F64_WAVE_INSTR_PEAK, 4)}
        # the SIMDs' vector issue and matrix pipes: busy cycles (SQ_ACTIVE_INST_VALU counts quad-cycles)
        # over the stage's SIMD-cycles at the nominal 2.4 GHz
        simd_cycles = SIMDS * CLOCK_HZ * sec
        if c.get("valu_active_quad_cycles"):
            e["valu_issue"] = {"busy_simd_cycles": c["valu_active_quad_cycles"] * 4,
                               "frac": round(4 * c["valu_active_quad_cycles"] / simd_cycles, 4)}
        if c.get("mfma_busy_cycles"):
            e["mfma_busy"] = {"busy_simd_cycles": c["mfma_busy_cycles"],
                              "frac": round(c["mfma_busy_cycles"] / simd_cycles, 4)}
        lim = {k: v["frac"] for k, v in e.items() if isinstance(v, dict)}
        if lim:
            e["bound"] = max(lim, key=lim.get)
            e["frac"] = lim[e["bound"]]
        out[st] = e
    return {"stages": out, "source": os.path.relpath(path, ROOT) + " (per-stage counts per span call) + this run's "
                                                                    "stage times"}


def c5_stage_bytes(stage, path=C5_PMC):
    """HBM bytes (read + write, PMC) of one C5 stage per span call, or None"""
    try:
        with open(path) as f:
            c = json.load(f)["stages"][stage]
        return c["hbm_read_bytes"] + c["hbm_write_bytes"]
    except (OSError, ValueError, KeyError):
        return None


def chain_flops_per_sample(rf_taps=151, taps=151, audio_decim=5, up=19, down=80):
    """FP32 flops (2 per multiply-add) of the C5 chain's FIR work per complex input sample, as
    the kernels run it: the RF FIR on I and Q at 1/10 of the
    input rate, then per demod sample the stage filters (stage_macs_per_demod: the RDS LPF and
    resampler as the composite filter).  The demod atan2, the NCOs and the PLLs (f64) are not
    counted."""
    macs_demod = sum(stage_macs_per_demod(taps, audio_decim, up, down).values())
    return 2.0 * (2 * rf_taps + macs_demod) / 10.0


def stage_macs_per_demod(taps=151, audio_decim=5, up=19, down=80, stereo=True, rds=True):
    """Multiply-adds per demod-rate sample of each receiver stage as the kernels run them
    (csrc/rx.hip, the bench's keep set): stage A = audio LPF /5 + pilot BPF + stereo BPF + RDS
    extract BPF, B = the RDS square BPF, C = the stereo mixer LPF /5, D = the RDS I/Q mixers +
    3 kHz LPF + x19 /80 resampler as one composite filter (158 taps per output, 19/80 outputs
    per sample), E = RRC I/Q at the resampled rate.  The NCOs the mixers form (f64 sincos) are
    not counted."""
    m = {"filters_of_demod": taps / audio_decim + (2 * taps if stereo else 0) + (taps if rds else 0)}
    if rds:
        m["rds_square"] = taps
    m["mix_lpf"] = taps / audio_decim if stereo else 0
    if rds:
        # the RDS mixers + LPF + resampler as one composite polyphase filter: (taps + 7)
        # multiply-adds per output and channel, up/down outputs per demod sample
        m["resample"] = 2 * (taps + (taps - 1) // up) * up / down
        m["rrc"] = 2 * taps * up / down
    return m


def c5_measure(ctx, S, K, steps, warmup, rank, ws, pipeline=True, cpu=False, args=None, B=None, stereo=True,
               rds=True, u8=True, rf_taps=151):
    """configs[4] per GPU: S independent u8 streams of K reference blocks each, device-resident,
    mono + stereo + RDS to the RRC output, K blocks of every stream per receiver call (one
    span: the time-parallel receiver).  The synthetic span is K x 64 ms, over
    which every tone of the composite completes whole cycles, so repeating it is seamless
    (the PLLs stay locked across steps); stream s is the span rotated by s/S of its length.
    Also the span form of configs[3] (c4_span: B = 51 200 f32, stereo without RDS; K chosen
    so that the span is a whole number of every tone's cycles too)."""
    import rtsdr
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    B = C5_B if B is None else B
    rf_b, au_b = rtsdr.design.mono_coeffs(rf_taps, 151)
    n = K * B
    dt = np.uint8 if u8 else np.float32
    base = rtsdr.synth.fm_iq(n, seed=rank * 1009, dtype=dt)
    rows = np.stack([np.roll(base, 2 * ((s * n // S) // 50 * 50)) for s in range(S)])
    del base
    d_iq = _lib.DeviceBuffer.from_array(ctx, rows)
    cpu_rows = rows[0, :16 * 2 * B].copy() if cpu else None
    del rows
    rx = rtsdr.Receiver(S, n, stereo=stereo, rds=rds, iq_dtype=dt, rf_coeff=rf_b, audio_coeff=au_b,
                        pipeline=pipeline, keep=LEAN_KEEP, ctx=ctx)

    def step():
        rx.process_dev(d_iq.ptr, n)

    for _ in range(warmup):
        step()
    ctx.synchronize()
    rx.set_timing(True)                       # per-stage GPU times: a separate pass
    stages = []
    for _ in range(2):
        step()
        stages.append(rx.stage_ms())
    rx.set_timing(False)
    stage_ms = {k: round(float(np.mean([st[k] for st in stages])), 4) for k in stages[0]}
    rx.pll_stats(reset=True)
    barrier(ws)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    barrier(ws)
    elapsed = max_over_ranks(ws, time.perf_counter() - t0)
    pll = rx.pll_stats()
    # one call on its own (nothing else in flight): the latency of a span, next to the
    # pipelined throughput above
    t1 = time.perf_counter()
    step()
    ctx.synchronize()
    latency = time.perf_counter() - t1
    rx.close()
    d_iq.free()
    total = S * n * steps * ws
    fps = chain_flops_per_sample() if rds else None
    dom = max(stage_ms, key=stage_ms.get)
    out = {
        "value": round(total / elapsed / 1e6, 1), "unit": "MS/s",
        "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps, "warmup": warmup,
        "mode": (f"span: {K} blocks of every stream per receiver call, device-resident (pipelined calls); not the "
                 f"per-block real-time loop -- one call covers {K * B / 2.4e6:.2f} s of radio"),
        "ms_per_call": round(elapsed / steps * 1e3, 4), "call_latency_ms": round(latency * 1e3, 4),
        "config": {"streams_per_gpu": S, "blocks_per_stream_per_step": K, "block_complex": B,
                   "complex_per_step": S * n, "iq": "u8" if u8 else "f32", "rf_taps": rf_taps,
                   "pipeline": bool(pipeline),
                   "chain": ("FE + mono + stereo + RDS to the RRC output (fmMonoBlock.py:80-173, fmRDSblock.py:127-204)"
                             if rds else "FE + mono + stereo (fmMonoBlock.py:80-173)")},
        "stage_ms": stage_ms,
        "dominant_stage": {"stage": dom, "ms": stage_ms[dom],
                           "bound": ("PLL: pseudo-blocks solved in parallel from warm-up guesses and chained "
                                     "(f64, csrc/pll.hip long calls)") if dom == "pll" else
                           ("HBM: IQ in, demod out" if dom == "fe" else
                            "FIR multiply-adds (span rows on the matrix cores, f16 hi/lo; per-block rows on the "
                            "FP32 VALU)")},
        "pll_solver": pll,
    }
    # per-stage achieved FP32 TFLOP/s (2 flops per multiply-add) against VALU_PEAK_TFLOPS, and the
    # FE's HBM GB/s (IQ in, demod out)
    demod = S * n / 10
    out["stage_tflops"] = {k: round(2 * v * demod / (stage_ms[k] * 1e-3) / 1e12, 1)
                           for k, v in stage_macs_per_demod(stereo=stereo, rds=rds).items()
                           if stage_ms.get(k, 0) > 0}
    out["fe_gbs"] = (round((S * n * (2 if u8 else 8) + 4 * demod) / (stage_ms["fe"] * 1e-3) / 1e9, 1)
                     if stage_ms.get("fe") else None)
    pr = pll_roofline(stage_ms.get("pll", 0.0), S, K, B, (2 if rds else 1) * S * (n // 10)) if stereo else None
    if pr is not None:
        out["pll_roofline"] = pr
    if fps is not None:
        # the chain's f32-equivalent FIR rate (2 flops per useful multiply-add, whatever unit runs it):
        # a throughput figure, not a roofline fraction (the span filters run on the matrix cores)
        out["chain_f32eq_tflops"] = round(fps * S * n * steps / elapsed / 1e12, 3)
    if out["fe_gbs"] is not None:
        # without committed per-stage counts: the FE's algorithmic HBM rate (IQ in, demod out)
        out["roofline"] = {"bound": "hbm", "kernel_stage": "fe", "achieved": out["fe_gbs"], "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(out["fe_gbs"] / HBM_PEAK_GBS, 4), "traffic": None,
                           "note": "the FE stage's algorithmic bytes / its time (no per-stage PMC counts committed)"}
    sr = c5_stage_roofline(stage_ms, S, K, B) if (stereo and rds and u8) else None
    if sr is not None:
        out["stage_roofline"] = sr
        # the line's roofline: the dominant stage's own, against the ceiling it comes closest to
        d = sr["stages"].get(dom)
        if d is not None and "bound" in d:
            unit = {"hbm": "GB/s", "mfma_f16": "TFLOP/s", "mfma_i8": "TOP/s", "f64_issue": "G f64 wave-instr/s",
                    "valu_issue": "SIMD-cycles", "mfma_busy": "SIMD-cycles"}[d["bound"]]
            b = d[d["bound"]]
            ach = next(v for k, v in b.items() if k.startswith("achieved") or k.startswith("busy"))
            peak = {"hbm": HBM_PEAK_GBS, "mfma_f16": MFMA_F16_PEAK_TFLOPS, "mfma_i8": MFMA_I8_PEAK_TOPS,
                    "f64_issue": round(F64_WAVE_INSTR_PEAK / 1e9, 1),
                    "valu_issue": round(SIMDS * CLOCK_HZ * d["ms"] * 1e-3),
                    "mfma_busy": round(SIMDS * CLOCK_HZ * d["ms"] * 1e-3)}[d["bound"]]
            out["roofline"] = {"bound": d["bound"], "kernel_stage": dom, "achieved": ach, "peak": peak, "unit": unit,
                               "frac": d["frac"], "traffic": c5_stage_bytes(dom),
                               "note": ("the dominant stage's own ceiling (stage_roofline); traffic: its HBM bytes per "
                                        "span call (PMC)")}
    if cpu and args is not None:
        out["cpu_baseline"] = ref_rx_baseline(args, cpu_rows, B, u8, stereo, rds, rf_taps)
    return out


def u8_measure(ctx, blocks, steps, warmup, rank, settle_ms=250.0):
    """The u8 fused FE + mono kernel (fe_mfma_mono_kernel: the RF FIR on the int8 matrix
    cores) over `blocks` x 1 024 000 u8 samples of one device-resident stream: HIP events
    around the launches on the libsdr stream."""
    import rtsdr
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    lib, h = ctx.lib, ctx.handle
    rf_b, au_b = rtsdr.design.mono_coeffs(101, 151)
    n = blocks * BLOCK
    M = (n + 9) // 10
    A = (M + 4) // 5
    d_iq = _lib.DeviceBuffer.from_array(ctx, rtsdr.synth.fm_iq(n, seed=rank, dtype=np.uint8))
    d_au = _lib.DeviceBuffer(ctx, 4 * A)
    rfp, aup = _lib.f64p(rf_b), _lib.f64p(au_b)

    def launch():
        _lib.check(lib.sdr_fe_mono_dev(h, d_iq.ptr, _lib.SDR_IQ_U8, n, n, 1, rfp, 101, 10, aup, 151, 5, d_au.ptr, A),
                   "fe_mono u8")

    for _ in range(warmup):
        launch()
    ctx.synchronize()
    # clock settle (as the headline's): this leg runs after the receiver legs in the same
    # process, and 10 warm-up launches alone measured it 25 % slow
    t_set = time.perf_counter()
    while (time.perf_counter() - t_set) * 1e3 < settle_ms:
        for _ in range(16):
            launch()
        ctx.synchronize()
    tm = _lib.Timer(ctx)
    e0, e1 = tm.event(), tm.event()
    tm.record(e0)
    for _ in range(steps):
        launch()
    tm.record(e1)
    k_ms = tm.elapsed_ms(e0, e1) / steps
    tm.close()
    d_iq.free()
    d_au.free()
    k_bytes = n * 2 + A * 4
    gbs = k_bytes / (k_ms * 1e-3) / 1e9
    return {"value": round(n / (k_ms * 1e-3) / 1e6, 1), "unit": "MS/s", "avg_launch_ms": round(k_ms, 5),
            "config": {"blocks": blocks, "block_complex": BLOCK, "iq": "u8", "rf_taps": 101, "audio_taps": 151},
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(os.path.join(ROOT, "profiles", "fe_pmc_traffic.json"), 101, blocks,
                                                 "u8_mfma"),
                         "kernel": "fe_mfma_mono_kernel (RF FIR on v_mfma_i32_16x16x64_i8) + audio FIR",
                         "algorithmic_bytes_per_launch": k_bytes}}


def run_c5_span(args, ws, rank, local):
    """--workload c5 (span > 1): the time-parallel receiver, one JSON line."""
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    ctx = _lib.Context(local)
    m = c5_measure(ctx, args.streams, args.span, args.steps, args.warmup, rank, ws,
                   pipeline=not args.no_pipeline, cpu=(ws == 1 and not args.no_cpu and rank == 0), args=args)
    if rank == 0:
        result = {"metric": "IQ MSamples/s through the multi-stream mono+stereo+RDS receiver (c5); "
                            "the dominant stage against its roofline",
                  "value": m["value"], "unit": "MS/s", "n_gpus": args.devices["distinct"], "devices": args.devices,
                  "steps": args.steps, "warmup": args.warmup,
                  "ms_per_step": m["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                  "dtype": "f32",
                  "data": "synthetic FM IQ (u8), device-resident, one seamless span per stream repeated",
                  "config": dict(m["config"], workload="configs[4]: independent streams, mono + stereo + RDS to the "
                                                       "RRC output, time-parallel spans",
                                 parallelism=f"independent streams x{args.streams * ws}"),
                  "roofline": m.get("roofline"), "stage_ms": m["stage_ms"], "dominant_stage": m["dominant_stage"],
                  "stage_roofline": m.get("stage_roofline"), "pll_roofline": m.get("pll_roofline"),
                  "pll_solver": m["pll_solver"], "cpu_baseline": m.get("cpu_baseline")}
        print(json.dumps(result), flush=True)
    if ws > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def live_run(cmd, data: bytes, repeat: int, env=None):
    """One live-receiver process: `data` written `repeat` times to its stdin (as rtl_sdr would
    pipe it), stdout discarded (the int16 stream is counted), stderr kept.  Returns (wall
    seconds from process start to exit, stdout bytes, stderr text, return code)."""
    import subprocess
    import threading
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env)
    nout = [0]
    err = []

    def feed():
        try:
            for _ in range(repeat):
                p.stdin.write(data)
            p.stdin.close()
        except BrokenPipeError:
            pass

    def drain_out():
        while True:
            b = p.stdout.read(1 << 20)
            if not b:
                break
            nout[0] += len(b)

    def drain_err():
        err.append(p.stderr.read().decode(errors="replace"))

    th = [threading.Thread(target=f, daemon=True) for f in (feed, drain_out, drain_err)]
    for t in th:
        t.start()
    rc = p.wait()
    for t in th:
        t.join()
    return time.perf_counter() - t0, nout[0], "".join(err), rc


def run_live(args, ws, rank, local):
    """SURVEY §8f row 2, end to end: fm_radio_gpu mode 0 (stereo + --rds) on a u8 stream fed
    through its stdin, int16 L/R counted off its stdout, beside the reference's own fm_radio
    (src/fm_radio.cpp, all of src/ compiled by oracle/Makefile `ref` into oracle/_ref/) on the
    same bytes on the same host.  The stream is a seamless synthetic span (every tone completes
    whole cycles over it, coded RDS groups) of --span blocks of 307 200 bytes, written
    --live-repeat times; wall time from process start to exit (startup included), and the
    marginal rate between a 1x and an Nx run (startup excluded)."""
    import rtsdr
    if rank != 0:
        return
    K = args.span
    data = rtsdr.synth.fm_iq(K * C5_B, seed=11, dtype=np.uint8, rds_groups=True).tobytes()
    env = dict(os.environ, SDR_DEVICE=str(local))
    gpu_bin = os.path.join(ROOT, "real-time-software-defined-radio_amd", "fm_radio_gpu")
    ref_bin = os.path.join(ROOT, "oracle", "_ref", "fm_radio")
    out = {"metric": "IQ MSamples/s end to end through the live receiver (u8 stdin -> int16 L/R stdout), mode 0 "
                     "stereo + RDS; real-time factor vs 2.4 MS/s",
           "unit": "MS/s", "n_gpus": 1, "higher_is_better": True, "scaling": "replicas only", "vs_baseline": None,
           "dtype": "f32", "data": f"synthetic u8 FM IQ with coded RDS groups, {K} blocks of {2 * C5_B} bytes, "
                                   f"fed through stdin",
           "config": {"workload": "SURVEY §8f row 2: live pipeline (src/fm_radio.cpp:31-441, 732-798)",
                      "blocks_per_pass": K, "block_bytes": 2 * C5_B, "cmd": "fm_radio_gpu --rds"}}

    def measure(cmd, reps):
        rows = []
        for r in reps:
            wall, nbytes, err, rc = live_run(cmd, data, r, env=env)
            if rc != 0:
                raise SystemExit(f"bench live: {cmd[0]} exited {rc}: {err[-2000:]}")
            n = r * K * C5_B
            rows.append({"passes": r, "complex": n, "wall_s": round(wall, 4), "MS/s": round(n / wall / 1e6, 3),
                         "realtime_factor": round(n / wall / 2.4e6, 2), "stdout_bytes": nbytes,
                         "syndrome_lines": err.count("Syndrome")})
        a, b = rows[0], rows[-1]
        marg = (b["complex"] - a["complex"]) / max(b["wall_s"] - a["wall_s"], 1e-9)
        return rows, round(marg / 1e6, 3)

    reps = [1, args.live_repeat]
    g_rows, g_marg = measure([gpu_bin, "--rds"], reps)
    out["runs"] = g_rows
    out["value"] = g_rows[-1]["MS/s"]
    out["realtime_factor"] = g_rows[-1]["realtime_factor"]
    out["marginal_MS/s"] = g_marg
    out["marginal_realtime_factor"] = round(g_marg / 2.4, 2)
    out["host_threads"] = 1
    visible, model = cpu_cores()
    if os.path.exists(ref_bin) and not args.no_cpu:
        r_rows, r_marg = measure([ref_bin], [1, 2])
        out["cpu_baseline"] = {"value": r_rows[-1]["MS/s"], "unit": "MS/s", "cores": 4, "kind": "reference",
                               "cpu": model, "cores_visible": visible, "marginal_MS/s": r_marg,
                               "realtime_factor": r_rows[-1]["realtime_factor"], "runs": r_rows,
                               "sample": f"oracle/_ref/fm_radio (the reference's src/ compiled -O3 -pthread; its "
                                         f"4 threads rf / mono_stereo / rds / frame), mode 0, the same bytes, "
                                         f"1x and 2x passes; {ref_provenance()}"}
    else:
        out["cpu_baseline"] = {"value": None, "kind": "reference",
                               "sample": "not run: oracle/_ref/fm_radio absent (make -C oracle ref, where "
                                         "/root/reference exists)" if not args.no_cpu else "skipped (--no-cpu)"}
    out["steps"] = args.live_repeat
    out["warmup"] = 0
    out["ms_per_step"] = round(g_rows[-1]["wall_s"] / args.live_repeat * 1e3, 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
