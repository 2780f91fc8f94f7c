"""bench.py's N>1 path on CPU: world_size-2 gloo ranks exercise dist_setup, the barrier
and the max-over-ranks reduction that bench.py's timed region uses (no GPU, no RCCL:
the data path has no collective); and the --split-stream data path: each rank
takes its range of ONE stream plus the read-only halo before it (bench.split_range,
rtsdr.split_halo), runs it through the C oracle (oracle/_build/liboracle.so, the checker:
no GPU here), and the ranks' outputs gathered in rank order equal the whole-stream pass."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys, json
sys.path.insert(0, os.environ["ROOT"])
import bench
class A: pass
ws, rank, local = bench.dist_setup(A())
assert ws == 2 and rank == int(os.environ["RANK"]) and local == rank
bench.barrier(ws)
m = bench.max_over_ranks(ws, 1.5 + rank)          # each rank's "elapsed"
import torch.distributed as dist
print(json.dumps({"rank": rank, "max": m}), flush=True)
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_gloo_barrier_and_max():
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-c", WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    import json
    res = sorted((json.loads(o.strip().splitlines()[-1]) for o, _ in outs), key=lambda d: d["rank"])
    assert [d["max"] for d in res] == [2.5, 2.5]


SPLIT_WORKER = r"""
import ctypes, os, sys, json
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
import bench, rtsdr
class A: pass
ws, rank, local = bench.dist_setup(A())
lib = ctypes.CDLL(os.path.join(os.environ["ROOT"], "oracle", "_build", "liboracle.so"))
P = np.ctypeslib.ndpointer
lib.orc_fe_mono.argtypes = [P(np.float32), ctypes.c_int64, P(np.float64), ctypes.c_int, P(np.float64), ctypes.c_int,
                            ctypes.c_void_p, P(np.float64)]
rf_b, au_b = rtsdr.design.mono_coeffs(101, 151)
def fe_mono(iq):
    n = iq.size // 2
    out = np.empty(((n + 9) // 10 + 4) // 5)
    lib.orc_fe_mono(np.ascontiguousarray(iq), n, rf_b, len(rf_b), au_b, len(au_b), None, out)
    return out
n_total = int(os.environ["N_TOTAL"])
iq = rtsdr.synth.fm_iq(n_total, seed=0)
w0, s0, s1 = bench.split_range(n_total, ws, rank, rtsdr.split_halo(len(rf_b), len(au_b)))
a = fe_mono(iq[2 * w0:2 * s1])
mine = a[(s0 - w0) // 50:(s1 - w0 + 49) // 50]         # audio samples of IQ positions [s0, s1)
import torch.distributed as dist
parts = [None] * ws
dist.all_gather_object(parts, (rank, w0, s0, s1, mine.tolist()))
if rank == 0:
    parts.sort()
    got = np.concatenate([np.array(p[4]) for p in parts])
    want = fe_mono(iq)
    print(json.dumps({"ranges": [p[1:4] for p in parts], "n": int(got.size), "n_want": int(want.size),
                      "maxdiff": float(np.max(np.abs(got - want))) if got.size == want.size else None}), flush=True)
else:
    print(json.dumps({"rank": rank}), flush=True)
dist.destroy_process_group()
"""


def test_two_rank_split_stream_ranges_gather_to_the_whole_pass():
    """Two gloo ranks, one stream of 6 x 51 200 + 7 samples split at a whole audio sample:
    every audio sample comes from exactly one rank, and the concatenation equals the
    whole-stream oracle.  (To f64 rounding: the oracle's demod carries the reference's
    accumulated unwrapped phase, model/fmSupportLib.py:40-44, whose magnitude -- and so its
    rounding -- depends on where a pass starts; the GPU kernels' split is bit-identical,
    tests/test_gpu_parity.py::test_split_stream_ranges_equal_single_pass.)"""
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), N_TOTAL=str(6 * 51200 + 7))
        procs.append(subprocess.Popen([sys.executable, "-c", SPLIT_WORKER], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    import json
    res = json.loads(outs[0][0].strip().splitlines()[-1])
    (w0a, s0a, s1a), (w0b, s0b, s1b) = res["ranges"]
    assert s0a == 0 and s1a == s0b and s1b == 6 * 51200 + 7 and w0b < s0b
    assert res["n"] == res["n_want"]
    assert res["maxdiff"] < 1e-12, res


def test_device_for_refuses_to_wrap():
    """A line must not claim N GPUs that did not run: more ranks than visible devices is
    refused unless --allow-wrap (one-GPU rehearsals), which wraps the ranks."""
    sys.path.insert(0, ROOT)
    import bench
    import pytest
    assert bench.device_for(1, count=2) == 1
    with pytest.raises(SystemExit):
        bench.device_for(3, count=2)
    assert bench.device_for(3, allow_wrap=True, count=2) == 1
    with pytest.raises(SystemExit):
        bench.device_for(0, count=0)


DEVMAP_WORKER = r"""
import os, sys, json
sys.path.insert(0, os.environ["ROOT"])
import bench
class A: pass
ws, rank, local = bench.dist_setup(A())
shared = os.environ["SHARED"] == "1"
pci = "0000:05:00.0" if shared else f"0000:{5 + rank:02x}:00.0"
dmap = bench.device_map(ws, rank, {"device": local, "pci_bus_id": pci, "cus": 256})
res = {"rank": rank, "map": dmap}
try:
    res["distinct"] = bench.check_devices(dmap, allow_wrap=False)
except SystemExit as e:
    res["refused"] = str(e)
res["wrapped"] = bench.check_devices(dmap, allow_wrap=True)
import torch.distributed as dist
print(json.dumps(res), flush=True)
dist.destroy_process_group()
"""


def _run2(worker, extra):
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **extra)
        procs.append(subprocess.Popen([sys.executable, "-c", worker], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    import json
    return sorted((json.loads(o.strip().splitlines()[-1]) for o, _ in outs), key=lambda d: d["rank"])


def test_two_rank_device_map():
    """bench.py's rank -> device map, gathered over gloo: two ranks on two devices report 2
    distinct; two ranks on ONE device (a misconfigured node) are refused unless wrapping was
    asked for, in which case the line counts 1 device."""
    res = _run2(DEVMAP_WORKER, {"SHARED": "0"})
    for d in res:
        assert d["distinct"] == 2 and [m["rank"] for m in d["map"]] == [0, 1]
        assert [m["pci_bus_id"] for m in d["map"]] == ["0000:05:00.0", "0000:06:00.0"]
    res = _run2(DEVMAP_WORKER, {"SHARED": "1"})
    for d in res:
        assert "refused" in d and "distinct" not in d and d["wrapped"] == 1
