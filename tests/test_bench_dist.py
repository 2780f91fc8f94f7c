"""bench.py's N>1 path on CPU: world_size-2 gloo ranks exercise dist_setup, the barrier
and the max-over-ranks reduction that bench.py's timed region uses (no GPU, no RCCL:
the data path has no collective)."""
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
