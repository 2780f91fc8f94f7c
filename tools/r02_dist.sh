#!/bin/bash
# r02: multi-stream C-ABI tests, then two ranks on the one GPU (device wrap) for the mono and c5 benches
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_multistream_capi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ms.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_dist_mono.json 2> gpurun_out/bench_dist_mono.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --workload c5 --steps 64 --warmup 5 > gpurun_out/bench_dist_c5.json 2> gpurun_out/bench_dist_c5.err
