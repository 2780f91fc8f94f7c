#!/bin/bash
# r02: split-stream parity test, then the split-stream bench on 1 and 2 ranks (one GPU)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k split -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_split.log 2>&1
timeout -k 10 300 python3 bench.py --split-stream --no-cpu > gpurun_out/bench_split1.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --split-stream --steps 20 --warmup 5 > gpurun_out/bench_split2.json 2> gpurun_out/bench_split2.err
