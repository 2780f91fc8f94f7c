#!/bin/bash
# r02 iteration: GPU tests, then the bench on both paths (each step time-limited; stop at the first failure)
set -e
tag=${1:-it}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1
timeout -k 10 120 python3 bench.py --no-cpu > gpurun_out/bench_${tag}_fused.json
timeout -k 10 120 python3 bench.py --no-cpu --path split > gpurun_out/bench_${tag}_split.json
