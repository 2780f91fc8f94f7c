#!/bin/bash
# usage (on the GPU box, repo root): tools/gpu_check.sh <tag> [pytest-args...]
# GPU parity tests, then the bench (both paths), then a kernel-trace --stats profile of
# each path.  Every GPU step has its own time limit; the chain stops at the first failure.
set -e
tag=$1; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
  > $O/pytest_gpu_$tag.log 2>&1
timeout -k 10 180 python3 bench.py > $O/bench_$tag.json
timeout -k 10 120 python3 bench.py --no-cpu --path split > $O/bench_${tag}_split.json
SDR_FE_KERNEL=circ timeout -k 10 120 python3 bench.py --no-cpu > $O/bench_${tag}_circ.json
export TMPDIR=/tmp
cd /tmp
for path in fused split; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_${tag}_${path} -o prof --output-format csv \
    -- python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --path $path > $O/prof_${tag}_${path}.json
done
