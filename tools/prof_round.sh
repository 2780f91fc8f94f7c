#!/bin/bash
# usage (on the GPU box, repo root): tools/prof_round.sh <round-tag>
# 1) kernel-trace --stats of the bench (both paths)   -> gpurun_out/prof_<tag>_{split,fused}/
# 2) HBM traffic counters, one counter group per pass  -> gpurun_out/pmc_<tag>_{path}_{fetch,write}/
# Each GPU step has its own time limit; the chain stops at the first failure.
set -e
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for path in split fused; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${tag}_${path} -o prof --output-format csv \
    -- python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --path $path > $R/gpurun_out/prof_${tag}_${path}.json
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_${tag}_${path}_fetch -o pmc --output-format csv \
    -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 --path $path > /dev/null
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_${tag}_${path}_write -o pmc --output-format csv \
    -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 --path $path > /dev/null
done
