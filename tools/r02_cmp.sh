#!/bin/bash
# harness vs bench on one box: ring ablation harness, then the bench's split path under a kernel trace
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 120 $R/tools/ring_ab > $R/gpurun_out/ring_ab_$1.log 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$1_split -o prof --output-format csv \
  -- python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --path split > $R/gpurun_out/prof_$1_split.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$1_fused -o prof --output-format csv \
  -- python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --path fused > $R/gpurun_out/prof_$1_fused.json
