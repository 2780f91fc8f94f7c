#!/bin/bash
# r02: the headline at 128 blocks per step: bench (default), kernel traces + FETCH/WRITE passes
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 200 python3 bench.py --no-cpu --path split > gpurun_out/bench_split.json
bash tools/prof_round.sh r02b
