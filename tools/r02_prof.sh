#!/bin/bash
# r02 headline profile: default bench, kernel-trace stats of both paths, FETCH_SIZE / WRITE_SIZE
# passes (one counter group per run), each step time-limited
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
timeout -k 10 120 python3 bench.py --no-cpu --path split > gpurun_out/bench_split.json
timeout -k 10 120 python3 bench.py --no-cpu --iq u8 > gpurun_out/bench_u8.json
bash tools/prof_round.sh r02
