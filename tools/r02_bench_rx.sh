#!/bin/bash
# r02: bench lines for the receiver workloads, then a kernel-trace profile of c5
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
for w in c3 c4 c5; do
  timeout -k 10 240 python3 bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
done
timeout -k 10 120 python3 bench.py --workload c5 --streams 64 --steps 64 --no-cpu > gpurun_out/bench_c5_s64.json 2>> gpurun_out/bench_c5.err
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o prof --output-format csv \
  -- python3 $R/bench.py --workload c5 --steps 64 --no-cpu > $R/gpurun_out/prof_c5.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o prof --output-format csv \
  -- python3 $R/bench.py --workload c3 --steps 100 --no-cpu > $R/gpurun_out/prof_c3.json
