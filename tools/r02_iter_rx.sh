#!/bin/bash
# r02: receiver tests, the three receiver bench lines, a kernel trace of c3 (each step time-limited)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_receiver.py tests/test_gpu_parity.py tests/test_live.py tests/test_rds_link.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rx.log 2>&1
for w in c3 c4 c5; do
  timeout -k 10 240 python3 bench.py --workload $w --no-cpu > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o prof --output-format csv \
  -- python3 $R/bench.py --workload c3 --steps 100 --no-cpu > $R/gpurun_out/prof_c3.json
