#!/bin/bash
# r02 full refresh: GPU suite, smoke, every bench line (with CPU baselines), kernel traces of c5 / c3
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
for w in c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
done
timeout -k 10 200 python3 bench.py --workload c5 --streams 64 --steps 64 --no-cpu > gpurun_out/bench_c5_s64.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o prof --output-format csv \
  -- python3 $R/bench.py --workload c5 --steps 64 --no-cpu > $R/gpurun_out/prof_c5.json
