#!/bin/bash
# HIP API timing of the per-block c4 / c3 workloads (rocprofv3 HIP runtime trace + stats):
# where the host's time per block goes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b_api
mkdir -p "$O"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d "$O/c4" -o c4 \
  -- python3 "$R/bench.py" --workload c4 --no-cpu --steps 200 > "$O/c4.json" 2> "$O/c4.err" || exit $?
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats --output-format csv -d "$O/c3" -o c3 \
  -- python3 "$R/bench.py" --workload c3 --no-cpu --steps 200 > "$O/c3.json" 2> "$O/c3.err" || exit $?
ls -R "$O" | head -40
