#!/bin/bash
# Round-4b GPU call: the PLL bisection (tools/gpu_bisect_r04b.sh), the -m gpu suite, then
# interleaved A/Bs of this round's changes (headline prologue, PLL step loops, receiver
# submission depth).  A test FAILURE (pytest rc 1) does not stop the A/Bs; anything else (a
# fault, an abort, a time limit) ends the call.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
bash tools/gpu_bisect_r04b.sh || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.txt" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.txt"
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
set -e
bash tools/ab_bench.sh gpurun_out/r04b/ab_ring 3 "--no-extras,--no-cpu" base prod q16
bash tools/ab_bench.sh gpurun_out/r04b/ab_c5 2 "--workload,c5,--steps,5,--no-cpu" base prod nofast oldcorr
bash tools/ab_bench.sh gpurun_out/r04b/ab_c4 2 "--workload,c4,--no-cpu" base prod
bash tools/ab_bench.sh gpurun_out/r04b/ab_c4d1 2 "--workload,c4,--no-cpu,--depth,1" base prod
bash tools/ab_bench.sh gpurun_out/r04b/ab_c3 2 "--workload,c3,--no-cpu" prod
bash tools/ab_bench.sh gpurun_out/r04b/ab_c3d1 2 "--workload,c3,--no-cpu,--depth,1" prod
bash tools/ab_bench.sh gpurun_out/r04b/ab_c5b64 2 "--workload,c5,--streams,64,--span,1,--steps,20,--warmup,5,--no-cpu" base prod
