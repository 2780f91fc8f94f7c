#!/bin/bash
# Round-4b final check of the tree (run under gpurun from the repo root): the -m gpu suite and
# smoke, the receiver's event trimming A/B on c3 / c4 (libsdr_prev.so = the tree before it),
# then the default bench line.  The first failure ends the call.
set -e
O=gpurun_out/r04b_final
bash tools/gpu_round.sh $O tests
bash tools/ab_bench.sh $O/ab_c4 3 "--workload,c4,--no-cpu" prev prod
bash tools/ab_bench.sh $O/ab_c3 3 "--workload,c3,--no-cpu" prev prod
bash tools/gpu_round.sh $O bench
