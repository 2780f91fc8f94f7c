#!/bin/bash
# Final check with the PLL on its own stream by default (pipelined receivers): the -m gpu suite
# and smoke, the c4 and live A/Bs against SDR_RX_PLL_STREAM=0 (the previous rule for one or two
# recurrences), then the default line.  The first failure ends the call.
set -e
O=gpurun_out/r04c_pll
bash tools/gpu_round.sh $O tests
tail -1 $O/pytest_gpu.txt
bash tools/ab_bench.sh $O/ab_c4 4 "--workload,c4,--no-cpu,--steps,3000,--warmup,200" SDR_RX_PLL_STREAM=0 prod
bash tools/ab_bench.sh $O/ab_live 3 "--workload,live,--no-cpu" SDR_RX_PLL_STREAM=0 prod
python3 tools/ab_summary.py $O/ab_c4 $O/ab_live
bash tools/gpu_round.sh $O bench
