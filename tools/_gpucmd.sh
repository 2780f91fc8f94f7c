# scratch GPU command: the full GPU suite + smoke, the default bench line, the C5 span trace
set -e
bash tools/gpu_round.sh gpurun_out/r04a tests bench prof:c5s8:--workload,c5,--streams,8,--span,256,--steps,5,--warmup,2,--no-cpu
