set -e
bash tools/gpu_round.sh gpurun_out/r04a tests bench
