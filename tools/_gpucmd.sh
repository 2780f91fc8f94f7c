set -e
mkdir -p gpurun_out
timeout -k 10 150 tools/ab_tune 8 > gpurun_out/ab_slotdma.log 2>&1
