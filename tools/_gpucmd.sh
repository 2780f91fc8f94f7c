set -e
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --kernel-trace -d $R/gpurun_out/clk -o clk --output-format csv -- $R/tools/ab_tune 2 fused > $R/gpurun_out/clk.log 2>&1
