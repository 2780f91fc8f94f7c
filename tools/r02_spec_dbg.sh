set -e
O=$GRAFT_REPO_ROOT/gpurun_out/specdbg
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 env SDR_PLL_SPEC_DEBUG=1 python -u tools/pll_spec_ab.py > $O/ab_256.txt 2>&1
cp tools/_alt/libsdr.so real-time-software-defined-radio_amd/libsdr.so
timeout -k 10 120 env SDR_PLL_SPEC_DEBUG=1 python -u tools/pll_spec_ab.py > $O/ab_512.txt 2>&1
