#!/bin/bash
# u8 mono kernel A/B: the A fragments from an L1-resident table at 4 waves per SIMD
# (libsdr_afrl1.so, -DSDR_FE_MFMA_AFR_L1=1) against the product; the u8 MFMA parity tests on
# the variant first.  Each step has its own limit; the first failure ends the call.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/afr
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_afrl1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
  -m gpu -k "u8" -v --timeout 120 --timeout-method thread > "$O/pytest_afrl1.txt" 2>&1
tail -2 "$O/pytest_afrl1.txt"
bash tools/ab_bench.sh gpurun_out/afr/ab_u8 3 "--iq,u8,--no-extras,--no-cpu" prod afrl1 "${@}"
python3 tools/ab_summary.py gpurun_out/afr/ab_u8
