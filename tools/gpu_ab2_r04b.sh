#!/bin/bash
# Round-4b second A/B: the per-block solve's warm-up (SDR_SPEC_W 32 -> 16) and thread count
# (256 -> 512 threads for c4's 5 120-step blocks), each variant's PLL tests first.  A test
# failure does not stop the script; anything else (a fault, an abort, a time limit) ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b_ab2
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for v in w16 t512 w16t512; do
  SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_$v.so timeout -k 10 300 python -u -m pytest \
    tests/test_pll_spec.py tests/test_offsets.py tests/test_receiver.py tests/test_span.py -m gpu -q \
    --timeout 200 --timeout-method thread > "$O/pytest_$v.txt" 2>&1
  rc=$?
  echo "$v: rc $rc $(tail -1 $O/pytest_$v.txt)"
  [ $rc -le 1 ] || exit $rc
done
set -e
bash tools/ab_bench.sh gpurun_out/r04b_ab2/ab_c4 3 "--workload,c4,--no-cpu" prod w16 t512 w16t512
bash tools/ab_bench.sh gpurun_out/r04b_ab2/ab_c5b64 2 "--workload,c5,--streams,64,--span,1,--steps,20,--warmup,5,--no-cpu" prod w16
