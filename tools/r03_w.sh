# r03: spec warm-up length variants (libsdr_w*.so) on the long-call tests and the S8 K256 span
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_w
mkdir -p $O
cd $GRAFT_REPO_ROOT
P=$GRAFT_REPO_ROOT/real-time-software-defined-radio_amd
for v in w0 w16 w32; do
  timeout -k 10 200 env SDR_LIB=$P/libsdr_$v.so python -u -m pytest -x -q -s --timeout 150 --timeout-method thread -m gpu tests/test_pll_spec.py tests/test_span.py > $O/pytest_$v.txt 2>&1
  timeout -k 10 120 env SDR_LIB=$P/libsdr_$v.so python -u tools/long_diag.py 8 256 3 1 > $O/diag_$v.txt 2>&1
done
timeout -k 10 120 python -u tools/long_diag.py 8 256 3 1 > $O/diag_w64.txt 2>&1
timeout -k 10 120 env SDR_LIB=$P/libsdr_dbg.so python -u tools/long_diag.py 8 256 2 1 > $O/diag_prof.txt 2>&1
