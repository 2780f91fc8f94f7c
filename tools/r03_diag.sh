set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_diag4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pll_spec.py tests/test_span.py > $O/pytest.txt 2>&1
timeout -k 10 120 python -u tools/long_diag.py 1 64 3 1 > $O/diag_s1_k64.txt 2>&1
SDR_LIB=$GRAFT_REPO_ROOT/real-time-software-defined-radio_amd/libsdr_dbg.so timeout -k 10 120 python -u tools/long_diag.py 1 256 2 1 > $O/diag_dbg_k256.txt 2>&1
timeout -k 10 120 python -u tools/long_diag.py 8 256 3 1 > $O/diag_s8_k256.txt 2>&1
