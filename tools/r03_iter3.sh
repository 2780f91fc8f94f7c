set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_iter3
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_pll_spec.py tests/test_span.py tests/test_receiver.py tests/test_dropin.py > $O/pytest.txt 2>&1
timeout -k 10 120 python -u tools/long_diag.py 8 256 3 1 > $O/diag_s8_k256.txt 2>&1
SDR_LIB=$GRAFT_REPO_ROOT/real-time-software-defined-radio_amd/libsdr_dbg.so timeout -k 10 120 python -u tools/long_diag.py 1 256 2 1 > $O/diag_dbg.txt 2>&1
bash tools/r03_pmc.sh
