# r03: PLL solver counters, long calls, spans, offset sweep; then the c4 PLL-stage trace
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_pll
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_pll_spec.py > $O/pytest_pll.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -m gpu tests/test_receiver.py tests/test_span.py > $O/pytest_rx_span.txt 2>&1
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread -m gpu tests/test_offsets.py > $O/pytest_offsets.txt 2>&1
