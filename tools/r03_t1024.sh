# per-block PLL solve with 1 024 threads: PLL / receiver / offset tests, C5 per-block lines
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_t1024
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_offsets.py tests/test_pll_spec.py tests/test_receiver.py tests/test_dropin.py tests/test_span.py tests/test_live.py > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/c5b64.json 2> $O/c5b64.err
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --span 1 --no-cpu > $O/c5b8.json 2> $O/c5b8.err
