# u8 MFMA demod kernel with non-temporal demod stores: receiver tests, C5 spans and per-block
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_nt
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_receiver.py tests/test_span.py tests/test_gpu_parity.py tests/test_live.py > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_s8.json 2> $O/c5_s8.err
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/c5_b64.json 2> $O/c5_b64.err
