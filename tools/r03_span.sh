# r03: drift-aware guess (offset sweep), span benches, c4 PLL-stage trace
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_span
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_pll_spec.py tests/test_receiver.py tests/test_dropin.py tests/test_multistream_capi.py > $O/pytest_pll.txt 2>&1
timeout -k 10 400 python -u -m pytest -v -s --timeout 200 --timeout-method thread -m gpu tests/test_offsets.py tests/test_span.py > $O/pytest_offsets.txt 2>&1 || true
timeout -k 10 300 python -u bench.py --workload c5 --streams 8 --span 256 --steps 5 --warmup 2 --no-cpu > $O/bench_c5_s8.json 2> $O/bench_c5_s8.err
timeout -k 10 300 python -u bench.py --workload c5 --streams 1 --span 256 --steps 10 --warmup 2 --no-cpu > $O/bench_c5_s1.json 2> $O/bench_c5_s1.err
timeout -k 10 300 python -u bench.py --workload c4 --no-cpu > $O/bench_c4.json 2> $O/bench_c4.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --streams 8 --span 256 --steps 5 --warmup 2 --no-cpu > $O/prof_c5.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --no-cpu --steps 50 > $O/prof_c4.json 2>&1
