# r03 iteration: receiver/PLL/span/offset/live tests, c5 benches (block mode 64 streams, S8 span), c5 span rocprof
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_iter13
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_pll_spec.py tests/test_span.py tests/test_offsets.py tests/test_receiver.py tests/test_dropin.py tests/test_live.py > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/bench_b64.json 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/bench_s8.json 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --streams 8 --span 256 --steps 5 --warmup 2 --no-cpu > $O/prof_c5.json 2>&1
