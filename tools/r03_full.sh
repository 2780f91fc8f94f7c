# r03: the whole GPU suite, then the c5 benches (block 64, S8 span, 1 stream) and a c5 span rocprof
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_full2
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/bench_b64.json 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/bench_s8.json 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 1 --no-cpu > $O/bench_s1.json 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --streams 8 --span 256 --steps 5 --warmup 2 --no-cpu > $O/prof_c5.json 2>&1
