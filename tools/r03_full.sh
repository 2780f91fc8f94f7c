# r03: full GPU suite, default bench (headline + c5 + u8 extras), c5 span rocprof
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_full
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu_full.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --streams 8 --span 256 --steps 5 --warmup 2 --no-cpu > $O/prof_c5.json 2>&1
