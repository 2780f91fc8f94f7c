# r03 iteration: GPU suite, u8 bench (128 blocks), c5 benches (block 64, S8 span, 1 stream)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r03_iter14
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --iq u8 --blocks 128 --no-cpu --no-extras > $O/bench_u8.json 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/bench_b64.json 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/bench_s8.json 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 1 --no-cpu > $O/bench_s1.json 2>&1
