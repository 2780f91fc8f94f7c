# round-3 closing set, part A: full GPU suite, offsets table, smoke, every bench line with CPU baselines
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${R03_OUT:-r03_final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu_full.txt 2>&1
timeout -k 10 200 python -u -m pytest -s -q --timeout 200 --timeout-method thread tests/test_offsets.py > $O/offsets.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err
for w in c3 c4; do
  timeout -k 10 240 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
done
timeout -k 10 200 python bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/bench_c5_b64.json 2> $O/bench_c5_b64.err
