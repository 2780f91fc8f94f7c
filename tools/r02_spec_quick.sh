# parallel PLL solve variant: its tests, A/B, c4/c5 lines
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/specq
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pll_spec.py tests/test_receiver.py > $O/pytest_spec.txt 2>&1
timeout -k 10 120 python -u tools/pll_spec_ab.py > $O/ab.txt 2>&1
for w in c4 c5; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err
done
timeout -k 10 200 python3 bench.py --workload c5 --streams 64 --steps 64 --no-cpu > $O/bench_c5_s64.json 2> $O/bench_c5_s64.err
