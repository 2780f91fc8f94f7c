# parallel PLL solve: new tests, A/B, full GPU suite, c4/c5 bench lines with it on and off
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/spec
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_pll_spec.py > $O/pytest_spec.txt 2>&1
timeout -k 10 120 env SDR_PLL_SPEC=0 python -u tools/pll_spec_ab.py > $O/ab.txt 2>&1
timeout -k 10 120 python -u tools/pll_spec_ab.py >> $O/ab.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu_full.txt 2>&1
for w in c4 c5; do
  timeout -k 10 240 python bench.py --workload $w --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err
  timeout -k 10 240 env SDR_PLL_SPEC=0 python bench.py --workload $w --no-cpu > $O/bench_${w}_seq.json 2> $O/bench_${w}_seq.err
done
timeout -k 10 200 python3 bench.py --workload c5 --streams 64 --steps 64 --no-cpu > $O/bench_c5_s64.json 2> $O/bench_c5_s64.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --no-cpu --steps 64 > $O/prof_c5.json 2>&1
