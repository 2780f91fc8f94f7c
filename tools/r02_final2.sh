# round-2 closing refresh: full GPU suite, smoke, every bench line with CPU baselines, PLL A/B, rocprof c5 + fused
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/final2
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu_full.txt 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 120 python -u tools/pll_spec_ab.py > $O/ab.txt 2>&1
timeout -k 10 240 python bench.py > $O/bench_default.json 2> $O/bench_default.err
timeout -k 10 240 python bench.py --iq u8 > $O/bench_u8.json 2> $O/bench_u8.err
for w in c3 c4 c5; do
  timeout -k 10 240 python bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
done
timeout -k 10 200 python3 bench.py --workload c5 --streams 64 --steps 64 --no-cpu > $O/bench_c5_s64.json 2> $O/bench_c5_s64.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --no-cpu --steps 64 > $O/prof_c5.json 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -o fused -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --steps 20 > $O/prof_default.json 2>&1
