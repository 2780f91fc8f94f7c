set -e
O=$GRAFT_REPO_ROOT/gpurun_out/qf
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/pll_probe > $O/pll_probe.log 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_receiver.py tests/test_multistream_capi.py tests/test_live.py tests/test_gpu_parity.py tests/test_dropin.py > $O/pytest.txt 2>&1
for w in c4 c5; do timeout -k 10 200 python bench.py --workload $w --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err; done
timeout -k 10 200 python bench.py --workload c5 --no-cpu --streams 64 > $O/bench_c5_s64.json 2> $O/bench_c5_s64.err
