# r03: C5 block mode at 64 streams, not pipelined: per-launch kernel trace (rx_stage tile shapes)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_b64
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_receiver.py tests/test_span.py tests/test_gpu_parity.py tests/test_live.py > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/bench_b64.json 2>&1
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 $R/bench.py --no-cpu --no-pipeline --workload c5 --streams 64 --span 1 --steps 20 --warmup 5 > $O/bench_b64_nopipe.json 2> $O/trace.err
