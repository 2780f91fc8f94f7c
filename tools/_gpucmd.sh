set -e
mkdir -p gpurun_out
timeout -k 10 120 tools/ab_tune 6 > gpurun_out/ab_slot3.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_slot3.log 2>&1
timeout -k 10 120 python3 bench.py --no-cpu > gpurun_out/bench_slot3.json
timeout -k 10 120 python3 bench.py --no-cpu --path split > gpurun_out/bench_slot3_split.json
