set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pll.log 2>&1
timeout -k 10 240 python3 tools/bench_configs.py > gpurun_out/bench_configs2.json 2> gpurun_out/bench_configs2.err
