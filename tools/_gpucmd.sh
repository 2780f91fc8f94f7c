set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_u8f.log 2>&1
timeout -k 10 120 python3 bench.py --no-cpu --iq u8 > gpurun_out/bench_u8f.json
