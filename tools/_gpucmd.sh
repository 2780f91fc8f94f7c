set -e
mkdir -p gpurun_out/r04_base
O=gpurun_out/r04_base
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
