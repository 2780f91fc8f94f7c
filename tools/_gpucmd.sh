set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_final.log 2>&1
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/smoke_final.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err
timeout -k 10 900 bash tools/prof_round.sh v5 > gpurun_out/prof_v5.log 2>&1
