# u8 MFMA demod kernel (receivers' FE) reordered: full GPU suite, C5 spans and per-block
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_dm
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_s8.json 2> $O/c5_s8.err
timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/c5_b64.json 2> $O/c5_b64.err
