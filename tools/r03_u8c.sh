# r03: u8 MFMA mono kernel with two tiles of image loads in flight (DEPTH 2) -- tests, A/B vs
# DEPTH 1, waves-per-CU sweep, HBM traffic passes, c5 S8
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_u8c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
A="--iq u8 --blocks 128 --no-cpu --no-extras"
timeout -k 10 200 python3 bench.py $A > $O/bench_u8_d2.json 2> $O/bench_u8.err
SDR_FE_MFMA_DEPTH=1 timeout -k 10 200 python3 bench.py $A > $O/bench_u8_d1.json 2>> $O/bench_u8.err
for w in 8 10; do
  SDR_FE_MFMA_WPC=$w timeout -k 10 200 python3 bench.py $A > $O/bench_u8_d2_wpc$w.json 2>> $O/bench_u8.err
  SDR_FE_MFMA_DEPTH=1 SDR_FE_MFMA_WPC=$w timeout -k 10 200 python3 bench.py $A > $O/bench_u8_d1_wpc$w.json 2>> $O/bench_u8.err
done
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/bench_s8.json 2>&1
export TMPDIR=/tmp
cd /tmp
B="$A --steps 20 --warmup 5 --settle-ms 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 $R/bench.py $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py $B > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 $R/bench.py $B > /dev/null 2>&1
