# r03: u8 MFMA kernels after the LDS halo carry: tests, u8 bench (128 blocks), FETCH pass, c5 S8
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_u8b
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
timeout -k 10 300 python3 bench.py --iq u8 --blocks 128 --no-cpu --no-extras > $O/bench_u8.json 2> $O/bench_u8.err
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/bench_s8.json 2>&1
export TMPDIR=/tmp
cd /tmp
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 20 --warmup 5 --settle-ms 0"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py $A > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- python3 $R/bench.py $A > /dev/null 2>&1
cd $R
for w in 6 8 10; do
  SDR_FE_MFMA_WPC=$w timeout -k 10 200 python3 bench.py --iq u8 --blocks 128 --no-cpu --no-extras > $O/bench_u8_wpc$w.json 2>> $O/bench_u8.err
done
