# r03: SQ / TCC counters on the C5 span receiver's kernels, separate passes
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_run.sh c5span --workload c5 --streams 8 --span 64
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_c5span_fetch -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 --workload c5 --streams 8 --span 64 > /dev/null
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_c5span_write -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 --workload c5 --streams 8 --span 64 > /dev/null
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_c5span_c -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 --workload c5 --streams 8 --span 64 > /dev/null
