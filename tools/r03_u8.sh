# r03: the u8 FE + mono MFMA kernel (128 blocks) -- bench, kernel trace, SQ counters; copy / read probes
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_u8
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --iq u8 --blocks 128 --no-cpu --no-extras > $O/bench_u8.json 2> $O/bench_u8.err
export TMPDIR=/tmp
cd /tmp
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 20 --warmup 5 --settle-ms 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o tr -- python3 $R/bench.py $A > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VALU -d $O/pmc_a -o pmc --output-format csv -- python3 $R/bench.py $A > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $O/pmc_b -o pmc --output-format csv -- python3 $R/bench.py $A > /dev/null 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $R/bench.py $A > /dev/null 2>&1
