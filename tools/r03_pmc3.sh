# r03: kernel traces + SQ / TCC counter passes on the current kernels:
# C5 block mode at 64 streams (rx_stage_kernel<151>, fe_slot_kernel, pll_spec_kernel<512,false>)
# and the S8 span (pll_spec_kernel<512,true>); then the default bench line
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_pmc3
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B64="--workload c5 --streams 64 --span 1 --steps 20 --warmup 5"
SPN="--workload c5 --streams 8 --span 64 --steps 3 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_b64 -o tr -- python3 $R/bench.py --no-cpu --no-pipeline $B64 > $O/bench_b64.json 2> $O/trace_b64.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_span -o tr -- python3 $R/bench.py --no-cpu $SPN > $O/bench_span.json 2> $O/trace_span.err
for tag in b64 span; do
  if [ $tag = b64 ]; then A="--no-pipeline $B64"; else A="$SPN"; fi
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    -d $O/pmc_${tag}_a -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM \
    -d $O/pmc_${tag}_b -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F16 \
    -d $O/pmc_${tag}_c -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1 || echo "pass c failed" > $O/pmc_${tag}_c.err
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${tag}_fetch -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${tag}_write -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
done
cd $R
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err
