# round-3 closing set, part C: SQ / TCC counter passes on C5 block mode at 64 streams
# (rx_stage_kernel<151>, fe_slot_kernel, pll_spec_kernel<512,false>), the S8 span
# (fe_mfma_demod_kernel, pll_spec_kernel<512,true>) and the u8 MFMA mono kernel
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${R03_OUT:-r03_final}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B64="--workload c5 --streams 64 --span 1 --no-pipeline --steps 20 --warmup 5"
SPN="--workload c5 --streams 8 --span 64 --steps 3 --warmup 1"
U8="--iq u8 --blocks 128 --no-extras --steps 20 --warmup 5"
for tag in b64 span u8; do
  case $tag in b64) A="$B64";; span) A="$SPN";; u8) A="$U8";; esac
  timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU \
    -d $O/pmc_${tag}_a -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM \
    -d $O/pmc_${tag}_b -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_BUSY_CYCLES \
    -d $O/pmc_${tag}_c -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1 || echo "pass c failed" > $O/pmc_${tag}_c.err
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${tag}_fetch -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${tag}_write -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $A > /dev/null 2>&1
done
