#!/bin/bash
# usage (on the GPU box): tools/pmc_run.sh <tag> <bench args...>
# Two SQ counter passes (separate rocprofv3 runs, --pmc only with --kernel-trace-free
# collection) over a short bench run; CSVs land in gpurun_out/pmc_<tag>_{a,b}.
set -e
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  -d $R/gpurun_out/pmc_${tag}_a -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 "$@" > /dev/null
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_VMEM \
  -d $R/gpurun_out/pmc_${tag}_b -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 5 --warmup 2 --settle-ms 0 "$@" > /dev/null
