#!/bin/bash
# SQ counters of the ablation harness and the morph probe (two passes each, --pmc only)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_ab_$1
mkdir -p $O
export TMPDIR=/tmp AB_QUICK=1
cd /tmp
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM"
B="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
timeout -s KILL 120 rocprofv3 --pmc $A -d $O/ra -o pmc --output-format csv -- $R/tools/ring_ab > /dev/null
timeout -s KILL 120 rocprofv3 --pmc $B -d $O/rb -o pmc --output-format csv -- $R/tools/ring_ab > /dev/null
timeout -s KILL 120 rocprofv3 --pmc $A -d $O/ma -o pmc --output-format csv -- $R/tools/morph_probe > /dev/null
timeout -s KILL 120 rocprofv3 --pmc $B -d $O/mb -o pmc --output-format csv -- $R/tools/morph_probe > /dev/null
