#!/bin/bash
# Round-4b closing set on the final tree (run under gpurun from the repo root).
#   bash tools/gpu_close_r04b.sh a   tests, smoke, the default bench line, C5 per block at 64
#                                    streams, the live pipeline, rocprofv3 --kernel-trace --stats
#   bash tools/gpu_close_r04b.sh b   FETCH_SIZE / WRITE_SIZE passes and the PLL SQ passes
# Each step has its own time limit (tools/gpu_round.sh); the first failure ends the call.
set -e
O=gpurun_out/r04b_close
case "$1" in
  a)
    bash tools/gpu_round.sh $O tests bench \
      bench:c5b64:--workload,c5,--streams,64,--span,1,--steps,20,--warmup,5 bench:live:--workload,live \
      prof:fused:--no-extras,--no-cpu,--steps,20 prof:u8:--iq,u8,--no-extras,--no-cpu,--steps,20 \
      prof:c5s8:--workload,c5,--steps,5,--no-cpu prof:c4:--workload,c4,--no-cpu,--steps,100 \
      prof:c3:--workload,c3,--no-cpu,--steps,100 \
      prof:c5b64:--workload,c5,--streams,64,--span,1,--steps,20,--warmup,5,--no-cpu ;;
  b)
    bash tools/gpu_round.sh $O \
      pmc:fused_fetch:FETCH_SIZE:--no-extras,--steps,10 pmc:fused_write:WRITE_SIZE:--no-extras,--steps,10 \
      pmc:u8_fetch:FETCH_SIZE:--iq,u8,--no-extras,--steps,10 pmc:u8_write:WRITE_SIZE:--iq,u8,--no-extras,--steps,10 \
      pmc:c5_fetch:FETCH_SIZE:--workload,c5,--steps,3 pmc:c5_write:WRITE_SIZE:--workload,c5,--steps,3 \
      pmc:pll_a:SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVES:--workload,c5,--steps,3 \
      pmc:pll_b:SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VMEM,SQ_LDS_BANK_CONFLICT:--workload,c5,--steps,3 ;;
  *)
    echo "usage: gpu_close_r04b.sh a|b" >&2; exit 2 ;;
esac
