# scratch GPU command 2: A/B of the per-block PLL split, PLL counters, live pipeline, rocprof stats
set -e
O=gpurun_out/r04b
C5S8=--workload,c5,--streams,8,--span,256,--steps,5,--warmup,2,--no-cpu
bash tools/gpu_round.sh $O bench:c5s8:$C5S8 bench:c4:--workload,c4,--no-cpu bench:c5b64:--workload,c5,--streams,64,--span,1,--no-pipeline,--steps,20,--warmup,5,--no-cpu
SDR_PLL_SPLIT=0 bash tools/gpu_round.sh $O/nosplit bench:c4:--workload,c4,--no-cpu bench:c5b64:--workload,c5,--streams,64,--span,1,--no-pipeline,--steps,20,--warmup,5,--no-cpu
bash tools/gpu_round.sh $O pmc:pll_a:SQ_INSTS_VALU,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVES:$C5S8
bash tools/gpu_round.sh $O pmc:pll_b:SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VMEM,SQ_LDS_BANK_CONFLICT:$C5S8
bash tools/gpu_round.sh $O bench:c3:--workload,c3,--no-cpu prof:c3:--workload,c3,--no-cpu,--steps,50
bash tools/gpu_round.sh $O bench:live:--workload,live,--span,256,--live-repeat,4
