# u8 fused FE + mono A/B: image loads in flight (SDR_FE_MFMA_DEPTH) x waves per CU cap (SDR_FE_MFMA_WPC)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_u8ab
mkdir -p $O
cd $R
for d in 1 2; do for w in 8 12; do
  SDR_FE_MFMA_DEPTH=$d SDR_FE_MFMA_WPC=$w timeout -k 10 120 python bench.py --iq u8 --blocks 128 --no-cpu --no-extras --steps 50 --warmup 10 > $O/u8_d${d}_w${w}.json 2> $O/u8_d${d}_w${w}.err
done; done
