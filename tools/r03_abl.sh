# u8 MFMA mono kernel: parity tests of the product build, then the ablation builds' launch times
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_abl
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "u8 or mfma or mono" > $O/pytest.txt 2>&1
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 50 --warmup 10"
timeout -k 10 120 python bench.py $A > $O/prod.json 2> $O/prod.err
SDR_FE_MFMA_DEPTH=1 timeout -k 10 120 python bench.py $A > $O/prod_d1.json 2> $O/prod_d1.err
for m in 1 2 4 8 24 3; do
  SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_abl$m.so timeout -k 10 120 python bench.py $A > $O/abl$m.json 2> $O/abl$m.err
done
