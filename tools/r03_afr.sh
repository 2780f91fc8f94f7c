# u8 MFMA mono kernel iteration: u8 parity tests, u8 bench (twice), waves-per-CU sweep
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_u8it
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "u8 or mfma or mono" > $O/pytest.txt 2>&1
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 50 --warmup 10"
timeout -k 10 120 python bench.py $A > $O/u8_1.json 2> $O/u8_1.err
timeout -k 10 120 python bench.py $A > $O/u8_2.json 2> $O/u8_2.err
for w in 8 10; do SDR_FE_MFMA_WPC=$w timeout -k 10 120 python bench.py $A > $O/u8_w$w.json 2> $O/u8_w$w.err; done
