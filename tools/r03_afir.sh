# u8 MFMA mono kernel: deferred audio stores (product) vs immediate stores (libsdr_afir0, the
# previous build)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_q
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "u8 or mfma or mono" > $O/pytest.txt 2>&1
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 50 --warmup 10"
timeout -k 10 120 python bench.py $A > $O/prod.json 2> $O/prod.err
SDR_FE_MFMA_DEPTH=1 SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_afir0.so timeout -k 10 120 python bench.py $A > $O/prev.json 2> $O/prev.err
timeout -k 10 120 python bench.py $A > $O/prod2.json 2> $O/prod2.err
for w in 8 10; do SDR_FE_MFMA_WPC=$w timeout -k 10 120 python bench.py $A > $O/prod_w$w.json 2> $O/prod_w$w.err; done
