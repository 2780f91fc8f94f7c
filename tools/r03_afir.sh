# u8 MFMA mono kernel: software-pipelined tiles (product build) vs the plain loop (libsdr_pipe0)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_pipe
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "u8 or mfma or mono" > $O/pytest.txt 2>&1
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 50 --warmup 10"
timeout -k 10 120 python bench.py $A > $O/pipe.json 2> $O/pipe.err
SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_pipe0.so timeout -k 10 120 python bench.py $A > $O/plain.json 2> $O/plain.err
for w in 8 10 16; do SDR_FE_MFMA_WPC=$w timeout -k 10 120 python bench.py $A > $O/pipe_w$w.json 2> $O/pipe_w$w.err; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_span.py tests/test_pll_spec.py tests/test_receiver.py > $O/pytest_pll.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_s8.json 2> $O/c5_s8.err
