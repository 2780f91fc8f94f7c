# PLL / span iteration: PLL / span / receiver / offset tests, C5 span bench (8 and 1 streams),
# the spec kernel's phase timers (diagnostic build libsdr_prof.so)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_it
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_span.py tests/test_pll_spec.py tests/test_receiver.py tests/test_offsets.py tests/test_dropin.py > $O/pytest.txt 2>&1
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_s8.json 2> $O/c5_s8.err
timeout -k 10 200 python -u bench.py --workload c5 --streams 1 --no-cpu > $O/c5_s1.json 2> $O/c5_s1.err
SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_prof.so timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu --steps 2 --warmup 1 > $O/prof.txt 2> $O/prof.err
