# phase timers of pll_spec_kernel<512, LONG> in a C5 span (diagnostic build libsdr_prof.so)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_specprof
mkdir -p $O
cd $R
SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_prof.so timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu --steps 2 --warmup 1 > $O/c5.json 2> $O/c5.err
grep spec_prof $O/c5.err | tail -200 > $O/spec_prof.txt || true
