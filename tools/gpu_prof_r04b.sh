#!/bin/bash
# The per-block solve's phase timers (libsdr_prof.so: tools/build_dbg.sh prof -DSDR_PLL_SPEC_PROF;
# diagnostic, never the product) on the c4 and C5-span workloads.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b_prof
mkdir -p "$O"
cd "$R"
L=$R/real-time-software-defined-radio_amd/libsdr_prof.so
SDR_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --no-cpu --steps 20 > $O/c4.json 2> $O/c4.err || exit $?
SDR_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --steps 5 --warmup 2 --no-cpu > $O/c5b64.json 2> $O/c5b64.err || exit $?
grep -c spec_prof $O/c4.json $O/c5b64.json
