# r03: kernel trace + SQ / TCC counter passes for the receiver kernels:
# C5 block mode at 64 streams (rx_stage_kernel, fe_slot_kernel) and the S8 span (pll_spec_kernel)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_pmc2
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
B64="--workload c5 --streams 64 --span 1 --steps 20 --warmup 5"
SPN="--workload c5 --streams 8 --span 64 --steps 3 --warmup 1"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_b64 -o tr -- python3 $R/bench.py --no-cpu $B64 > $O/bench_b64.json 2> $O/trace_b64.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_span -o tr -- python3 $R/bench.py --no-cpu $SPN > $O/bench_span.json 2> $O/trace_span.err
cd $R
bash tools/pmc_run.sh r03_b64 $B64
bash tools/pmc_run.sh r03_span $SPN
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -d $O/pmc_b64_$c -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $B64 > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc $c -d $O/pmc_span_$c -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --settle-ms 0 $SPN > /dev/null 2>&1
done
