# round-3 closing set, part B: kernel-trace --stats summaries (headline fused, c5 S8 span, c5 block 64
# streams, u8 MFMA mono) and HBM traffic passes for the headline and u8
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${R03_OUT:-r03_final}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
timeout -k 10 240 $P -d $O/prof_fused -o prof -- python3 $R/bench.py --no-cpu --no-extras --steps 20 --warmup 5 > $O/prof_fused.json 2> $O/prof_fused.err
timeout -k 10 240 $P -d $O/prof_c5_s8 -o prof -- python3 $R/bench.py --workload c5 --streams 8 --no-cpu > $O/prof_c5_s8.json 2> $O/prof_c5_s8.err
timeout -k 10 240 $P -d $O/prof_c5_b64 -o prof -- python3 $R/bench.py --workload c5 --streams 64 --span 1 --no-pipeline --no-cpu --steps 20 --warmup 5 > $O/prof_c5_b64.json 2> $O/prof_c5_b64.err
timeout -k 10 240 $P -d $O/prof_u8 -o prof -- python3 $R/bench.py --iq u8 --blocks 128 --no-cpu --no-extras --steps 20 --warmup 5 > $O/prof_u8.json 2> $O/prof_u8.err
for tag in fused u8; do
  if [ $tag = fused ]; then A="--no-extras"; else A="--iq u8 --blocks 128 --no-extras"; fi
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${tag}_fetch -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --settle-ms 0 $A > /dev/null 2>&1
  timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${tag}_write -o pmc --output-format csv -- python3 $R/bench.py --no-cpu --steps 20 --warmup 5 --settle-ms 0 $A > /dev/null 2>&1
done
