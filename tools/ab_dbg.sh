#!/bin/bash
# A/B of a diagnostic libsdr build (tools/build_dbg.sh) against the shipped one on one box:
# bench.py with the same args, interleaved, each run under its own time limit; the chain stops
# at the first failure (set -e), nothing is retried.
#   tools/ab_lib.sh <out-dir> <libsdr_X.so> <reps> <bench args, commas for spaces>
# -> <out-dir>/{base,alt}_<i>.json
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1; LIB=$2; N=$3; ARGS=$(echo "$4" | tr ',' ' ')
case "$O" in /*) ;; *) O=$R/$O ;; esac
mkdir -p "$O"
cd "$R"
for i in $(seq 1 "$N"); do
  timeout -k 10 300 python -u bench.py $ARGS > "$O/base_$i.json" 2> "$O/base_$i.err"
  SDR_LIB="$R/real-time-software-defined-radio_amd/$LIB" timeout -k 10 300 python -u bench.py $ARGS \
    > "$O/alt_$i.json" 2> "$O/alt_$i.err"
done
# (run r06/f: tools/ab_dbg.sh gpurun_out/th32 libsdr_th32.so 2 --workload,c5,--no-cpu)
