#!/bin/bash
# A/B of library builds on ONE box (run under gpurun from the repo root): each variant is a
# libsdr.so under _ab/<variant>/ (git-ignored; built with other -D flags / sources), loaded by
# bench.py through SDR_LIB; the variants alternate, <reps> rounds.  Every run has its own limit
# and the chain stops at the first failure.
#   tools/ab_lib.sh <out-dir> <reps> <bench args, commas for spaces> <variant> [<variant> ...]
# e.g. tools/ab_lib.sh gpurun_out/ab 2 --workload,c5,--no-cpu w8 w16
set -e
O=$1; R=$2; A=$(echo "$3" | tr ',' ' '); shift 3
mkdir -p "$O"
for i in $(seq "$R"); do
  for v in "$@"; do
    SDR_LIB=$PWD/_ab/$v/libsdr.so timeout -k 10 200 python -u bench.py $A >> "$O/$v.json" 2>> "$O/err.txt"
  done
done
