#!/bin/bash
# Interleaved A/B of libsdr variants on one GPU box (run under gpurun from the repo root):
#   tools/ab_bench.sh <out-dir> <reps> "<bench args, commas for spaces>" <lib-name> [<lib-name> ...]
# lib-name "prod" is the product libsdr.so, NAME=VALUE the product library under that environment
# variable, any other name libsdr_<name>.so (tools/ab_lib.sh).
# Each rep runs every variant once, in order; one JSON line per run -> <out-dir>/ab_<name>_<rep>.json.
# Every run has its own time limit; the first failure ends the script (set -e), nothing is retried.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$1; reps=$2; args=$(echo "$3" | tr ',' ' '); shift 3
case "$O" in /*) ;; *) O=$R/$O ;; esac
mkdir -p "$O"
cd "$R"
for rep in $(seq 1 "$reps"); do
  for v in "$@"; do
    lib=$R/real-time-software-defined-radio_amd/libsdr.so
    envs=""
    case "$v" in
      prod) ;;
      *=*) envs="$v" ;;                     # NAME=VALUE: the product library with that environment
      *) lib=$R/real-time-software-defined-radio_amd/libsdr_$v.so ;;
    esac
    env $envs SDR_LIB=$lib timeout -k 10 300 python -u bench.py $args > "$O/ab_${v}_$rep.json" 2> "$O/ab_${v}_$rep.err"
    python3 - "$O/ab_${v}_$rep.json" "$v" "$rep" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(f"{sys.argv[2]:>10} rep {sys.argv[3]}: value {d['value']:.1f} {d['unit']}  ms/step {d['ms_per_step']}  "
      f"kernel ms {r.get('avg_launch_ms')}  frac {r.get('frac')}  {json.dumps(d.get('kernels_ms', {}))}  "
      f"stages {json.dumps(d.get('stage_ms', {}))}")
EOF
  done
done
