#!/bin/bash
# Submission depth 2 against 3 (bench.py --depth) for c3 and c4, interleaved, 3 000 blocks a run.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/depth
cd "$R"
for w in c4; do
  mkdir -p "$O/$w"
  for rep in 1 2 3 4; do
    for d in 2 3; do
      timeout -k 10 300 python -u bench.py --workload $w --no-cpu --steps 3000 --warmup 200 --depth $d \
        > "$O/$w/ab_d${d}_$rep.json" 2> "$O/$w/ab_d${d}_$rep.err"
    done
  done
done
python3 tools/ab_summary.py "$O/c4"
