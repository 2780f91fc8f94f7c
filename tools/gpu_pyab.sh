#!/bin/bash
# Interleaved A/B of the Python side of Receiver.submit: this tree against a copy of it with
# ab_tmp/old_blocks.py (the previous blocks.py) -- c4 and c3, four reps of 3 000 blocks each; the receiver's
# GPU tests first.  Each step has its own limit; the first failure ends the call.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pyab
mkdir -p "$O/c4" "$O/c3"
cd "$R"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_receiver.py -m gpu -v --timeout 120 --timeout-method thread > "$O/pytest_receiver.txt" 2>&1
tail -1 "$O/pytest_receiver.txt"
OLD=$TMPDIR/pyab_old_$$
rm -rf "$OLD" && mkdir -p "$OLD" && cp -r bench.py rtsdr.py real-time-software-defined-radio_amd "$OLD/"
cp ab_tmp/old_blocks.py "$OLD/real-time-software-defined-radio_amd/blocks.py"
for rep in 1 2 3 4; do
  for w in c4 c3; do
    for v in new old; do
      d=$R; [ $v = old ] && d=$OLD
      (cd "$d" && timeout -k 10 300 python -u bench.py --workload $w --no-cpu --steps 3000 --warmup 200) > "$O/$w/ab_${v}_$rep.json" 2> "$O/$w/ab_${v}_$rep.err"
      echo "$w $v $rep: $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" "$O/$w/ab_${v}_$rep.json")"
    done
  done
done
rm -rf "$OLD"
python3 tools/ab_summary.py "$O/c4" "$O/c3"
