#!/bin/bash
# Submit one command through gpurun, waiting for a box: a call that did not get a box
# ("no free box right now", "backing off", "stopped responding while being prepared":
# nothing ran, nothing was charged) is submitted again after the wait gpurun asks for.  A
# call that ran -- passed, failed, faulted or timed out -- is never resubmitted.
#   tools/gpurun_wait.sh <log> <timeout-s> <command> [max-tries]
log=$1; to=$2; cmd=$3; tries=${4:-12}
for i in $(seq 1 "$tries"); do
  timeout $((to + 1500)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "no free box right now\|backing off\|stopped responding while being prepared\|slot(s) on this pod are busy\|nothing was charged" "$log" && \
     ! grep -q "status=\(ok\|fail\|error\|timeout\)" "$log"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    echo "try $i: no box; waiting ${wait_s:-240}s" >> "$log.tries"
    sleep $(( ${wait_s:-240} + 15 ))
    continue
  fi
  echo "try $i: ran (rc $rc)" >> "$log.tries"
  exit $rc
done
echo "gave up after $tries tries" >> "$log.tries"
exit 3
