#!/bin/bash
# Round-4b PLL bisection (run under gpurun from the repo root): the span test and the PLL solve
# tests on the product library and on A/B builds with one r04b PLL change each undone
# (tools/ab_lib.sh pll.hip -DSDR_PLL_NOFAST / -DSDR_PLL_OLDCORR).  A failing test does not stop
# the script; anything else (a fault, an abort, a time limit) ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04b_bis
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
for v in prod nofast oldcorr; do
  lib=$R/real-time-software-defined-radio_amd/libsdr.so
  [ "$v" = prod ] || lib=$R/real-time-software-defined-radio_amd/libsdr_$v.so
  SDR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_span.py tests/test_pll_spec.py -m gpu -v -s \
    --timeout 200 --timeout-method thread > "$O/pytest_$v.txt" 2>&1
  rc=$?
  echo "$v: rc $rc $(tail -1 $O/pytest_$v.txt)"
  [ $rc -le 1 ] || exit $rc
done
