# nco_long_kernel outputs per thread A/B (SDR_NCO_NR builds): span tests, C5 S8 stage times
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_ncor
mkdir -p $O
cd $R
for v in 8 4 16; do
  if [ $v = 8 ]; then L=$R/real-time-software-defined-radio_amd/libsdr.so; else L=$R/real-time-software-defined-radio_amd/libsdr_nr$v.so; fi
  SDR_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_span.py tests/test_pll_spec.py > $O/pytest_nr$v.txt 2>&1 || echo "nr$v failed" >> $O/fail.txt
  SDR_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_nr$v.json 2> $O/c5_nr$v.err
done
