# per-block PLL solve warm-up length A/B (SDR_SPEC_W builds): offset sweep + PLL tests, c4 / c5 per-block lines
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_specw
mkdir -p $O
cd $R
for w in 256 128 64; do
  if [ $w = 256 ]; then L=$R/real-time-software-defined-radio_amd/libsdr.so; else L=$R/real-time-software-defined-radio_amd/libsdr_w$w.so; fi
  SDR_LIB=$L timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread -m gpu tests/test_offsets.py tests/test_pll_spec.py tests/test_receiver.py tests/test_dropin.py > $O/pytest_w$w.txt 2>&1 || echo "w$w tests failed" >> $O/fail.txt
  SDR_LIB=$L timeout -k 10 200 python -u bench.py --workload c4 --no-cpu > $O/c4_w$w.json 2> $O/c4_w$w.err
  SDR_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --streams 64 --span 1 --no-cpu > $O/c5b64_w$w.json 2> $O/c5b64_w$w.err
done
