set -e
O=gpurun_out/r05ab; mkdir -p $O
for i in 1 2 3; do
  for v in a b; do
    SDR_LIB=$PWD/_ab/$v/libsdr.so timeout -k 10 120 python -u bench.py --iq u8 --no-extras --no-cpu >> $O/u8_$v.json 2>>$O/err.txt
  done
done
for i in 1 2; do
  for v in a b; do
    SDR_LIB=$PWD/_ab/$v/libsdr.so timeout -k 10 200 python -u bench.py --workload c5 --no-cpu >> $O/c5_$v.json 2>>$O/err.txt
  done
done
