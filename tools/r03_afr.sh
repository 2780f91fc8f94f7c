# host-built MFMA A fragments (product) vs built in every wave (libsdr_noafr), same box
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03_afr2
mkdir -p $O
cd $R
A="--iq u8 --blocks 128 --no-cpu --no-extras --steps 50 --warmup 10"
for k in 1 2; do
timeout -k 10 120 python bench.py $A > $O/u8_afr$k.json 2> $O/u8_afr$k.err
SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_noafr.so timeout -k 10 120 python bench.py $A > $O/u8_noafr$k.json 2> $O/u8_noafr$k.err
done
timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_afr.json 2> $O/c5_afr.err
SDR_LIB=$R/real-time-software-defined-radio_amd/libsdr_noafr.so timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --no-cpu > $O/c5_noafr.json 2> $O/c5_noafr.err
