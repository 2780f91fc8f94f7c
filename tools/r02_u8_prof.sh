# u8 fused (int8 MFMA) kernel: rocprof kernel stats, SQ counters, HBM fetch/write (separate passes)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/u8p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --iq u8 --no-cpu --steps 20 --warmup 3 --settle-ms 50"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o u8 -- $B > $O/stats.json 2>$O/stats.err
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d $O/sq -o u8 -- $B > $O/sq.json 2>$O/sq.err
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o u8 -- $B > $O/fetch.json 2>$O/fetch.err
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o u8 -- $B > $O/write.json 2>$O/write.err
