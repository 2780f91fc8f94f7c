set -e
O=gpurun_out/r04d
bash tools/gpu_round.sh $O tests bench:c4:--workload,c4,--no-cpu bench:c5b64:--workload,c5,--streams,64,--span,1,--no-pipeline,--steps,20,--warmup,5,--no-cpu prof:c4:--workload,c4,--no-cpu,--steps,50
SDR_LIB=$GRAFT_REPO_ROOT/real-time-software-defined-radio_amd/libsdr_prof.so timeout -k 10 200 python -u bench.py --workload c4 --no-cpu --steps 20 > $O/prof_spec_c4.json 2> $O/prof_spec_c4.err
SDR_LIB=$GRAFT_REPO_ROOT/real-time-software-defined-radio_amd/libsdr_prof.so timeout -k 10 200 python -u bench.py --workload c5 --streams 8 --span 256 --steps 3 --warmup 1 --no-cpu > $O/prof_spec_c5.json 2> $O/prof_spec_c5.err
