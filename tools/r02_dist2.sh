# two ranks on the one-GPU box (ranks wrap onto the visible device): the torchrun path of c5 and the headline
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/dist2
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --workload c5 --no-cpu > $O/bench_c5_dist2.json 2> $O/bench_c5_dist2.err
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --no-cpu > $O/bench_default_dist2.json 2> $O/bench_default_dist2.err
