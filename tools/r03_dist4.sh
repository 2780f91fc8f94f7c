# four ranks on the one-GPU box (ranks wrap onto the visible device): the torchrun path of the
# default bench line (headline + C5 + u8 blocks) and of c5 spans
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/dist4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 --no-cpu > $O/bench_default_dist4.json 2> $O/bench_default_dist4.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 4 --workload c5 --no-cpu > $O/bench_c5_dist4.json 2> $O/bench_c5_dist4.err
