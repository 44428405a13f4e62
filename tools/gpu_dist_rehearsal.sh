# two ranks on the one GPU of the box over gloo: exercises bench.py's
# distributed path (sharding, bucket all-reduce, max-over-ranks, JSON line)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/dist2.json 2> gpurun_out/dist2.err || exit 1
