# Round 6: the N = 4 and N = 8 bench paths rehearsed on one GPU (gloo, every
# rank on cuda:0): the weak headline (27 cameras per rank) and the 27-camera
# split, so the driver's SCALE run meets no untested rank count.  Timing is
# meaningless here (the ranks share one GPU); the JSON lines and exit codes
# are the check.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06n8}
mkdir -p $O
for n in 4 8; do
  GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 2 \
    --warmup 1 --no-cpu-baseline > $O/weak$n.json 2> $O/weak$n.err || { tail -20 $O/weak$n.err; exit 1; }
  python -c "import json; d = json.loads(open('$O/weak$n.json').read().strip().splitlines()[-1]); print('weak', $n, d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d.get('split_step', {}) and d['split_step'].get('cams_per_rank'))"
done
