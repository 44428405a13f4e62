# The two-rank gloo rehearsals of bench.py on the one GPU (weak headline +
# split step, and --cams-total 27), each under its own time limit, with a
# heartbeat line every 30 s (a rehearsal is silent until its JSON line).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05d2}; mkdir -p $O
run() {  # name, port, extra args
  local t0=$(date +%s)
  GS_BENCH_TRACEBACKS=${TB:-60} GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 ${LIMIT:-500} python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py --gpus 2 --steps 3 --warmup 1 $3 \
    > $O/$1.json 2> $O/$1.err &
  local pid=$!
  while kill -0 $pid 2>/dev/null; do sleep 30; echo "$1: $(( $(date +%s) - t0 )) s"; done
  wait $pid || { echo "$1 failed"; tail -20 $O/$1.err; return 1; }
  python -c "import json; d=json.load(open('$O/$1.json')); print('$1', d['value'], d['ms_per_step'], (d.get('split_step') or {}).get('ms_per_step'), d['config']['grad_exchange'][:50])"
}
run ${NAMES:-dist2_strong} 29534 "${ARGS---cams-total 27}"
