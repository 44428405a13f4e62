# bench.py's overlapped feature all-reduce (N > 1) rehearsed with two ranks on
# the box's one GPU over gloo: the parameters after the timed steps must match
# the unoverlapped exchange (GS_BENCH_OVERLAP=0) to within the run-to-run
# noise of the float-atomic gradient sums (tools/compare_params.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-overlap}
mkdir -p $O
A="--gpus 2 --steps 3 --warmup 1 --gaussians 100000 --cams 4 --width 400 --height 400 --no-cpu-baseline"
run() {  # name, port, extra env
  env GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 $3 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py $A --dump-params $O/$1.npz \
    > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
}
run ov1 29561 GS_BENCH_OVERLAP=1 && run ov0a 29562 GS_BENCH_OVERLAP=0 && run ov0b 29563 GS_BENCH_OVERLAP=0 || exit 1
python -c "import json; d=json.load(open('$O/ov1.json')); print(d['config']['grad_exchange'], d['ms_per_step'])"
python tools/compare_params.py $O/ov1.npz $O/ov0a.npz $O/ov0b.npz || { rm -f $O/*.npz; exit 1; }
# The same exchange over RCCL at a world of one (RCCL refuses two ranks on one
# GPU): GS_BENCH_OVERLAP=force runs the async all-reduce on RCCL's stream and
# the side stream's wait on it; its parameters against two unoverlapped runs.
rrun() {  # name, port, overlap setting
  env GS_BENCH_FORCE_DIST=1 GS_BENCH_OVERLAP=$3 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $2 bench.py ${A/--gpus 2/--gpus 1} \
    --dump-params $O/$1.npz > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
}
rrun rccl_ov1 29571 force && rrun rccl_ov0a 29572 0 && rrun rccl_ov0b 29573 0 || exit 1
python -c "import json; d=json.load(open('$O/rccl_ov1.json')); print(d['config']['grad_exchange'], d['ms_per_step'])"
python tools/compare_params.py $O/rccl_ov1.npz $O/rccl_ov0a.npz $O/rccl_ov0b.npz; rc=$?
rm -f $O/*.npz  # the dumps are large; the comparisons above are the record
exit $rc
