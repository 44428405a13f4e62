# bench.py's gradient exchanges at N > 1 rehearsed on the box's one GPU; the
# parameters after the timed steps of every variant must match the plain
# exchange (GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0: one all-reduce, the full Adam
# on every rank) to within the run-to-run noise of the float-atomic gradient
# sums (tools/compare_params.py against three runs of the plain exchange):
#   zov  the default: sharded Adam (reduce-scatter, 1/N update, all-gather)
#        with the feature exchange behind the next step
#   z    sharded Adam, in line
#   ov   all-reduce with the overlapped feature exchange
# First two ranks over gloo (sharing the GPU), then the same over RCCL at a
# world of one (RCCL refuses two ranks on one GPU; the =force settings run
# the collectives there anyway).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-overlap}
mkdir -p $O
# the step-level race check first (tools/zov_check.py: each step's gradients vs
# a replay from what it read, the reads vs an in-line Adam replay, bit for bit)
GS_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29560 tools/zov_check.py > $O/zov_check.json 2> $O/zov_check.err \
  || { tail -20 $O/zov_check.err; cat $O/zov_check.json; exit 1; }
python -c "import json; d=json.load(open('$O/zov_check.json')); print('zov_check ok:', d['ok'], 'max grad rel:', max(max(r.values()) for x in d['ranks'] for r in x['grad_rel']))"
A="--gpus 2 --steps 3 --warmup 1 --gaussians 100000 --cams 4 --width 400 --height 400 --no-cpu-baseline"
run() {  # name, port, extra env
  env GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 $3 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $2 bench.py $A --dump-params $O/$1.npz \
    > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
}
run ref_a 29561 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0" && run ref_b 29562 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0" \
  && run ref_c 29566 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0" \
  && run zov 29563 "GS_BENCH_ZERO=1 GS_BENCH_OVERLAP=1" && run z 29564 "GS_BENCH_ZERO=1 GS_BENCH_OVERLAP=0" \
  && run ov 29565 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=1" || exit 1
rc=0
for t in zov z ov; do
  python -c "import json; d=json.load(open('$O/$t.json')); print('$t:', d['config']['grad_exchange'], d['ms_per_step'])"
  python tools/compare_params.py $O/$t.npz $O/ref_a.npz $O/ref_b.npz $O/ref_c.npz || rc=1
done
rrun() {  # name, port, extra env
  env GS_BENCH_FORCE_DIST=1 $3 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $2 bench.py ${A/--gpus 2/--gpus 1} \
    --dump-params $O/$1.npz > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
}
rrun rccl_ref_a 29571 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0" && rrun rccl_ref_b 29572 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0" \
  && rrun rccl_ref_c 29576 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=0" \
  && rrun rccl_zov 29573 "GS_BENCH_ZERO=force GS_BENCH_OVERLAP=force" \
  && rrun rccl_z 29574 "GS_BENCH_ZERO=force GS_BENCH_OVERLAP=0" \
  && rrun rccl_ov 29575 "GS_BENCH_ZERO=0 GS_BENCH_OVERLAP=force" || exit 1
for t in rccl_zov rccl_z rccl_ov; do
  python -c "import json; d=json.load(open('$O/$t.json')); print('$t:', d['config']['grad_exchange'], d['ms_per_step'])"
  python tools/compare_params.py $O/$t.npz $O/rccl_ref_a.npz $O/rccl_ref_b.npz $O/rccl_ref_c.npz || rc=1
done
rm -f $O/*.npz  # the dumps are large; the comparisons above are the record
exit $rc
