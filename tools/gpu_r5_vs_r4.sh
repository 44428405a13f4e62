# Same-box interleaved A/B of this tree against the round-4 tree (a git
# worktree of 795f5da built in-tree at ./r4tree): the 4-camera rank shape
# (bench.py --cams 4) and the 27-camera headline, 100-step windows; this
# tree both with the sync-free forward and with the two-phase one
# (GS_BENCH_SYNC_FREE=0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r05vs4}
mkdir -p $O
run() {  # name, dir, cams, env
  f=$O/$1.json
  (cd $2 && env $4 timeout -k 10 200 python bench.py --cams $3 --no-cpu-baseline --steps 100 --warmup 10) \
    > $f 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('$1', d['ms_per_step'], round(d['value'], 1))"
}
for rep in $(seq 1 ${REPS:-3}); do
  run c4_new_$rep . 4 GS_BENCH_SYNC_FREE=1 || exit 1
  run c4_new2p_$rep . 4 GS_BENCH_SYNC_FREE=0 || exit 1
  run c4_r4_$rep r4tree 4 X=1 || exit 1
  run c27_new_$rep . 27 GS_BENCH_SYNC_FREE=1 || exit 1
  run c27_r4_$rep r4tree 27 X=1 || exit 1
done
