# Interleaved A/B of the sync-free forward: the bench
# step with GS_BENCH_SYNC_FREE=1 (gs_forward_batch) vs 0 (the two-phase
# plan -> host read -> render), at 4 cameras (an 8-rank split's rank shape)
# and at 27 (the headline).  100-step windows.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r05sfab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
for cams in 4 27; do
for sf in 1 0; do
  f=$O/c${cams}_sf${sf}_$rep.json
  GS_BENCH_SYNC_FREE=$sf timeout -k 10 200 python bench.py --cams $cams --no-cpu-baseline --steps 100 --warmup 10 \
    > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('cams', $cams, 'sync_free', $sf, $rep, d['ms_per_step'], d['config']['forward'][:10])"
done
done
done
