# batch-mode bench per build variant ($VARIANTS, "-" = product): step time and stage times
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for rep in $(seq ${REPS:-1}); do
for v in ${VARIANTS:-"-"}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --mode batch ${BENCH_ARGS:-} > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || { tail -5 gpurun_out/var_$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/var_$n.json')); print('$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
