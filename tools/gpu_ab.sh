# Interleaved A/B of build variants on the bench scene (27-camera batch,
# F = 32).  VARIANTS: space-separated build variants ("-" = the product
# library), REPS rounds, TAG names gpurun_out/$TAG.  One summary line per run:
# headline Mpix/s, ms per step and the per-stage device times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-ab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARIANTS:--}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items() if v > 0.05})"
done
done
