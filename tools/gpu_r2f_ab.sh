# Interleaved A/B of build variants on the bench scene (27-camera batch,
# F = 32): VARIANTS (default: product, exp_fulw, exp_ulw), REPS rounds.
# -> gpurun_out/r2f_ab/*.json, one summary line per run.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2f_ab
mkdir -p $O
for rep in $(seq 1 ${REPS:-3}); do
for v in ${VARIANTS:-- exp_fulw exp_ulw}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()}, 'percam', d['other_mode']['ms_per_step'])"
done
done
