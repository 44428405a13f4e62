# configs[1] (100k Gaussians, one 800x800 camera, F = 0): the current tree vs
# a previous revision ("old", tools/build_rev.sh <rev>), interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2f_c1ab
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
for v in - old; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --gaussians 100000 --cams 1 --features 0 --steps 20 --warmup 3 > $O/c1_${n}_$rep.json 2> $O/c1_${n}_$rep.err || { tail -5 $O/c1_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_${n}_$rep.json')); print('c1', '$n', d['value'], d['ms_per_step'], 'percam', d['other_mode']['ms_per_step'], {k: round(v,4) for k, v in d['stages_ms_per_step'].items()})"
done
done
