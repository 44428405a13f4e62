# Tile-sort variants at BASELINE configs[4] scale (1M Gaussians, 1920x1080,
# 4 cameras, F = 32) and at the bench scene, interleaved.
set -o pipefail
if [ -n "${TESTS:-}" ]; then cd $GRAFT_REPO_ROOT; timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sortab_tests.log 2>&1 || { tail -30 gpurun_out/sortab_tests.log; exit 1; }; tail -2 gpurun_out/sortab_tests.log; fi
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/sortab
mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-- exp_bsl10 exp_bsl12}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --gaussians 1000000 --width 1920 --height 1080 --cams 4 --steps 5 --warmup 2 > $O/c4_${n}_$rep.json 2> $O/c4_${n}_$rep.err || { tail -5 $O/c4_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${n}_$rep.json')); print('c4', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
