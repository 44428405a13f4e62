# Tile sort: 512-thread workgroups for the classes past the short one (exp_mid512) vs the product
# (SKIP_TESTS=1: timing only), interleaved bench runs at
# the bench scene and at BASELINE configs[4] scale.  -> gpurun_out/r2f_mid512
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2f_mid512
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
fi
for rep in $(seq 1 ${REPS:-3}); do
for v in - exp_mid512; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --gaussians 1000000 --width 1920 --height 1080 --cams 4 --steps 5 --warmup 2 > $O/c4_${n}_$rep.json 2> $O/c4_${n}_$rep.err || { tail -5 $O/c4_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${n}_$rep.json')); print('c4', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
