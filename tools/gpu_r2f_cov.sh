# cov3D stored once per Gaussian (camera 0) and read once by preprocess_bwd (product)
# vs the previous tree ("old", tools/build_rev.sh).  GPU suite on the product first.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2f_cov
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
fi
for rep in $(seq 1 ${REPS:-2}); do
for v in - old; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], 'pre', round(d['stages_ms_per_step']['preprocess'],4), 'pbwd', round(d['stages_ms_per_step']['preprocess_bwd'],4), 'bwd', round(d['stages_ms_per_step']['render_bwd'],3))"
done
done
