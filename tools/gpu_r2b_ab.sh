# GPU parity tests of the blend kernels, then batch-bench A/B of build variants
# ($VARIANTS, "-" = product; $REPS interleaved rounds)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/ab
mkdir -p $O
if [ -n "${TESTS:-}" ]; then
timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
for rep in $(seq ${REPS:-1}); do
for v in ${VARIANTS:-"-"}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --mode batch ${BENCH_ARGS:-} > $O/var_${n}_$rep.json 2> $O/var_${n}_$rep.err || { tail -5 $O/var_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/var_${n}_$rep.json')); print('$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
