# Column scan with 1024-thread workgroups (product) vs 256 (exp_rs256, the previous product)
# GPU suite, then interleaved bench runs at
# the bench scene and at BASELINE configs[4] scale.  -> gpurun_out/r2f_rowscan
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r2f_rowscan
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
fi
for rep in $(seq 1 ${REPS:-3}); do
for v in - exp_rs256; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --gaussians 1000000 --width 1920 --height 1080 --cams 4 --steps 5 --warmup 2 > $O/c4_${n}_$rep.json 2> $O/c4_${n}_$rep.err || { tail -5 $O/c4_${n}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${n}_$rep.json')); print('c4', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
