# GPU tests + stage-kernel A/B of build variants ($AB_VARIANTS, "-" = product) + bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${TEST_ARGS:-} > gpurun_out/r2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r2_tests.log; exit 1; }
tail -2 gpurun_out/r2_tests.log
fi
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/abp
for round in $(seq ${AB_ROUNDS:-1}); do
for v in ${AB_VARIANTS:-"-"}; do
  n=${v}; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abp/${n}_$round -o k --output-format csv -- python3 $R/tools/stage_bench.py --features ${AB_F:-32} --cams 4 --reps 5 --no-timing > $R/gpurun_out/abp_${n}_$round.log 2>&1 || exit 2
done
done
cd $R && python tools/ab_prof_summary.py
if [ "${BENCH:-1}" = "1" ]; then
for i in $(seq ${BENCH_REPS:-1}); do
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/r2_bench_$i.json 2> gpurun_out/r2_bench_$i.err || exit 3
python -c "import json; d=json.load(open('gpurun_out/r2_bench_$i.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
fi
