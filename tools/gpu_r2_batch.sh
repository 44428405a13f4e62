# batch path: GPU tests, bench batch vs per-camera, rocprof kernel stats of the batch bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${TEST_ARGS:-} > gpurun_out/r2_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r2_tests.log; exit 1; }
tail -2 gpurun_out/r2_tests.log
fi
for rep in $(seq ${REPS:-2}); do
for mode in ${MODES:-batch percam}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --mode $mode ${BENCH_ARGS:-} > gpurun_out/bm_${mode}_$rep.json 2> gpurun_out/bm_${mode}_$rep.err || { tail -20 gpurun_out/bm_${mode}_$rep.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/bm_${mode}_$rep.json')); print('$mode', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
if [ "${PROF:-1}" = "1" ]; then
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/bprof_batch
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bprof_batch -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 --mode batch > $R/gpurun_out/bprof_batch.json 2> $R/gpurun_out/bprof_batch.err || exit 4
cd $R && f=$(find gpurun_out/bprof_batch -name bench_kernel_stats.csv | head -1) && python - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{r['Name'].split('(')[0].replace('void ','')[:44]:44s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  {r['Percentage']}%")
PY
fi
