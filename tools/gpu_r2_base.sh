# round-2 baseline: GPU tests, stage kernel durations (rocprofv3), blend work counters, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r2_tests.log; exit 1; }
tail -3 gpurun_out/r2_tests.log
timeout -k 10 300 python tools/render_stats.py --features 32 --cams 2 > gpurun_out/r2_stats.json 2> gpurun_out/r2_stats.err || exit 2
cat gpurun_out/r2_stats.json
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err || exit 3
cat gpurun_out/r2_bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/abp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abp/product_1 -o k --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 4 --reps 5 --no-timing > $R/gpurun_out/abp_product_1.log 2>&1 || exit 4
cd $R && python tools/ab_prof_summary.py
