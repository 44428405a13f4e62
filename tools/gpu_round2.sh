# round deliverables: GPU tests, smoke, bench (with CPU baseline), rocprofv3 kernel stats of bench, PMC traffic
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "tests exit $?" >> gpurun_out/t2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bprof.json 2> $R/gpurun_out/bprof.err || exit 3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcF -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcF.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcW -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcW.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/pmcV -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcV.log 2>&1 || exit 6
