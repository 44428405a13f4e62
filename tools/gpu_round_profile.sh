# round profile: rocprofv3 kernel stats of bench.py, then the HBM-traffic and
# instruction-count counters of the stage benchmark (separate --pmc passes,
# kernel trace only, no other tracing)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/bprof $R/gpurun_out/pmcF $R/gpurun_out/pmcW $R/gpurun_out/pmcV
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bprof.json 2> $R/gpurun_out/bprof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmcF -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcF.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/pmcW -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcW.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/pmcV -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcV.log 2>&1 || exit 4
