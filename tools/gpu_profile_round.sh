# round profile: rocprofv3 kernel stats of bench.py, then HBM traffic counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bprof.json 2> $R/gpurun_out/bprof.err || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcF -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcF.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcW -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmcW.log 2>&1 || exit 3
