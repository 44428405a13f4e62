# rocprofv3 kernel trace + stats of bench.py (no CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bprof.json 2> $R/gpurun_out/bprof.err || exit 1
