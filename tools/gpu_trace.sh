# kernel trace of the stage benchmark (per-kernel durations)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o tr --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 4 --reps 3 > $R/gpurun_out/trace.log 2>&1 || exit 1
