# dev loop: parity tests, then a kernel trace of the stage benchmark
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tq.log 2>&1; echo "tests exit $?" >> gpurun_out/tq.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/trace -o tr --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 4 --reps 3 > $R/gpurun_out/trace.log 2>&1 || exit 1
