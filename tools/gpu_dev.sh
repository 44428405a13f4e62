# dev loop on the GPU box: parity tests, stage timings, blend work counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tq.log 2>&1; echo "tests exit $?" >> gpurun_out/tq.log
timeout -k 10 300 python tools/stage_bench.py --features 0 32 --cams 4 --reps 5 > gpurun_out/stage.jsonl 2> gpurun_out/stage.err || exit 2
timeout -k 10 300 python tools/render_stats.py --features 32 --cams 2 > gpurun_out/stats.jsonl 2> gpurun_out/stats.err || exit 3
