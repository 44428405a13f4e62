# full GPU test suite + fused colour/seg timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tq.log 2>&1 || exit 1
timeout -k 10 300 python tools/fused_bench.py --cams 8 --reps 5 > gpurun_out/fused_bench.jsonl 2> gpurun_out/fused_bench.err || exit 2
