# fused colour+seg tests on the GPU box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_fused.py -m gpu -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tf.log 2>&1 || exit 1
timeout -k 10 300 python tools/fused_bench.py --cams 8 --reps 5 > gpurun_out/fused_bench.jsonl 2> gpurun_out/fused_bench.err || exit 2
