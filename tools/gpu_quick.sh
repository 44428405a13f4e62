# parity tests of the rasterizer + stage timing (dev loop)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tq.log 2>&1 || exit 1
timeout -k 10 300 python tools/stage_bench.py --features 0 32 --cams 4 --reps 5 > gpurun_out/stage.jsonl 2> gpurun_out/stage.err || exit 2
