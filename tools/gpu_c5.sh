# BASELINE configs[4] scale check: 1M Gaussians at 1920x1080, F=32
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/stage_bench.py --gaussians 1000000 --width 1920 --height 1080 --features 32 --cams 2 --reps 2 > gpurun_out/c5.jsonl 2> gpurun_out/c5.err || exit 1
timeout -k 10 300 python tools/stage_bench.py --gaussians 100000 --width 800 --height 800 --features 0 32 --cams 2 --reps 3 > gpurun_out/c2.jsonl 2> gpurun_out/c2.err || exit 2
