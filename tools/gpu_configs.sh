# The other BASELINE configs through bench.py (one GPU): configs[1] 100k Gaussians,
# one 800x800 camera (F = 0 and F = 32); configs[4] 1M Gaussians at 1920x1080,
# F = 32, 4 cameras per rank (the 8-GPU case runs the same per-rank work).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
rm -f gpurun_out/configs.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline --gaussians 100000 --cams 1 --features 0 --steps 20 --warmup 3 >> gpurun_out/configs.jsonl 2> gpurun_out/configs.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --gaussians 100000 --cams 1 --features 32 --steps 20 --warmup 3 >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.err || exit 2
timeout -k 10 300 python bench.py --no-cpu-baseline --gaussians 1000000 --width 1920 --height 1080 --cams 4 --features 32 --steps 5 --warmup 2 >> gpurun_out/configs.jsonl 2>> gpurun_out/configs.err || exit 3
