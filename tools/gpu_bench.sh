# bench (with and without the CPU baseline) + stage timings with/without events
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/stage_bench.py --features 32 --cams 4 --reps 5 > gpurun_out/stage_t.jsonl 2> gpurun_out/stage_t.err || exit 1
timeout -k 10 300 python tools/stage_bench.py --features 32 --cams 4 --reps 5 --no-timing > gpurun_out/stage_nt.jsonl 2> gpurun_out/stage_nt.err || exit 2
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3
