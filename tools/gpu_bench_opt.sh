# bench with the fused optimizer vs torch's Adam (no CPU baseline), then the default bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
GS_BENCH_OPTIM=torch timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_torchadam.json 2> gpurun_out/bench_torchadam.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fusedadam.json 2> gpurun_out/bench_fusedadam.err || exit 2
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 3
