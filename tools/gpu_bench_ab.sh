# A/B of bench.py settings (no CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
GS_BENCH_FUSED_ADAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_a.json 2> gpurun_out/ab_a.err || exit 1
GS_BENCH_FUSED_ADAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_b.json 2> gpurun_out/ab_b.err || exit 2
