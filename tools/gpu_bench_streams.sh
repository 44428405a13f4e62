# bench at 1, 2, 3 camera streams (no CPU baseline)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for n in 4 6; do
  GS_BENCH_STREAMS=$n timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_s$n.json 2> gpurun_out/bench_s$n.err || exit $n
done
