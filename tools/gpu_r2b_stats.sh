# work counters of the blend kernels (stats build) + the default bench line
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/r02b
mkdir -p $O
timeout -k 10 300 python tools/render_stats.py --features 32 --cams 4 > $O/stats.json 2> $O/stats.err || { tail $O/stats.err; exit 1; }
cat $O/stats.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
cat $O/bench.json
