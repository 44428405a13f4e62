# Kernel split of the configs[4] per-rank shape (1M Gaussians, 1080p, 4 cameras) under rocprofv3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05c4p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rm -rf $O/tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr -o c4 --output-format csv -- python3 $R/bench.py --gaussians 1000000 --width 1920 --height 1080 --cams 4 --features 32 --steps 10 --warmup 3 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
cd $R && python tools/kernel_split.py $(find $O/tr -name "*kernel_trace.csv") $O/split.json > $O/split.txt && head -30 $O/split.txt
rm -f $(find $O/tr -name "*kernel_trace.csv")
