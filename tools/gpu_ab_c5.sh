# A/B of library builds on the configs[4] scale (1M Gaussians, 1920x1080, F = 32) by rocprofv3 kernel durations
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/abc5
for v in ${AB_VARIANTS:-"-" old}; do
  n=${v}; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abc5/${n}_1 -o k --output-format csv -- python3 $R/tools/stage_bench.py --gaussians 1000000 --width 1920 --height 1080 --features 32 --cams 2 --reps 2 --no-timing > $R/gpurun_out/abc5_${n}.log 2>&1 || exit 2
done
