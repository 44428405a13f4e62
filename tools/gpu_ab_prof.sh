# A/B of library builds by rocprofv3 kernel durations (stage benchmark,
# F = ${AB_F:-32}); variants in $AB_VARIANTS ("-" = product), $AB_ROUNDS rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/abp
for round in $(seq ${AB_ROUNDS:-1}); do
for v in ${AB_VARIANTS:-"-" old}; do
  n=${v}; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abp/${n}_$round -o k --output-format csv -- python3 $R/tools/stage_bench.py --features ${AB_F:-32} --cams 4 --reps 5 --no-timing > $R/gpurun_out/abp_${n}_$round.log 2>&1 || exit 2
done
done
