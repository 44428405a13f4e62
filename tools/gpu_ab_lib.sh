# A/B of library builds on the stage benchmark: GSPLAT_VARIANT in $AB_VARIANTS
# ("-" = product), run in $AB_ROUNDS interleaved rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
: > gpurun_out/ab_lib.jsonl
for round in $(seq ${AB_ROUNDS:-1}); do
for v in ${AB_VARIANTS:-"-" old}; do
  [ "$v" = "-" ] && v=""
  echo "variant=$v" >> gpurun_out/ab_lib.jsonl
  GSPLAT_VARIANT=$v timeout -k 10 300 python tools/stage_bench.py --features ${AB_F:-0 32} --cams 4 --reps 5 >> gpurun_out/ab_lib.jsonl 2>> gpurun_out/ab_lib.err || exit 2
done
done
