# timing experiments: stage benchmark under build variants
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
: > gpurun_out/exp.jsonl
for v in "" exp_fwd_noload exp_fwd_nomfma exp_bwd_nomfma exp_noatomic exp_noacc exp_nofeat; do
  echo "variant=$v" >> gpurun_out/exp.jsonl
  GSPLAT_VARIANT=$v timeout -k 10 300 python tools/stage_bench.py --features 32 --cams 4 --reps 5 >> gpurun_out/exp.jsonl 2>> gpurun_out/exp.err || exit 2
done
