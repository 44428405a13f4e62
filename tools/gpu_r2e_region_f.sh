set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for v in - exp_region; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --features 0 > gpurun_out/f0_$n.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/f0_$n.json')); print('F0', '$n', d['value'], d['ms_per_step'], d['stages_ms_per_step']['render_bwd'], d['stages_ms_per_step']['render_fwd'])"
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --features 16 > gpurun_out/f16_$n.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/f16_$n.json')); print('F16', '$n', d['value'], d['ms_per_step'], d['stages_ms_per_step']['render_bwd'], d['stages_ms_per_step']['render_fwd'])"
done; done
