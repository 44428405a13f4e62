# configs[1] (host-bound, one camera per step): zero-filled vs fresh gradients, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/ab_gradnone.txt
for r in 1 2 3; do
for g in 0 1; do
  GS_BENCH_GRAD_NONE=$g timeout -k 10 200 python bench.py --no-cpu-baseline --gaussians 100000 --cams 1 --features 0 --steps 100 --warmup 10 > gpurun_out/gn_tmp.json 2>/dev/null || exit 2
  echo "grad_none=$g $(python3 -c "import json;r=json.loads(open('gpurun_out/gn_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/ab_gradnone.txt
done
done
