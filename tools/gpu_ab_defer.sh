# bench A/B: each camera's backward issued right after its forward vs after the next camera's forward
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/ab_defer.txt
for r in 1 2 3; do
for d in 0 1; do
  GS_BENCH_DEFER_BWD=$d timeout -k 10 200 python bench.py --no-cpu-baseline --steps 60 --warmup 15 > gpurun_out/ad_tmp.json 2>/dev/null || exit 2
  echo "defer=$d $(python3 -c "import json;r=json.loads(open('gpurun_out/ad_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/ab_defer.txt
done
done
for d in 0 1; do
  GS_BENCH_DEFER_BWD=$d timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ad_tmp.json 2>/dev/null || exit 3
  echo "default-window defer=$d $(python3 -c "import json;r=json.loads(open('gpurun_out/ad_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/ab_defer.txt
done
