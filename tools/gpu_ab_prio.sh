# (historical: the companion-stream code this A/B switched was measured slower and removed)
# plan chain on a high-priority companion stream: tests, then bench A/B (long windows, repeated)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/ab_prio.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/tq_prio.log 2>&1 || exit 1
for r in 1 2 3; do
for p in 0 1; do
  GS_PLAN_PRIORITY=$p timeout -k 10 200 python bench.py --no-cpu-baseline --steps 60 --warmup 15 > gpurun_out/ap_tmp.json 2>/dev/null || exit 2
  echo "prio=$p $(python3 -c "import json;r=json.loads(open('gpurun_out/ap_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/ab_prio.txt
done
done
