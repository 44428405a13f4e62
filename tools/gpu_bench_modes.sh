# bench step-time modes vs the number of HIP streams (long windows, repeated)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/bench_modes.txt
for r in 1 2 3; do
for ns in 1 2 4; do
  GS_BENCH_STREAMS=$ns timeout -k 10 200 python bench.py --no-cpu-baseline --steps 60 --warmup 15 --step-times > gpurun_out/bm_tmp.json 2>/dev/null || exit 2
  echo "streams=$ns $(python3 -c "
import json,statistics as s
r=json.loads(open('gpurun_out/bm_tmp.json').read().strip().splitlines()[-1])
h=r['host_step_ms']
print(r['value'], r['ms_per_step'], 'host step ms median %.2f min %.2f max %.2f' % (s.median(h), min(h), max(h)))")" >> gpurun_out/bench_modes.txt
done
done
