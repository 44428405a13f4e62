# GPU_MAX_HW_QUEUES 4 vs 8 at 4 camera streams, interleaved pairs
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/bench_hwq2.txt
for r in 1 2 3 4; do
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu-baseline --steps 60 --warmup 15 > gpurun_out/bq_tmp.json 2>/dev/null || exit 2
  echo "hwq=$q $(python3 -c "import json;r=json.loads(open('gpurun_out/bq_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/bench_hwq2.txt
done
done
