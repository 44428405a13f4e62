# bench step-time modes vs hardware queues per process (GPU_MAX_HW_QUEUES) and camera streams
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/bench_hwq.txt
for r in 1 2 3; do
for cfg in "GPU_MAX_HW_QUEUES=4 GS_BENCH_STREAMS=4" "GPU_MAX_HW_QUEUES=8 GS_BENCH_STREAMS=4" "GPU_MAX_HW_QUEUES=8 GS_BENCH_STREAMS=8"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 60 --warmup 15 > gpurun_out/bq_tmp.json 2>/dev/null || exit 2
  echo "$cfg $(python3 -c "import json;r=json.loads(open('gpurun_out/bq_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/bench_hwq.txt
done
done
