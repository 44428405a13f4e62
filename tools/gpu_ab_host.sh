set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sink_tests.log 2>&1 || exit 1
for r in 1 2; do
for cfg in "GS_SINK_OLD=1 GS_BENCH_GRAD_NONE=0" "GS_SINK_OLD=0 GS_BENCH_GRAD_NONE=0" "GS_SINK_OLD=0 GS_BENCH_GRAD_NONE=1"; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_tmp.json 2>/dev/null || exit 2
  echo "$cfg $(python3 -c "import json;r=json.loads(open('gpurun_out/ab_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/ab_host.txt
done
done
