# bench run-to-run spread: default window vs longer warmup / window
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; rm -f gpurun_out/bench_var.txt
for r in 1 2 3; do
for a in "--steps 20 --warmup 3" "--steps 60 --warmup 15"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/bv_tmp.json 2>/dev/null || exit 2
  echo "$a $(python3 -c "import json;r=json.loads(open('gpurun_out/bv_tmp.json').read().strip().splitlines()[-1]);print(r['value'], r['ms_per_step'])")" >> gpurun_out/bench_var.txt
done
done
