# bench run-to-run spread by camera-stream count (GS_BENCH_STREAMS), interleaved runs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for rep in $(seq ${REPS:-3}); do
for ns in ${STREAMS:-1 2 4}; do
  GS_BENCH_STREAMS=$ns timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-30} --warmup 3 > gpurun_out/var_$ns_$rep.json 2> gpurun_out/var.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/var_$ns_$rep.json')); print('streams', $ns, 'rep', $rep, d['value'], d['ms_per_step'])"
done
done
