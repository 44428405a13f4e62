# Interleaved A/B of bench.py settings given as environment assignments
# (the same product library): ENVS = space-separated "NAME=value" settings
# ("-" = none), REPS rounds, BENCH_ARGS, TAG names gpurun_out/$TAG.  One
# summary line per run: headline Mpix/s, ms per step, per-stage device times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-envab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
for e in ${ENVS:--}; do
  n=$(echo "$e" | tr '=' '_')
  if [ "$e" = "-" ]; then
    timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  else
    env "$e" timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 1; }
  fi
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items() if v > 0.04})"
done
done
