# configs[3] per-rank proxies of the 27-camera windows split over N ranks
# (bench.py --proxy-world N --proxy-rank r), REPS interleaved runs of every
# rank (the bench default window: 20 steps after 3 warm-up steps, as the
# single-GPU line -- the parameters train, so the scene drifts over a run),
# after the single-GPU 27-camera bench line the
# speed-up is quoted against; then tools/split_predict.py over all of them.
# With the measured-feedback balance (bench.py --balance measured, the
# default) rank 0's first run measures every rank's shard and the others
# reuse its factors (--whole-scale), so all proxies cut the same windows.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r05px}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'])"
WS=""
for rep in $(seq 1 ${REPS:-3}); do
for r in ${RANKS:-0 1 2 3 4 5 6 7}; do
  f=$O/proxy_r${r}_$rep.json
  timeout -k 10 200 python bench.py --cams-total 27 --proxy-world ${N:-8} --proxy-rank $r --no-cpu-baseline \
    --steps ${STEPS:-20} --warmup ${WARMUP:-3} ${WS:+--whole-scale $WS} ${BENCH_ARGS:-} > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
  python -c "import json; d=json.load(open('$f')); m=d['split_model']['ranks'][$r]; print('proxy', $r, $rep, d['ms_per_step'], m['pieces'], m['model_load'])"
  if [ -z "$WS" ]; then
    WS=$(python -c "import json; d=json.load(open('$f')); w=d['split_model'].get('whole_scale'); print(','.join(str(x) for x in w) if w else '')")
    python -c "import json; d=json.load(open('$f')); print('cuts (fwd+bwd ms per rank):', d['split_model'].get('cut_fwd_bwd_ms'), 'whole_scale:', d['split_model'].get('whole_scale'))"
  fi
done
done
python tools/split_predict.py $O/bench.json $O/proxy_r*_*.json --n ${N:-8} > $O/split_prediction.json
python -c "import json; d=json.load(open('$O/split_prediction.json')); print(d['slowest_rank'], d['slowest_rank_ms'], {k: v['speedup_vs_1gpu'] for k, v in d['predictions'].items()})"
