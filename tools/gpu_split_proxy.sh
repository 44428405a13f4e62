# Per-rank shapes of the 27-camera rig split over N ranks (BASELINE configs[3]),
# one rank at a time on one GPU (bench.py --proxy-world N --proxy-rank r):
# SPLITS ("cameras windows"), RANKS, REPS, N (default 8); one summary line per
# run; JSON lines in gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-split}
mkdir -p $O
for rep in $(seq 1 ${REPS:-1}); do
for sp in ${SPLITS:-cameras windows}; do
for r in ${RANKS:-0}; do
  f=$O/proxy_${sp}_n${N:-8}_r${r}_$rep.json
  timeout -k 10 200 python bench.py --cams-total 27 --proxy-world ${N:-8} --proxy-rank $r --split $sp --no-cpu-baseline ${BENCH_ARGS:-} > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
  python -c "import json; d=json.load(open('$f')); print('proxy', '$sp', $r, d['ms_per_step'], d['config']['cams_per_rank'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items() if v > 0.04})"
done
done
done
