# The 4-camera rank (BASELINE configs[3] with whole cameras: rank 0 of 8 holds
# cameras 0, 8, 16, 24): --split cameras --proxy-world 8 with the sharded
# Adam (GS_BENCH_ZERO=1, a rank's own 1/8 slice) and without (the full Adam),
# and the plain --cams 4 line (one GPU owning all parameters); interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05c4}; mkdir -p $O
for rep in 1 2 3; do
  for v in zero full cams4; do
    case $v in
      zero) env="GS_BENCH_ZERO=1"; a="--cams-total 27 --split cameras --proxy-world 8 --proxy-rank 0";;
      full) env="GS_BENCH_ZERO=0"; a="--cams-total 27 --split cameras --proxy-world 8 --proxy-rank 0";;
      cams4) env="GS_BENCH_OTHER=0"; a="--cams 4";;
    esac
    f=$O/${v}_$rep.json
    env $env timeout -k 10 200 python bench.py $a --no-cpu-baseline > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
    python -c "import json; d=json.load(open('$f')); print('$v', $rep, d['ms_per_step'], d['config']['cams_per_rank'])"
  done
done
