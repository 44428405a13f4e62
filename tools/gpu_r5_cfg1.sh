# BASELINE configs[1] (100k Gaussians, one 800x800 camera, fwd+bwd+Adam per
# step): the per-camera drop-in (GaussianRasterizer, two-phase plan) against
# the camera batch with one camera, sync-free and two-phase; interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05c1}; mkdir -p $O
A="--gaussians 100000 --cams 1 --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline"
for rep in 1 2; do
  for v in percam batch_sf batch_2p; do
    case $v in
      percam) env="GS_BENCH_OTHER=0"; m=percam;;
      batch_sf) env="GS_BENCH_OTHER=0 GS_BENCH_SYNC_FREE=1"; m=batch;;
      batch_2p) env="GS_BENCH_OTHER=0 GS_BENCH_SYNC_FREE=0"; m=batch;;
    esac
    f=$O/${v}_$rep.json
    env $env timeout -k 10 200 python bench.py $A --mode $m > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 1; }
    python -c "import json; d=json.load(open('$f')); print('$v', $rep, d['ms_per_step'], d['value'])"
  done
done
