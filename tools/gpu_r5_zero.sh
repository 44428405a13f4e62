# Sharded Adam (distributed.ShardedAdam) and the batch's gradient
# destinations: their GPU tests, then an interleaved A/B of configs[3]
# per-rank proxies with the sharded optimizer (GS_BENCH_ZERO=1, the default
# for a rank of N) against the full Adam on every rank (GS_BENCH_ZERO=0),
# on the committed round-5 window cut (--whole-scale).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r05z}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sharded_adam.py \
  tests/test_gpu_batch.py tests/test_gpu_raw_params.py tests/test_gpu_feature_ready.py tests/test_gpu_sync_free.py \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
WS=1.0285,0.9956,0.9957,1.0156,0.9863,1.0037,0.9442,1.0316
for rep in $(seq 1 ${REPS:-2}); do
for r in ${RANKS:-2 5}; do
for z in 0 1; do
  f=$O/proxy_r${r}_z${z}_$rep.json
  GS_BENCH_ZERO=$z timeout -k 10 200 python bench.py --cams-total 27 --proxy-world 8 --proxy-rank $r \
    --no-cpu-baseline --whole-scale $WS > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
  python -c "import json; d=json.load(open('$f')); print('proxy', $r, 'zero', $z, $rep, d['ms_per_step'], d['config']['optimizer'][:40])"
done
done
done
