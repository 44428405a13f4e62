# The bucket pass's staged copy-out loop unrolled by 4 (its LDS reads of
# consecutive keys batched ahead of the stores) against the previous library
# (frozen as variant r05_bk_v1): binning parity tests, then interleaved bench
# lines at the bench scene and rank 5's configs[3] proxy.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05bku}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_walk_order.py tests/test_gpu_sync_free.py tests/test_gpu_batch.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
E="GSPLAT_VARIANT=r05_bk_v1 GSPLAT_VARIANT=ctl"
TAG=${TAG:-r05bku}/bench REPS=3 ENVS="$E" BENCH_ARGS="--steps 20" bash tools/gpu_env_ab.sh || exit 2
TAG=${TAG:-r05bku}/px5 REPS=2 ENVS="$E" BENCH_ARGS="--cams-total 27 --proxy-world 8 --proxy-rank 5 --steps 100 --warmup 10" bash tools/gpu_env_ab.sh || exit 3
