# The ranking sort with its depth-range reduction in one barrier (per-wave
# ranges folded by every thread, no LDS atomics) against the previous
# commit (frozen as variant r05_rank_v1): the binning parity tests, then
# interleaved bench lines at the bench scene, configs[4] per rank and rank
# 5's configs[3] proxy.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05rank3}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_walk_order.py tests/test_gpu_sync_free.py tests/test_gpu_batch.py tests/test_gpu_windows.py \
  tests/test_gpu_sweep.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
E="GSPLAT_VARIANT=r05_rank_v1 GSPLAT_VARIANT=ctl"
TAG=${TAG:-r05rank3}/bench REPS=3 ENVS="$E" BENCH_ARGS="--steps 20" bash tools/gpu_env_ab.sh || exit 2
TAG=${TAG:-r05rank3}/cfg4 REPS=2 ENVS="$E" BENCH_ARGS="--gaussians 1000000 --width 1920 --height 1080 --cams 4 --features 32 --steps 10 --warmup 3" bash tools/gpu_env_ab.sh || exit 3
TAG=${TAG:-r05rank3}/px5 REPS=2 ENVS="$E" BENCH_ARGS="--cams-total 27 --proxy-world 8 --proxy-rank 5 --steps 100 --warmup 10" bash tools/gpu_env_ab.sh || exit 4
