# Round 6, first GPU call: the sharded-step tests (overlapped ZeRO-1 race
# checks, the driver on the sharded step), the suites touched this round, the
# bench line, and BASELINE configs[3] at its stated length (150 timesteps).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_step.py tests/test_gpu_sharded_adam.py \
  tests/test_gpu_sync_free.py tests/test_gpu_timesteps.py -x -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 2; }
tail -3 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cut -c1-400 $O/bench.json
timeout -k 10 400 python tools/timesteps_run.py --timesteps 150 --iters 2 --features 32 --neighbors --sharded \
  --per-timestep --out $O/ts150.json > $O/ts150.log 2> $O/ts150.err || { tail -30 $O/ts150.err; exit 4; }
python -c "import json; d=json.load(open('$O/ts150.json')); print({k: d[k] for k in ('ms_per_iteration','after_t1','optimizer_step')})"
