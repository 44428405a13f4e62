# The difference-array count pass (tile_count_kernel) against the
# per-instance one (GS_COUNT_MODE=instance): the binning parity tests, then
# interleaved bench lines at the bench scene and at configs[4] per rank.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05cnt}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_walk_order.py tests/test_gpu_sync_free.py tests/test_gpu_batch.py tests/test_gpu_windows.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
C4="--gaussians 1000000 --width 1920 --height 1080 --cams 4 --features 32 --steps 10 --warmup 3"
for rep in 1 2 3; do
  for v in per_instance diff; do
    env="GS_COUNT_MODE=diff"; [ $v = per_instance ] && env="GS_COUNT_MODE=instance"
    for cfg in bench cfg4; do
      a=""; [ $cfg = cfg4 ] && a="$C4"
      f=$O/${cfg}_${v}_$rep.json
      env GS_BENCH_OTHER=0 $env timeout -k 10 300 python bench.py $a --no-cpu-baseline > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
      python -c "import json; d=json.load(open('$f')); s=d['stages_ms_per_step']; print('$cfg $v', $rep, d['ms_per_step'], s['scan'], s['duplicate'], d['config']['binning_walk'][:8])"
    done
  done
done
