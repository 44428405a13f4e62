# The tile sort's short length class in 128-thread workgroups against 256
# (GS_SORT_SHORT_NT): the binning parity tests under the new default, then
# interleaved bench lines at the bench scene and at rank 5's configs[3]
# proxy (3 whole cameras + 2 window pieces).  The switch and the 128-thread
# variant were removed after this run: kept as the
# record of the measurement.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05sort}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_walk_order.py tests/test_gpu_sync_free.py tests/test_gpu_batch.py tests/test_gpu_windows.py \
  tests/test_gpu_sweep.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PX="--cams-total 27 --proxy-world 8 --proxy-rank 5 --steps 100 --warmup 10"
for rep in 1 2 3; do
  for nt in 256 128; do
    for cfg in bench px5; do
      a=""; [ $cfg = px5 ] && a="$PX"
      f=$O/${cfg}_${nt}_$rep.json
      env GS_BENCH_OTHER=0 GS_SORT_SHORT_NT=$nt timeout -k 10 300 python bench.py $a --no-cpu-baseline > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
      python -c "import json; d=json.load(open('$f')); s=d['stages_ms_per_step']; print('$cfg nt=$nt', $rep, d['ms_per_step'], 'sort', s['sort'], 'dup', s['duplicate'])"
    done
  done
done
