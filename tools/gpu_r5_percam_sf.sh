# The per-camera drop-in without the host round trip: the GPU suite's
# per-camera and sync-free tests, then interleaved bench lines of the drop-in
# (--mode percam) with it (GS_PERCAM_SYNC_FREE=1, the default) and without,
# at BASELINE configs[1] (one camera, 100k Gaussians) and the bench scene
# (27 cameras on 4 streams).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05psf}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sync_free.py \
  tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_streams.py tests/test_gpu_envelope.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 0 1; do
    f=$O/cfg1_sf${v}_$rep.json
    GS_BENCH_OTHER=0 GS_PERCAM_SYNC_FREE=$v timeout -k 10 200 python bench.py --mode percam --gaussians 100000 \
      --cams 1 --steps 200 --warmup 20 --no-cpu-baseline > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
    python -c "import json; d=json.load(open('$f')); print('cfg1 percam sf=$v', $rep, d['ms_per_step'])"
    f=$O/bench_sf${v}_$rep.json
    GS_BENCH_OTHER=0 GS_PERCAM_SYNC_FREE=$v timeout -k 10 200 python bench.py --mode percam --no-cpu-baseline \
      > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 3; }
    python -c "import json; d=json.load(open('$f')); print('27cam percam sf=$v', $rep, d['ms_per_step'])"
  done
done
