# Round 6: the forward-zeroed backward scratch (ABI 13) -- the batch GPU
# tests, then the bench interleaved with GS_FORWARD_ZERO_SCRATCH=0 (the
# backward's own fill) at 27 and 4 cameras, and a kernel trace of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06zero}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_sharded_step.py tests/test_gpu_fused.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for z in 1 0; do
    for c in 27 4; do
      GS_FORWARD_ZERO_SCRATCH=$z timeout -k 10 300 python bench.py --no-cpu-baseline --cams $c > $O/b_z${z}_c${c}_$rep.json 2> $O/b_z${z}_c${c}_$rep.err || { tail $O/b_z${z}_c${c}_$rep.err; exit 3; }
      python -c "import json; d=json.load(open('$O/b_z${z}_c${c}_$rep.json')); print('bench z=$z c=$c', d['value'], d['ms_per_step'], round(d['stages_ms_per_step']['render_fwd'],3), round(d['stages_ms_per_step']['render_bwd'],3))"
    done
  done
done
