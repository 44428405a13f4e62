# The binning walk order (ABI 12) at BASELINE configs[4] per rank (1M
# Gaussians, 1920x1080, F = 32, 4 cameras): GaussianRasterizerBatch's "auto"
# (the Morton walk once the lists outgrow the bucket pass's LDS staging)
# against the id order, interleaved; then the default bench line, where
# "auto" stays in id order.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05wk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_walk_order.py \
  tests/test_gpu_sync_free.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
A="--gaussians 1000000 --width 1920 --height 1080 --cams 4 --features 32 --steps 10 --warmup 3 --no-cpu-baseline"
for rep in 1 2 3; do
  for w in 0 auto; do
    f=$O/cfg4_w${w}_$rep.json
    GS_BENCH_OTHER=0 GS_BENCH_WALK=$w timeout -k 10 300 python bench.py $A > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
    python -c "import json; d=json.load(open('$f')); s=d['stages_ms_per_step']; print('cfg4 walk=$w', $rep, d['ms_per_step'], d['config']['binning_walk'][:12], s['scan'], s['duplicate'])"
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 3
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['config']['binning_walk'])"
