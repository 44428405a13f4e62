# Round 6: the configs[3] per-rank proxies (tools/gpu_r5_proxies.sh, 3
# interleaved runs of the 8 ranks) on this tree, after a quick check of the
# forward's feature-range pre-pass (kernel trace of a short bench).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06px}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 4; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/kt.json 2> $O/kt.err || { tail $O/kt.err; exit 1; }
cd $R && grep -E "absmax|render_fwd|Name" $O/kt/kt_kernel_stats.csv | cut -c1-160 | head -8
rm -f $O/kt/kt_kernel_trace.csv
# the other configs (configs[1] drop-in F = 0 / 32, configs[4] per rank)
bash tools/gpu_configs.sh || exit 3
cp gpurun_out/configs.jsonl $O/configs.jsonl
python -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); print('config', d['config']['workload'][:60], d['ms_per_step'], {k: round(v, 3) for k, v in d['stages_ms_per_step'].items()})"
TAG=${TAG:-r06px} bash tools/gpu_r5_proxies.sh
