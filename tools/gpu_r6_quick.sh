# Round 6: parity subset, a kernel trace of a short bench (stage check), and
# the bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06q}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_gpu_fused.py} -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 4; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $O/kt.json 2> $O/kt.err || { tail $O/kt.err; exit 1; }
cd $R && grep -E "absmax|render_fwd|render_bwd" $O/kt/kt_kernel_stats.csv | cut -c1-150 | head -8
rm -f $O/kt/kt_kernel_trace.csv
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['other_mode'])"
