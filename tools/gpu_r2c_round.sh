# Round evidence of the current tree on one MI355X: PMC of the batch launches
# (HBM traffic, instruction counts, atomic requests -> profiles/pmc_*.json read
# by bench.py), the GPU test suite, smoke(), the default bench line, and the
# rocprofv3 kernel stats of the same bench command.  Outputs in gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r02c}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 bash tools/gpu_r2_pmcbatch.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
cp profiles/pmc_traffic.json profiles/pmc_valu.json profiles/pmc_atomic.json $O/
tail -3 $O/pmc.log
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 4; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $O/bprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bprof.err || exit 5
cat $O/bench_under_rocprof.json
