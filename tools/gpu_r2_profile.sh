# round-2 evidence: GPU tests, smoke, the default bench line, and the
# rocprofv3 kernel stats of the same bench command (kernel trace only)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r02
O=$R/gpurun_out/r02
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 2; }
cat $O/smoke.log | tail -1
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 3; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $O/bprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bprof.err || exit 4
cat $O/bench_under_rocprof.json
