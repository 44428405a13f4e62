set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "tests exit $?" >> gpurun_out/t2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/bench_prof.err || exit 3
