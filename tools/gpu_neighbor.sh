# neighbour-loss tests + timing + kernel profile (+ HBM counters) on the GPU box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_neighbor.py tests/test_boundary.py -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tn.log 2>&1 || exit 1
timeout -k 10 300 python tools/neighbor_bench.py --n 150000 --k 20 --reps 20 > gpurun_out/nb_bench.jsonl 2> gpurun_out/nb_bench.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/nbprof -o nb --output-format csv -- python3 $R/tools/neighbor_bench.py --n 150000 --k 20 --reps 10 --hip-only > $R/gpurun_out/nbprof.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "nb_" -d $R/gpurun_out/nbpmcF -o pmc --output-format csv -- python3 $R/tools/neighbor_bench.py --n 150000 --k 20 --reps 2 --hip-only > $R/gpurun_out/nbpmcF.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "nb_" -d $R/gpurun_out/nbpmcW -o pmc --output-format csv -- python3 $R/tools/neighbor_bench.py --n 150000 --k 20 --reps 2 --hip-only > $R/gpurun_out/nbpmcW.log 2>&1 || exit 5
