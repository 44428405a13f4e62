# k-NN tests + timing on the GPU box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_knn.py tests/test_boundary.py -q -x --timeout 300 -p no:cacheprovider > gpurun_out/tk.log 2>&1 || exit 1
timeout -k 10 300 python tools/knn_bench.py > gpurun_out/knn_bench.jsonl 2> gpurun_out/knn_bench.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/knnprof -o knn --output-format csv -- python3 $R/tools/knn_bench.py --n 300000 --reps 2 > $R/gpurun_out/knnprof.log 2>&1 || exit 3
