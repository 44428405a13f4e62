# fused Adam + densification stats tests on the GPU box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/adam_probe.py > gpurun_out/adam_probe.jsonl 2> gpurun_out/adam_probe.err || exit 2
timeout -k 10 400 python -m pytest tests/test_optim.py tests/test_boundary.py -q -x --timeout 300 -p no:cacheprovider > gpurun_out/to.log 2>&1 || exit 1
timeout -k 10 300 python tools/optim_bench.py --gaussians 300000 --features 32 --reps 50 > gpurun_out/optim_bench.jsonl 2> gpurun_out/optim_bench.err || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/optprof -o opt --output-format csv -- python3 $R/tools/optim_bench.py --gaussians 300000 --features 32 --reps 20 > $R/gpurun_out/optprof.log 2>&1 || exit 4
