# full-size parity tests (BASELINE configs[0..2] vs the oracle, configs[4] properties)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/fullsize.log 2>&1 || exit 1
