# The GPU suite, then an interleaved A/B of build variants (tools/gpu_ab.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r05s}
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
fi
if [ -n "${VARIANTS:-}" ]; then
TAG=$TAG VARIANTS="$VARIANTS" REPS=${REPS:-3} bash tools/gpu_ab.sh || exit 2
fi
