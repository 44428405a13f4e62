# GPU suite + measured parity errors (tools/parity_errors.py) + a bench A/B
# of VARIANTS.  TAG names gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-check}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
fi
timeout -k 10 300 python -u tools/parity_errors.py ${PARITY_ARGS:-} > $O/parity.jsonl 2> $O/parity.err || { tail $O/parity.err; exit 2; }
python tools/parity_summary.py $O/parity.jsonl
TAG=${TAG:-check} bash tools/gpu_ab.sh
