# Round 6: a kernel change's parity tests (PYTEST_FILES) then an interleaved
# A/B against frozen variants (VARIANTS, "-" = this tree's product library
# under the native binding, ctl = under the ctypes binding).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06ab}
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests/test_gpu_parity.py tests/test_gpu_envelope.py tests/test_gpu_fullsize.py} \
  -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
grep "{" $O/tests.log | tail -4
VARIANTS="${VARIANTS:-f16a ctl}" REPS=${REPS:-3} TAG=${TAG:-r06ab}/ab bash tools/gpu_ab.sh
