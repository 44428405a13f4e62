# Round 6: the backward's fp16 two-piece weight contractions -- the whole GPU
# suite (parity vs the oracle, the fp32 summation envelope), then an
# interleaved A/B against the round-5 library (frozen copy, variant r5) under
# the same ctypes binding (variant ctl = this tree's product flags).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06f16}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  ${PYTEST_K:-} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -3 $O/tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_envelope.py -q -s --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $O/envelope.log 2>&1 || { tail -20 $O/envelope.log; exit 3; }
grep "{" $O/envelope.log
VARIANTS="${VARIANTS:-r5 ctl}" REPS=${REPS:-3} TAG=${TAG:-r06f16}/ab bash tools/gpu_ab.sh
