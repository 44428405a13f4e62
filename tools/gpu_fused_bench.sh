# GPU suite, then the fused colour + seg pass at F = 32 (+ seg) against the
# plain F = 32 render and the two-pass step (tools/fused_bench.py), product
# and VARIANTS.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-fused}
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
fi
for v in - ${VARIANTS:-}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 300 python -u tools/fused_bench.py --features 32 --cams 8 --reps 5 > $O/fused_$n.jsonl 2> $O/fused_$n.err || { tail $O/fused_$n.err; exit 2; }
  echo "== $n"; cat $O/fused_$n.jsonl
done
