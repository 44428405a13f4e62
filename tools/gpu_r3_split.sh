# Round 3: fp32-equivalent (3-piece bf16 split) blend contractions.
# GPU suite, measured parity errors (product and the round-2 two-piece split),
# and an interleaved bench A/B of the two (27-camera batch, F = 32).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r03b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/tests.log
tail -3 $O/tests.log
grep -q "tests rc=0" $O/tests.log || grep -q "failed" $O/tests.log || exit 1
timeout -k 10 300 python -u tools/parity_errors.py > $O/parity_split3.jsonl 2> $O/parity_split3.err || { tail $O/parity_split3.err; exit 2; }
GSPLAT_VARIANT=exp_split2 timeout -k 10 300 python -u tools/parity_errors.py > $O/parity_split2.jsonl 2> $O/parity_split2.err || { tail $O/parity_split2.err; exit 3; }
for rep in 1 2; do
for v in - exp_split2; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  GSPLAT_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${n}_$rep.json 2> $O/b_${n}_$rep.err || { tail -5 $O/b_${n}_$rep.err; exit 4; }
  python -c "import json; d=json.load(open('$O/b_${n}_$rep.json')); print('bench', '$n', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
done
