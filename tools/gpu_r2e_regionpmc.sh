# PMC of the 16x8-region backward (variant exp_region) vs the strip kernel:
# memory-side atomic requests, instruction counts, wave states.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/regpmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in exp_region -; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  i=0
  for set in "TCC_EA0_ATOMIC_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    GSPLAT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $set -d $O/${n}_p$i -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/${n}_p$i.log 2>&1 || { echo "pass $n $i failed"; tail -5 $O/${n}_p$i.log; exit 1; }
  done
  (cd $R/tools && python pmc_generic.py 27 $(find $O/${n}_p1 $O/${n}_p2 -name "*counter_collection.csv")) > $O/$n.json
  python -c "import json; d=json.load(open('$O/$n.json'))['kernels']; print('$n', {k: d[k] for k in d if 'render_bwd' in k})"
done
