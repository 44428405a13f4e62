# HBM traffic of the 27-camera batch launches per build variant: FETCH_SIZE
# and WRITE_SIZE passes (separate rocprofv3 --pmc runs over batch_steps.py)
# (CAMS cameras per launch, default 27) for each of VARIANTS ("-" = the product library); one JSON per variant in
# gpurun_out/$TAG/traffic_<variant>.json, summary via tools/pmc_variants_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-pmcv}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:--}; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/${n}_$c
    GSPLAT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $c -d $O/${n}_$c -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 --cams ${CAMS:-27} > $O/${n}_$c.log 2>&1 || { echo "pass $n $c failed"; tail -5 $O/${n}_$c.log; exit 1; }
  done
  PMC_TRAFFIC_OUT=$O/traffic_$n.json python3 $R/tools/pmc_traffic.py $(find $O/${n}_FETCH_SIZE -name "*counter_collection.csv") $(find $O/${n}_WRITE_SIZE -name "*counter_collection.csv") ${CAMS:-27} || exit 1
done
python3 $R/tools/pmc_variants_summary.py $O
