# wave-lifetime shares of the blend kernels (stamps build) + kernel durations of
# the stamps and product builds on the same batch program
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/stamps
mkdir -p $O
GSPLAT_VARIANT=stamps timeout -k 10 200 python tools/batch_steps.py --reps 2 --stamps > $O/stamps.log 2>&1 || { tail $O/stamps.log; exit 1; }
cat $O/stamps.log
cd /tmp && export TMPDIR=/tmp
for v in stamps -; do
  n=$v; [ "$v" = "-" ] && v="" && n=product
  rm -rf $O/prof_$n
  GSPLAT_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o k --output-format csv -- python3 $R/tools/batch_steps.py --reps 3 > $O/prof_$n.log 2>&1 || { tail $O/prof_$n.log; exit 2; }
  f=$(find $O/prof_$n -name "*kernel_stats.csv" | head -1)
  python3 -c "import csv; [print(\"$n\", r[\"Name\"][:40], r[\"Calls\"], round(float(r[\"AverageNs\"])/1e3, 1)) for r in csv.DictReader(open(\"$f\")) if \"render_\" in r[\"Name\"]]"
done
