# Effective shader clock of the blend kernels (tools/pmc_clock.py): one
# rocprofv3 run per camera count with GRBM_GUI_ACTIVE and the kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-clock}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${CAMS:-27 4}; do
  rm -rf $O/c$c
  timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $O/c$c -o run --output-format csv -- python3 $R/tools/batch_steps.py --cams $c --reps 4 > $O/c$c.log 2>&1 || { tail -5 $O/c$c.log; exit 1; }
  python3 $R/tools/pmc_clock.py $(find $O/c$c -name "*counter_collection.csv") $(find $O/c$c -name "*kernel_trace.csv") > $O/clock_c$c.json || exit 1
  head -c 1500 $O/clock_c$c.json; echo
done
