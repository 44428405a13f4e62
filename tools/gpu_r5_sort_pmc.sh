# Where the binning kernels' time goes: two PMC passes over the 27-camera
# batch launches (tools/batch_steps.py), restricted to the tile sort, bucket
# and count kernels -- the wave-cycle split (active / parked at s_waitcnt or a
# barrier / issue-stalled), instruction counts and the LDS array's cycles.
# Summarised per kernel by tools/pmc_split.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r05spmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  rm -rf $O/p$i
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "tile_(sort|bucket|hist|rowscan)" -d $O/p$i -o pmc \
    --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
cd $R && python tools/pmc_split.py $(find $O/p1 -name "*counter_collection.csv") $(find $O/p2 -name "*counter_collection.csv") > $O/split.txt && cat $O/split.txt
