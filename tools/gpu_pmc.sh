# PMC of the 27-camera batch launches: HBM traffic (FETCH_SIZE x2, WRITE_SIZE), instruction counts and memory-side atomic requests per camera
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcb
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmcb/*
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES" "TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $R/gpurun_out/pmcb/p$i -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $R/gpurun_out/pmcb/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmcb/p$i.log; exit 1; }
done
cd $R/tools
# the workload the counts belong to: bench.py attaches them only to a line of the same workload
export PMC_WORKLOAD='{"gaussians": 300000, "width": 800, "height": 800, "features": 32, "compat": "reference", "rig": 27, "cams_per_launch": 27, "seed": 0}'
python pmc_traffic.py $(find $R/gpurun_out/pmcb/p1 -name "*counter_collection.csv") $(find $R/gpurun_out/pmcb/p2 -name "*counter_collection.csv") 27
python pmc_valu.py $(find $R/gpurun_out/pmcb/p3 -name "*counter_collection.csv") 27
python pmc_atomic.py $(find $R/gpurun_out/pmcb/p4 -name "*counter_collection.csv") 27
