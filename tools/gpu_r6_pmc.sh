# Round 6: the 27-camera batch kernels' PMC on the workload they claim
# (tools/batch_steps.py: two-phase forward, every rep one launch per stage of
# the same work; tools/pmc_*.py refuse uneven launches) -> profiles/pmc_*.json,
# then the blend kernels' wave-cycle split (tools/pmc_split.py: issuing /
# parked at s_waitcnt or a barrier / issue-stalled, instruction mix, LDS, the
# VALU+MFMA co-execution) and their effective clock (GRBM_GUI_ACTIVE over the
# kernel trace, tools/pmc_clock.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES" "TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  rm -rf $O/p$i
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
cd $R/tools
export PMC_WORKLOAD='{"gaussians": 300000, "width": 800, "height": 800, "features": 32, "compat": "reference", "rig": 27, "cams_per_launch": 27, "seed": 0}'
python pmc_traffic.py $(find $O/p1 -name "*counter_collection.csv") $(find $O/p2 -name "*counter_collection.csv") 27 || exit 2
python pmc_valu.py $(find $O/p3 -name "*counter_collection.csv") 27 || exit 2
python pmc_atomic.py $(find $O/p4 -name "*counter_collection.csv") 27 || exit 2
cp $R/profiles/pmc_traffic.json $R/profiles/pmc_valu.json $R/profiles/pmc_atomic.json $O/
cd /tmp
j=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR" \
           "SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES"; do
  j=$((j+1))
  rm -rf $O/s$j
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "render_(fwd|bwd)" -d $O/s$j -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/s$j.log 2>&1 || { echo "split pass $j failed"; tail -5 $O/s$j.log; exit 3; }
done
cd $R && python tools/pmc_split.py $(find $O/s1 -name "*counter_collection.csv") $(find $O/s2 -name "*counter_collection.csv") $(find $O/s3 -name "*counter_collection.csv") > $O/blend_split.json || exit 4
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $O/clk -o run --output-format csv -- python3 $R/tools/batch_steps.py --reps 4 > $O/clk.log 2>&1 || { tail -5 $O/clk.log; exit 5; }
cd $R && python3 tools/pmc_clock.py $(find $O/clk -name "*counter_collection.csv") $(find $O/clk -name "*kernel_trace.csv") > $O/clock.json || exit 6
cat $O/blend_split.json | head -80
