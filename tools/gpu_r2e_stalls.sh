# Where the blend waves wait: SQ wave-state counters of the 27-camera batch
# launches (one rocprofv3 --pmc pass per counter set), the counter list of the
# box, and the blend kernels' work counters (stats build).  -> gpurun_out/stalls
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/stalls
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters_avail.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 $O/p$i.log; [ $rc -eq 1 ] || exit 1; fi
done
cd $R/tools
python pmc_generic.py 27 $(find $O -name "*counter_collection.csv") > $O/stalls.json && cat $O/stalls.json
cd $R
if [ -f dynamic3dgaussians_amd/lib/libgsplat_hip_stats.so ]; then
  timeout -k 10 300 python tools/render_stats.py --features 32 --cams 27 > $O/render_stats.json 2> $O/render_stats.err || tail -5 $O/render_stats.err
  cat $O/render_stats.json
fi
