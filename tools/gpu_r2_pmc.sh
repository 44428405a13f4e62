# PMC stall breakdown of the stage kernels (separate passes; --pmc only with kernel-trace-free runs)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > $R/gpurun_out/pmc2/counters.txt 2>&1 || true
i=0
for set in "${PMC1:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES}" "${PMC2:-SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_WAVES}" "${PMC3:-GRBM_GUI_ACTIVE GRBM_COUNT}"; do
  i=$((i+1))
  GSPLAT_VARIANT=${VARIANT:-} timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmc2/p$i -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmc2/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc2/p$i.log; exit 1; }
done
echo pmc done
