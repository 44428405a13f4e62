# parity tests, stage timings, then PMC counters of the blend kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider > gpurun_out/tq.log 2>&1; echo "tests exit $?" >> gpurun_out/tq.log
timeout -k 10 300 python tools/stage_bench.py --features 0 32 --cams 4 --reps 5 > gpurun_out/stage.jsonl 2> gpurun_out/stage.err || exit 2
cd /tmp && export TMPDIR=/tmp
for F in 0 32; do
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA --kernel-include-regex "render" -d $R/gpurun_out/pmcA$F -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features $F --cams 1 --reps 1 > $R/gpurun_out/pmcA$F.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-include-regex "render" -d $R/gpurun_out/pmcB$F -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features $F --cams 1 --reps 1 > $R/gpurun_out/pmcB$F.log 2>&1 || exit 4
done
