# kernel development loop on the GPU box: tests, stage timings, PMC counters
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 -p no:cacheprovider -x > gpurun_out/t3.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t3.log; exit 1; }
timeout -k 10 300 python tools/stage_bench.py --features 0 32 --cams 4 --reps 5 > gpurun_out/stage.jsonl 2> gpurun_out/stage.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex "render|preprocess|radix" -d $R/gpurun_out/pmc1 -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 1 --reps 1 > $R/gpurun_out/pmc1.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY --kernel-include-regex "render|preprocess|radix" -d $R/gpurun_out/pmc2 -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 1 --reps 1 > $R/gpurun_out/pmc2.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "render|preprocess|radix" -d $R/gpurun_out/pmc3 -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 1 --reps 1 > $R/gpurun_out/pmc3.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE TCC_EA0_ATOMIC_sum --kernel-include-regex "render|preprocess|radix" -d $R/gpurun_out/pmc4 -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 1 --reps 1 > $R/gpurun_out/pmc4.log 2>&1 || exit 6
