# atomics headroom in batch mode + atomic PMC counters of the backward blend
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
for v in "" exp_noatomic ""; do
  GSPLAT_VARIANT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --mode batch > gpurun_out/atom_$v.json 2> gpurun_out/atom.err || { tail -5 gpurun_out/atom.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/atom_$v.json')); print('variant=$v', d['value'], d['ms_per_step'], {k: round(v,3) for k, v in d['stages_ms_per_step'].items()})"
done
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_atom
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_EA0_ATOMIC_LEVEL_sum -d $R/gpurun_out/pmc_atom/p1 -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmc_atom_p1.log 2>&1 || { echo p1 failed; tail -3 $R/gpurun_out/pmc_atom_p1.log; exit 2; }
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_atom/p2 -o pmc --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 2 --reps 1 --no-timing > $R/gpurun_out/pmc_atom_p2.log 2>&1 || { echo p2 failed; tail -3 $R/gpurun_out/pmc_atom_p2.log; exit 3; }
cd $R
for p in p1 p2; do f=$(find gpurun_out/pmc_atom/$p -name "*counter_collection.csv" | head -1); python tools/pmc_summary.py $f | grep -E "render_bwd|render_fwd"; done
