# Timing-only ceiling of a backward tile merge: the
# commits a free merge would leave (exp_merge_commits), the LDS it would
# add (exp_merge_lds), both, and no atomics at all, against the control.
# The exp_merge_* variants were removed from the kernels after the measurement
# (git show 81d9110 for their code).
set -o pipefail
mkdir -p gpurun_out/${TAG:-r04o} && cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && for v in exp_merge_commits; do GSPLAT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d $R/gpurun_out/${TAG:-r04o}/pmc_$v -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $R/gpurun_out/${TAG:-r04o}/pmc_$v.log 2>&1 || exit 1; done && cd $R && E="GSPLAT_VARIANT=ctl GSPLAT_VARIANT=exp_merge_commits GSPLAT_VARIANT=exp_merge_lds GSPLAT_VARIANT=exp_merge_both GSPLAT_VARIANT=exp_noatomic" && TAG=${TAG:-r04o}/ab27 REPS=2 ENVS="$E" bash tools/gpu_env_ab.sh && TAG=${TAG:-r04o}/ab4 REPS=2 ENVS="$E" BENCH_ARGS="--cams 4 --steps 60" bash tools/gpu_env_ab.sh && for v in exp_merge_commits; do python tools/pmc_atomic.py $(find gpurun_out/${TAG:-r04o}/pmc_$v -name "*counter_collection.csv") 27 > gpurun_out/${TAG:-r04o}/atomic_$v.json; done; ls gpurun_out/${TAG:-r04o}
