# The tile sort's floor: the product's kernels (variant "ctl", the same
# ctypes binding) against two timing-only builds -- exp_sort_copy (each
# segment copied to the id list unsorted: the launch, its record and key
# loads and the list stores) and exp_sort_noins (the bucket sort without
# its insertion sorts) -- at the bench scene and at configs[4] per rank.
set -o pipefail
cd $GRAFT_REPO_ROOT
E="GSPLAT_VARIANT=ctl GSPLAT_VARIANT=exp_sort_copy GSPLAT_VARIANT=exp_sort_noins"
TAG=${TAG:-r05sfl}/bench REPS=2 ENVS="$E" BENCH_ARGS="--steps 20" bash tools/gpu_env_ab.sh || exit 1
TAG=${TAG:-r05sfl}/cfg4 REPS=2 ENVS="$E" BENCH_ARGS="--gaussians 1000000 --width 1920 --height 1080 --cams 4 --features 32 --steps 10 --warmup 3" bash tools/gpu_env_ab.sh || exit 2
