set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  TAG=r05d2/s$i LIMIT=150 TB=40 bash tools/gpu_r5_dist2.sh || exit 1
  TAG=r05d2/w$i LIMIT=150 TB=40 NAMES=dist2_weak ARGS=" " bash tools/gpu_r5_dist2.sh || exit 2
done
