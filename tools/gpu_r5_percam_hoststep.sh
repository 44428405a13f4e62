set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05hs2; mkdir -p $O
for rep in 1 2 3 4; do
  for v in 0 1; do
    GS_PERCAM_SYNC_FREE=$v timeout -k 10 120 python tools/host_step.py --mode percam --steps 300 > $O/hs_sf${v}_$rep.txt 2>&1 || exit 1
    echo "sf=$v $rep $(tail -1 $O/hs_sf${v}_$rep.txt)"
  done
done
