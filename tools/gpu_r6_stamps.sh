# Round 6: per-wave lifetime stamps of both blend kernels (stamps build) at
# the rank shape (4 cameras) and at 27 cameras, raw stamps dumped for the
# schedule analysis (tools/sched_sim.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-r06st}
mkdir -p $O
for c in ${CAMS:-4 27}; do
  GSPLAT_VARIANT=stamps timeout -k 10 300 python tools/batch_steps.py --cams $c --sync-free --reps 2 --stamps \
    --dump-stamps $O/stamps_c$c.npz > $O/stamps_c$c.txt 2> $O/stamps_c$c.err || { tail $O/stamps_c$c.err; exit 1; }
  tail -2 $O/stamps_c$c.txt | cut -c1-600
done
