# XCD rotation of the strip units at every camera count (product) vs only
# below 8 cameras (exp_rot_small_c), 27-camera step, interleaved; plus the
# render_fwd / render_bwd HBM reads of each (FETCH_SIZE x 2).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-rotab}
mkdir -p $O
TAG=${TAG:-rotab}/ab REPS=3 ENVS="GSPLAT_VARIANT=ctl GSPLAT_VARIANT=exp_rot_small_c" BENCH_ARGS="--steps 40" bash tools/gpu_env_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for v in ctl exp_rot_small_c; do
  GSPLAT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$v -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/f_$v.log 2>&1 || exit 1
  python3 -c "
import csv, collections, sys
t = collections.defaultdict(float); d = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    for k in ('render_fwd', 'render_bwd'):
        if k in r['Kernel_Name'] and r['Counter_Name'].startswith('FETCH_SIZE'):
            t[k] += float(r['Counter_Value']); d[k].add(r['Dispatch_Id'])
print('$v', {k: round(2 * t[k] * 1024 / len(d[k]) / 1e9, 3) for k in t}, 'GB read per 27-camera launch (FETCH_SIZE x2)')
" $(find $O/f_$v -name "*counter_collection.csv") || exit 1
done
