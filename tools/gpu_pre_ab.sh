# preprocess_fwd with the batch's cameras of a Gaussian slice dispatched
# together (exp_pre_cam_minor) vs camera-major (ctl = the product's flags):
# parity of the batch tests, interleaved timing, preprocess HBM reads.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-preab}
mkdir -p $O
GSPLAT_VARIANT=exp_pre_cam_minor timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_windows.py -k "not native" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
TAG=${TAG:-preab}/ab REPS=3 ENVS="GSPLAT_VARIANT=ctl GSPLAT_VARIANT=exp_pre_cam_minor" BENCH_ARGS="--steps 40" bash tools/gpu_env_ab.sh || exit 1
TAG=${TAG:-preab}/ab4 REPS=2 ENVS="GSPLAT_VARIANT=ctl GSPLAT_VARIANT=exp_pre_cam_minor" BENCH_ARGS="--cams 4 --steps 100" bash tools/gpu_env_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp
for v in ctl exp_pre_cam_minor; do
  GSPLAT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f_$v -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/f_$v.log 2>&1 || exit 1
  python3 -c "
import csv, collections, sys
t = collections.defaultdict(float); d = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name']
    if 'preprocess_fwd' in k and r['Counter_Name'].startswith('FETCH_SIZE'):
        t['preprocess_fwd'] += float(r['Counter_Value']); d['preprocess_fwd'].add(r['Dispatch_Id'])
print('$v', {k: round(2 * t[k] * 1024 / len(d[k]) / 1e9, 3) for k in t}, 'GB read per 27-camera launch (FETCH_SIZE x2)')
" $(find $O/f_$v -name "*counter_collection.csv") || exit 1
done
