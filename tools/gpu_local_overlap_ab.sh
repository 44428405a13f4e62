# One rank: the feature Adam step behind the next step's projection and
# binning (bench.py default) vs in line (GS_BENCH_OVERLAP=0): parameters
# after the timed steps against the run-to-run floor, then interleaved timing
# at 27 and 4 cameras.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-local_overlap}
mkdir -p $O
A="--steps 3 --warmup 1 --gaussians 100000 --cams 4 --width 400 --height 400 --no-cpu-baseline"
env GS_BENCH_OVERLAP=1 timeout -k 10 200 python bench.py $A --dump-params $O/l1.npz > $O/l1.json 2> $O/l1.err || { tail $O/l1.err; exit 1; }
env GS_BENCH_OVERLAP=0 timeout -k 10 200 python bench.py $A --dump-params $O/l0a.npz > $O/l0a.json 2> $O/l0a.err || exit 1
env GS_BENCH_OVERLAP=0 timeout -k 10 200 python bench.py $A --dump-params $O/l0b.npz > $O/l0b.json 2> $O/l0b.err || exit 1
python -c "import json; d=json.load(open('$O/l1.json')); print(d['config']['grad_exchange'])"
python tools/compare_params.py $O/l1.npz $O/l0a.npz $O/l0b.npz > $O/compare.txt; rc=$?
rm -f $O/*.npz
tail -1 $O/compare.txt
[ $rc = 0 ] || exit 1
TAG=${TAG:-local_overlap}/ab27 REPS=3 ENVS="GS_BENCH_OVERLAP=0 GS_BENCH_OVERLAP=1" BENCH_ARGS="--steps 40" bash tools/gpu_env_ab.sh || exit 1
TAG=${TAG:-local_overlap}/ab4 REPS=3 ENVS="GS_BENCH_OVERLAP=0 GS_BENCH_OVERLAP=1" BENCH_ARGS="--cams 4 --steps 100" bash tools/gpu_env_ab.sh || exit 1
