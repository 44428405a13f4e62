# Round evidence of the current tree on one MI355X, one command:
#   1. PMC passes of the 27-camera batch launches (gpu_pmc.sh) -> profiles/pmc_*.json
#      (read by bench.py's roofline.traffic / issue / atomics)
#   2. the GPU suite and smoke()
#   3. the default bench line (CPU baselines included)
#   4. rocprofv3 --kernel-trace --stats of the same bench command
#   5. a two-rank rehearsal of bench.py's distributed path on the one GPU
#      (gloo): the weak headline + the 27-camera split step, and --cams-total 27;
#      tools/timesteps_run.py (configs[3] shape) on one rank and on two;
#      the overlapped feature exchange against the serial one, over gloo
#      (two ranks) and over RCCL (one rank), tools/gpu_overlap_rehearsal.sh
# Outputs in gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-round}
O=$R/gpurun_out/$TAG
mkdir -p $O
if [ "${SKIP_PMC:-0}" != "1" ]; then
timeout -k 10 600 bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc.log; exit 1; }
cp profiles/pmc_traffic.json profiles/pmc_valu.json profiles/pmc_atomic.json $O/
tail -3 $O/pmc.log
fi
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 4; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $O/bprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/bprof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/bench_under_rocprof.json 2> $O/bprof.err || exit 5
cat $O/bench_under_rocprof.json
fi
cd $R
if [ "${SKIP_DIST:-0}" != "1" ]; then
GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 > $O/dist2_weak.json 2> $O/dist2_weak.err || { tail $O/dist2_weak.err; exit 6; }
GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 3 --warmup 1 --cams-total 27 > $O/dist2_strong.json 2> $O/dist2_strong.err || { tail $O/dist2_strong.err; exit 7; }
cat $O/dist2_weak.json $O/dist2_strong.json
# configs[3] shape: the timestep driver, one rank and two ranks (gloo, one GPU)
timeout -k 10 300 python tools/timesteps_run.py > $O/ts1.json 2> $O/ts1.err || { tail $O/ts1.err; exit 8; }
GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tools/timesteps_run.py > $O/ts2.json 2> $O/ts2.err || { tail $O/ts2.err; exit 9; }
cat $O/ts1.json $O/ts2.json
TAG=$TAG/overlap timeout -k 10 900 bash tools/gpu_overlap_rehearsal.sh > $O/overlap.log 2>&1 || { tail -30 $O/overlap.log; exit 10; }
grep -E "OK|MISMATCH|exchange" $O/overlap.log
fi
