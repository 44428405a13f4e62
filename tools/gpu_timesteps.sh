# The per-timestep driver on the GPU: its tests, then tools/timesteps_run.py
# (configs[3] shape) on one rank and on two ranks sharing the GPU over gloo.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=$R/gpurun_out/${TAG:-timesteps}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_timesteps.py tests/test_timesteps.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/timesteps_run.py ${TS_ARGS:-} > $O/ts1.json 2> $O/ts1.err || { tail $O/ts1.err; exit 3; }
cat $O/ts1.json
GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 tools/timesteps_run.py ${TS_ARGS:-} > $O/ts2.json 2> $O/ts2.err || { tail $O/ts2.err; exit 4; }
cat $O/ts2.json
