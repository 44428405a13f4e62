# Sync-free forward (gs_forward_batch): its GPU tests and the batch tests it
# now runs under, the default bench line, the 8 per-rank proxies (100-step
# windows) and a kernel trace of rank 5's proxy (tools/step_gaps.py).  (The
# header-path A/B it also ran, an in-stream copy of the headers, measured
# slower and was removed; DESIGN.md section 4 keeps the numbers.)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r05sf}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  ${TESTS:-tests/test_gpu_sync_free.py tests/test_gpu_batch.py tests/test_gpu_windows.py tests/test_gpu_raw_params.py} \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 2; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'])"
for rep in 1 2; do
for r in ${RANKS:-0 1 2 3 4 5 6 7}; do
  f=$O/proxy_r${r}_$rep.json
  timeout -k 10 200 python bench.py --cams-total 27 --proxy-world 8 --proxy-rank $r --no-cpu-baseline \
    --steps 100 --warmup 10 > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 3; }
  python -c "import json; d=json.load(open('$f')); print('proxy', $r, $rep, d['ms_per_step'])"
done
done
cd /tmp && export TMPDIR=/tmp
rm -rf $O/tr5
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr5 -o tr --output-format csv -- python3 $R/bench.py \
  --cams-total 27 --proxy-world 8 --proxy-rank 5 --no-cpu-baseline --steps 30 --warmup 5 \
  > $O/tr5.json 2> $O/tr5.err || { tail -5 $O/tr5.err; exit 5; }
cd $R && python tools/step_gaps.py $O/tr5/tr_kernel_trace.csv > $O/tr5_gaps.txt && head -3 $O/tr5_gaps.txt
