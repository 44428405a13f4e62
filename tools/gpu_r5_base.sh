# Round-5 baseline of the tree on one MI355X: the default bench line, the 8
# per-rank proxies of the 27-camera windows split (100-step windows, host
# step times), and rocprofv3 kernel traces of two proxies (ranks 0 and 5) for
# tools/step_trace.py.  Outputs in gpurun_out/$TAG.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r05base}
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'])"
for r in ${RANKS:-0 1 2 3 4 5 6 7}; do
  f=$O/proxy_r$r.json
  timeout -k 10 200 python bench.py --cams-total 27 --proxy-world 8 --proxy-rank $r --no-cpu-baseline \
    --steps 100 --warmup 10 --step-times > $f 2> ${f%.json}.err || { tail -5 ${f%.json}.err; exit 2; }
  python -c "import json; d=json.load(open('$f')); print('proxy', $r, d['ms_per_step'], d['config']['cams_per_rank'])"
done
cd /tmp && export TMPDIR=/tmp
for r in ${TRACE_RANKS:-0 5}; do
  rm -rf $O/tr$r
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr$r -o tr --output-format csv -- python3 $R/bench.py \
    --cams-total 27 --proxy-world 8 --proxy-rank $r --no-cpu-baseline --steps 30 --warmup 5 \
    > $O/tr$r.json 2> $O/tr$r.err || { tail -5 $O/tr$r.err; exit 3; }
  python -c "import json; d=json.load(open('$O/tr$r.json')); print('traced proxy', $r, d['ms_per_step'])"
done
