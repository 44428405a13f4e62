# The per-camera drop-in (bench.py --mode percam) under rocprofv3: GPU busy
# fraction over the last timed steps at 1 and 4 streams (the traces are
# deleted after the analysis: they exceed what gpurun copies back).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05pc2}; mkdir -p $O
export TMPDIR=/tmp
for st in ${STREAMS:-1 4}; do
  GS_BENCH_OTHER=0 GS_BENCH_STREAMS=$st timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_s$st -o k --output-format csv -- \
    python bench.py --mode percam --steps 10 --warmup 3 --no-cpu-baseline > $O/percam_s$st.json 2> $O/percam_s$st.err || exit 1
  python -c "import json; d=json.load(open('$O/percam_s$st.json')); print('streams $st', d['value'], d['ms_per_step'])"
  f=$(ls $O/prof_s$st/*kernel_trace.csv $O/prof_s$st/*/*kernel_trace.csv 2>/dev/null | tail -1)
  echo "trace: $f"
  python tools/busy_fraction.py $f 270 > $O/busy_s$st.txt && cat $O/busy_s$st.txt
  python tools/kernel_split.py $f $O/split_s$st.json > /dev/null
  rm -rf $O/prof_s$st
done
