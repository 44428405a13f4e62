# Round 6: kernel trace of the bench step at 27 and at 4 cameras, for the
# GPU idle gaps between launches (tools/step_gaps.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06gaps}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in 4 27; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt$c -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --cams $c --steps 10 --warmup 2 > $O/b$c.json 2> $O/b$c.err || { tail $O/b$c.err; exit 1; }
done
cd $R && ls $O/kt4 $O/kt27
