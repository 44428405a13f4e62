# Round 6: kernel traces of the 27-camera bench under two builds (VARIANTS)
# for the idle gap behind the plan header's kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r06gaps2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-ctl exp_nohdrfence}; do
  GSPLAT_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt_$v -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --cams ${CAMS:-27} --steps 10 --warmup 2 > $O/b_$v.json 2> $O/b_$v.err || { tail $O/b_$v.err; exit 1; }
done
