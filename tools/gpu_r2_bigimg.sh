# tail-free proxy: one large camera (k^2 x the pixels of 800x800) vs 800x800 cameras
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/big
for wh in 800 2400 4160; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/big/w$wh -o k --output-format csv -- python3 $R/tools/stage_bench.py --features 32 --cams 1 --reps 3 --width $wh --height $wh --no-timing > $R/gpurun_out/big_$wh.log 2>&1 || exit 1
done
cd $R
for wh in 800 2400 4160; do
  f=$(find gpurun_out/big/w$wh -name k_kernel_stats.csv | head -1)
  python - "$f" $wh <<'PY'
import csv, sys
wh = int(sys.argv[2]); mp = wh * wh / 0.64e6
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "")
    if "render" in n or "sort" in n or "hist" in n or "preprocess" in n:
        print(wh, f"{n[:32]:32s} avg {float(r['AverageNs'])/1e3:9.1f} us  per 800x800-equiv {float(r['AverageNs'])/1e3/mp:8.2f} us")
PY
done
