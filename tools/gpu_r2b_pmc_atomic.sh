# memory-side atomic requests of the batch blend kernels (TCC_EA0_ATOMIC_sum x 64 B)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmca
mkdir -p $O
rm -rf $O/*
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum -d $O/p1 -o pmc --output-format csv -- python3 $R/tools/batch_steps.py --reps 2 > $O/p1.log 2>&1 || { echo "pass failed"; tail -5 $O/p1.log; exit 1; }
f=$(find $O/p1 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    for key in ("render_bwd", "render_fwd", "preprocess_bwd"):
        if key in k:
            tot[key] += float(r["Counter_Value"]); n[key].add(r["Dispatch_Id"])
for k in tot:
    print(k, "atomic requests per launch", tot[k] / len(n[k]), "bytes (x64)", 64 * tot[k] / len(n[k]))
PY
