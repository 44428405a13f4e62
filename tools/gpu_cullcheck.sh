# exact strip culling vs box culling: bitwise comparison of the bench forward outputs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python tools/cull_check.py > gpurun_out/cc_default.log 2>&1 || exit 1
GSPLAT_VARIANT=exp_boxcull timeout -k 10 300 python tools/cull_check.py > gpurun_out/cc_box.log 2>&1 || exit 2
python - <<'PY' > gpurun_out/cullcheck.txt
import numpy as np
a = np.load("gpurun_out/cull_default.npz"); b = np.load("gpurun_out/cull_exp_boxcull.npz")
for k in a.files:
    print(k, "identical" if np.array_equal(a[k], b[k]) else f"DIFF max {np.abs(a[k]-b[k]).max()}")
PY
rm -f gpurun_out/cull_default.npz gpurun_out/cull_exp_boxcull.npz
