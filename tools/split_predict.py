#!/usr/bin/env python3
"""Predicted BASELINE configs[3] step at N ranks from single-GPU bench lines:
the 27-camera rig split camera c -> rank c mod N makes the busiest rank
render ceil(27 / N) cameras, so the split step is that rank's measured step
(bench.py --cams ceil(27/N): the same per-rank work, its own all-reduce
excluded) plus the gradient all-reduce of the bucket -- 46 fp32 per Gaussian
at F = 32 (means3D 3, rgb 3, rotation 4, opacity 1, scale 3, features 32) and
the 2 densification statistics -- as a ring all-reduce, 2 (N - 1) / N x bytes
over a bus rate.  Rates stated: one xGMI link (153 GB/s, a single ring on the
point-to-point fabric) and 300 GB/s (RCCL's rings over several of the 7
links).  With bench.py's overlapped exchange (N > 1, F > 0: the geometry
bucket, 14 fp32 per Gaussian, all-reduced before Adam; the feature bucket
all-reduced and stepped on a side stream while the next step projects and
bins, the blend waiting on gs_gaussians.feature_ready) only the geometry
all-reduce and the part of the feature all-reduce longer than the rank's
pre-blend stages (preprocess .. ranges of its stages_ms_per_step) stay on
the step.

    python tools/split_predict.py full.json cams4.json cams3.json [N=8] [P=300000] [F=32]
"""
import json
import math
import sys


def main():
    full, c4, c3 = (json.load(open(p)) for p in sys.argv[1:4])
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    P = int(sys.argv[5]) if len(sys.argv) > 5 else 300_000
    F = int(sys.argv[6]) if len(sys.argv) > 6 else 32
    busiest = math.ceil(27 / n)
    per_rank = {4: c4, 3: c3}[busiest]
    bucket = P * (3 + 3 + 4 + 1 + 3 + F + 2) * 4
    out = {"n_ranks": n, "busiest_rank_cams": busiest, "per_rank_ms": per_rank["ms_per_step"],
           "single_gpu_27cam_ms": full["ms_per_step"], "bucket_bytes": bucket, "predictions": {}}
    for rate in (153.0, 300.0):
        ar = 2 * (n - 1) / n * bucket / (rate * 1e9) * 1e3
        step = per_rank["ms_per_step"] + ar
        out["predictions"][f"{int(rate)}GB/s"] = {"allreduce_ms": round(ar, 3), "step_ms": round(step, 3),
                                                 "speedup_vs_1gpu": round(full["ms_per_step"] / step, 2)}
        geo = 2 * (n - 1) / n * P * 14 * 4 / (rate * 1e9) * 1e3
        feat = 2 * (n - 1) / n * P * F * 4 / (rate * 1e9) * 1e3
        st = per_rank.get("stages_ms_per_step", {})
        pre_blend = sum(st.get(k, 0.0) for k in ("preprocess", "scan", "duplicate", "sort", "ranges"))
        exposed = geo + max(0.0, feat - pre_blend)
        step = per_rank["ms_per_step"] + exposed
        out["predictions"][f"{int(rate)}GB/s overlapped"] = {
            "geometry_allreduce_ms": round(geo, 3), "feature_allreduce_ms": round(feat, 3),
            "pre_blend_ms": round(pre_blend, 3), "exposed_ms": round(exposed, 3), "step_ms": round(step, 3),
            "speedup_vs_1gpu": round(full["ms_per_step"] / step, 2)}
    out["target"] = {"speedup": 6.0, "step_ms": round(full["ms_per_step"] / 6.0, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
