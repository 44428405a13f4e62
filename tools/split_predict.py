#!/usr/bin/env python3
"""Predicted BASELINE configs[3] step at N ranks from single-GPU bench lines.

Each rank of the N-rank split of the 27-camera rig is measured on one GPU as
a proxy (bench.py --cams-total 27 --proxy-world N --proxy-rank r: exactly
that rank's cameras and tile windows, the same per-rank work, no
collective).  The predicted split step is the slowest rank's step (median of
its runs) plus the exposed gradient exchange:
  * serial: the whole gradient bucket -- 46 fp32 per Gaussian at F = 32
    (means3D 3, rgb 3, rotation 4, opacity 1, scale 3, features 32) and the
    2 densification statistics -- as a ring all-reduce, 2 (N - 1) / N x bytes
    over a bus rate;
  * overlapped (bench.py's exchange at N > 1, F > 0): the geometry bucket
    (14 fp32 per Gaussian) exchanged before the next step, the feature bucket
    exchanged and stepped on a side stream behind the next step's
    projection and binning (gs_gaussians.feature_ready), so only the part of
    it longer than the rank's pre-blend stages stays exposed.  With the
    sharded Adam (distributed.ShardedAdam, the default for a rank of N) an
    exchange is a reduce-scatter and an all-gather: (N - 1) / N x bytes
    each, the ring all-reduce's 2 (N - 1) / N in total, so the same bus
    time; the proxies run the rank's 1/N Adam slice.
Rates: one xGMI link (153 GB/s, a single ring on the point-to-point fabric)
and 300 GB/s (RCCL's rings over several of the 7 links).  The proxies also
run the feature Adam step in line, which the overlapped exchange moves to
the side stream: the prediction is conservative there.

    python tools/split_predict.py full.json proxy.json [proxy.json ...] [--n 8] [--P 300000] [--F 32]

`full.json`: the single-GPU 27-camera bench line the speed-up is quoted
against; the proxies: any number of runs of any ranks (the rank is read from
config.workload).
"""
import argparse
import json
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("full")
    ap.add_argument("proxies", nargs="+")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--P", type=int, default=300_000)
    ap.add_argument("--F", type=int, default=32)
    a = ap.parse_args()
    full = json.load(open(a.full))
    ranks = {}
    for p in a.proxies:
        d = json.load(open(p))
        m = re.match(r"rank (\d+) of (\d+)", d["config"]["workload"])
        if not m or int(m.group(2)) != a.n:
            raise SystemExit(f"{p}: not a proxy of an {a.n}-rank split")
        ranks.setdefault(int(m.group(1)), []).append(d)
    per_rank = {r: statistics.median(x["ms_per_step"] for x in v) for r, v in sorted(ranks.items())}
    slow = max(per_rank, key=per_rank.get)
    slow_runs = ranks[slow]
    step_rank = per_rank[slow]
    st = slow_runs[0].get("stages_ms_per_step", {})
    pre_blend = sum(st.get(k, 0.0) for k in ("preprocess", "scan", "duplicate", "sort", "ranges"))
    n, P, F = a.n, a.P, a.F
    bucket = P * (3 + 3 + 4 + 1 + 3 + F + 2) * 4
    out = {"n_ranks": n, "ranks_measured": sorted(per_rank), "runs_per_rank": {r: len(v) for r, v in ranks.items()},
           "per_rank_ms": {r: round(v, 4) for r, v in per_rank.items()},
           "per_rank_runs_ms": {r: [x["ms_per_step"] for x in v] for r, v in ranks.items()},
           "slowest_rank": slow, "slowest_rank_ms": round(step_rank, 4),
           "single_gpu_27cam_ms": full["ms_per_step"], "bucket_bytes": bucket, "predictions": {}}
    for rate in (153.0, 300.0):
        ar = 2 * (n - 1) / n * bucket / (rate * 1e9) * 1e3
        step = step_rank + ar
        out["predictions"][f"{int(rate)}GB/s serial"] = {
            "allreduce_ms": round(ar, 3), "step_ms": round(step, 4),
            "speedup_vs_1gpu": round(full["ms_per_step"] / step, 3)}
        geo = 2 * (n - 1) / n * P * 14 * 4 / (rate * 1e9) * 1e3
        feat = 2 * (n - 1) / n * P * F * 4 / (rate * 1e9) * 1e3
        exposed = geo + max(0.0, feat - pre_blend)
        step = step_rank + exposed
        out["predictions"][f"{int(rate)}GB/s overlapped"] = {
            "geometry_bytes": P * 14 * 4, "geometry_allreduce_ms": round(geo, 3),
            "feature_allreduce_ms": round(feat, 3), "pre_blend_ms": round(pre_blend, 3),
            "exposed_ms": round(exposed, 3), "step_ms": round(step, 4),
            "speedup_vs_1gpu": round(full["ms_per_step"] / step, 3)}
    out["target"] = {"speedup": 6.0, "step_ms": round(full["ms_per_step"] / 6.0, 4),
                     "rank_bar_ms_at_300GBs": round(full["ms_per_step"] / 6.0
                                                    - out["predictions"]["300GB/s overlapped"]["exposed_ms"], 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
