#!/usr/bin/env python3
"""Work counters of the blend kernels on the bench scene (stats build variant).

    GSPLAT_VARIANT=stats python -m dynamic3dgaussians_amd.build --force   # here
    python tools/render_stats.py --features 32 --cams 2                  # on the box

Counters (per camera): chunks, records gathered, strip survivors, inner-loop
iterations, iterations with >=1 active lane, active lanes -- forward and
backward -- plus waves and list lengths.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

os.environ["GSPLAT_VARIANT"] = "stats"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dynamic3dgaussians_amd import _lib  # noqa: E402
from tools.stage_bench import run  # noqa: E402

NAMES = {0: "fwd_chunks", 1: "fwd_records", 2: "fwd_survivors", 3: "fwd_iters",
         4: "fwd_iters_active", 5: "fwd_active_lanes", 6: "fwd_waves", 7: "fwd_list_total",
         18: "fwd_iters_one_half_active", 8: "bwd_chunks", 9: "bwd_records", 10: "bwd_survivors", 11: "bwd_iters",
         12: "bwd_iters_active", 13: "bwd_active_lanes", 14: "bwd_waves", 15: "bwd_walk_total"}
MAXES = {16: "fwd_wave_iters_max", 17: "bwd_wave_iters_max"}
HISTS = {20: "fwd_wave_iters_hist", 25: "bwd_wave_iters_hist"}  # <256,<512,<1024,<2048,more


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--cams", type=int, default=2)
    ap.add_argument("--gaussians", type=int, default=300_000)
    ap.add_argument("--scale-mult", type=float, default=1.0)
    a = ap.parse_args()
    L = _lib.load(auto_build=False)
    L.gs_stats_reset.restype = ctypes.c_int
    L.gs_stats_read.restype = ctypes.c_int
    L.gs_stats_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    # warm-up inside run() executes once more than reps: reset after a first call
    run(a.gaussians, a.features, 800, 800, a.cams, 1, "reference", a.scale_mult)
    torch.cuda.synchronize()
    assert L.gs_stats_reset() == 0
    res = run(a.gaussians, a.features, 800, 800, a.cams, 1, "reference", a.scale_mult)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    assert L.gs_stats_read(buf, 32) == 0
    n = 2 * a.cams  # run() = warm-up pass + 1 timed pass
    out = {NAMES[i]: round(buf[i] / n) for i in NAMES}
    out.update({MAXES[i]: buf[i] for i in MAXES})
    out.update({HISTS[i]: [round(buf[i + k] / n) for k in range(5)] for i in HISTS})
    out["L_per_cam"] = res["L_last"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
