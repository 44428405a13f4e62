#!/usr/bin/env python3
"""Per-stage timing of the rasterizer on the bench scene (one or more cameras),
for kernel development: forward + backward through the raw _C boundary,
repeated, with the library's live stage timers.

    python tools/stage_bench.py --features 0 32 --cams 4 --reps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import _C, _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def run(P, F, W, H, cams, reps, compat, scale_mult=1.0, timing=True):
    dev = "cuda"
    g = make_gaussians(P, F=F, seed=0, scale_mult=scale_mult, device=dev)
    rig = camera_rig(27, W, H)[:cams]
    e = torch.Tensor([])
    gen = torch.Generator(device=dev).manual_seed(1)
    dc = torch.randn(3, H, W, device=dev, generator=gen)
    df = torch.randn(F, H, W, device=dev, generator=gen)
    dd = torch.randn(1, H, W, device=dev, generator=gen)
    da = torch.zeros(1, H, W, device=dev)
    cams_t = []
    for c in rig:
        cams_t.append(dict(bg=torch.zeros(3, device=dev),
                           view=torch.from_numpy(c.viewmatrix.copy()).to(dev),
                           proj=torch.from_numpy(c.projmatrix.copy()).to(dev),
                           campos=torch.from_numpy(c.campos.copy()).to(dev), c=c))
    sem = g.get("semantic_feature")

    def once():
        for ct in cams_t:
            c = ct["c"]
            out = _C.rasterize_gaussians(ct["bg"], g["means3D"], g["colors"], sem, g["opacities"],
                                         g["scales"], g["rotations"], 1.0, e, ct["view"], ct["proj"],
                                         c.c_x, c.c_y, c.tanfovx, c.tanfovy, H, W, e, 0, ct["campos"],
                                         False, False, compat=compat)
            L, color, feat, depth, alpha, radii, geom, binning, img = out
            _C.rasterize_gaussians_backward(ct["bg"], g["means3D"], radii, g["colors"], sem,
                                            g["scales"], g["rotations"], 1.0, e, ct["view"],
                                            ct["proj"], c.tanfovx, c.tanfovy, c.c_x, c.c_y, dc, df,
                                            dd, da, e, 0, ct["campos"], geom, L, binning, img, alpha,
                                            False, compat=compat)
        return L

    once()
    torch.cuda.synchronize()
    _lib.timing_enable(timing)
    s0 = torch.cuda.Event(enable_timing=True)
    s1 = torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(reps):
        L = once()
    s1.record()
    torch.cuda.synchronize()
    st = _lib.timing_read()
    _lib.timing_enable(False)
    n = reps * cams
    return {"P": P, "F": F, "W": W, "H": H, "L_last": L,
            "total_ms_per_cam": round(s0.elapsed_time(s1) / n, 4),
            "stages_ms_per_cam": {k: round(v[0] / n, 4) for k, v in st.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300_000)
    ap.add_argument("--features", type=int, nargs="+", default=[0, 32])
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--cams", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--compat", default="reference")
    ap.add_argument("--scale-mult", type=float, default=1.0)
    ap.add_argument("--no-timing", action="store_true", help="no stage events (total time only)")
    a = ap.parse_args()
    _lib.load()
    for F in a.features:
        print(json.dumps(run(a.gaussians, F, a.width, a.height, a.cams, a.reps, a.compat,
                             a.scale_mult, timing=not a.no_timing)), flush=True)


if __name__ == "__main__":
    main()
