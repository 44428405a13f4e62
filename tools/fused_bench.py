#!/usr/bin/env python3
"""Colour + seg per training step: the reference's two rasterizations
(train.py:145, train.py:246-249) against the fused single pass
(dynamic3dgaussians_amd.fused), forward + backward through the drop-in
GaussianRasterizer on the bench scene.  One JSON line per mode.

    python tools/fused_bench.py --gaussians 300000 --cams 8 --reps 5
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.fused import render_colour_and_seg  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings,  # noqa: E402
                                               GaussianRasterizer)
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300000)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--cams", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda"
    g = make_gaussians(a.gaussians, seed=0, device=dev)
    seg_colors = (torch.rand(a.gaussians, 3, device=dev) > 0.5).float()
    leaves = dict(means3D=g["means3D"], colors_precomp=g["colors"], opacities=g["opacities"],
                  scales=g["scales"], rotations=g["rotations"], seg_colors=seg_colors)
    leaves = {k: v.clone().requires_grad_(True) for k, v in leaves.items()}
    W, H = a.width, a.height
    settings = []
    for c in camera_rig(27, W, H)[:a.cams]:
        settings.append(GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x,
            c_y=c.c_y, bg=torch.zeros(3, device=dev), scale_modifier=1.0,
            viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
            projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
            campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference"))
    target = torch.rand(3, H, W, device=dev)
    geo = {k: leaves[k] for k in ("means3D", "opacities", "scales", "rotations")}

    def two_pass():
        for rs in settings:
            ras = GaussianRasterizer(rs)
            m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
            im, _, depth = ras(means2D=m2, colors_precomp=leaves["colors_precomp"], **geo)
            m2s = torch.zeros_like(leaves["means3D"], requires_grad=True)
            seg, _, _ = ras(means2D=m2s, colors_precomp=leaves["seg_colors"], **geo)
            ((im - target).abs().mean() + (seg - target).abs().mean() + depth.mean()).backward()

    def fused():
        for rs in settings:
            m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
            im, _, depth, seg = render_colour_and_seg(rs, means2D=m2, colors_precomp=leaves["colors_precomp"],
                                                      seg_colors=leaves["seg_colors"], **geo)
            ((im - target).abs().mean() + (seg - target).abs().mean() + depth.mean()).backward()

    for name, fn in (("two_pass", two_pass), ("fused", fused)):
        fn()
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.reps):
            fn()
        s1.record()
        torch.cuda.synchronize()
        ms = s0.elapsed_time(s1) / (a.reps * a.cams)
        print(json.dumps({"mode": name, "ms_per_camera": round(ms, 4), "gaussians": a.gaussians,
                          "W": W, "H": H, "cams": a.cams, "reps": a.reps}), flush=True)


if __name__ == "__main__":
    main()
