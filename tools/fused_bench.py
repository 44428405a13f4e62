#!/usr/bin/env python3
"""Colour + seg per training step: the reference's two rasterizations
(train.py:145, train.py:246-249) against the fused single pass
(dynamic3dgaussians_amd.fused), forward + backward through the drop-in
GaussianRasterizer on the bench scene.  One JSON line per mode:
  plain     the colour render alone (no seg; the floor),
  two_pass  colour render + the seg render (the reference's step),
  fused     one pass with the seg colours as extra feature channels.
With --features 32 the colour render is the G3 call of dyn_train.py:244
(32 semantic channels + label): the fused pass is then F = 3 + 32 = 35,
run by the F = 36 instantiation (32 matrix-core channels + a VALU tail).

    python tools/fused_bench.py --gaussians 300000 --cams 8 --reps 5 [--features 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import _lib  # noqa: E402
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
    ap.add_argument("--features", type=int, default=0)
    a = ap.parse_args()
    dev = "cuda"
    g = make_gaussians(a.gaussians, F=a.features, seed=0, device=dev)
    seg_colors = (torch.rand(a.gaussians, 3, device=dev) > 0.5).float()
    leaves = dict(means3D=g["means3D"], colors_precomp=g["colors"], opacities=g["opacities"],
                  scales=g["scales"], rotations=g["rotations"], seg_colors=seg_colors)
    if a.features:
        leaves["semantic_feature"] = g["semantic_feature"]
    leaves = {k: v.clone().requires_grad_(True) for k, v in leaves.items()}
    label = torch.ones(a.gaussians, device=dev)
    ftarget = torch.rand(a.features, a.height, a.width, device=dev) if a.features else None
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

    def colour_render(ras):
        m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
        if a.features:   # G3: label + semantic features
            im, _, feat, depth, _ = ras(means2D=m2, colors_precomp=leaves["colors_precomp"],
                                        semantic_feature=leaves["semantic_feature"], label=label, **geo)
            return (im - target).abs().mean() + depth.mean() + (feat - ftarget).abs().mean()
        im, _, depth = ras(means2D=m2, colors_precomp=leaves["colors_precomp"], **geo)
        return (im - target).abs().mean() + depth.mean()

    def plain():
        for rs in settings:
            colour_render(GaussianRasterizer(rs)).backward()

    def two_pass():
        for rs in settings:
            ras = GaussianRasterizer(rs)
            loss = colour_render(ras)
            m2s = torch.zeros_like(leaves["means3D"], requires_grad=True)
            seg, _, _ = ras(means2D=m2s, colors_precomp=leaves["seg_colors"], **geo)
            (loss + (seg - target).abs().mean()).backward()

    def fused():
        for rs in settings:
            m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
            out = render_colour_and_seg(rs, means2D=m2, colors_precomp=leaves["colors_precomp"],
                                        seg_colors=leaves["seg_colors"], semantic_feature=leaves.get("semantic_feature"),
                                        label=label if a.features else None, **geo)
            im, _, depth, seg = out[:4]
            loss = (im - target).abs().mean() + (seg - target).abs().mean() + depth.mean()
            if a.features:
                loss = loss + (out[4] - ftarget).abs().mean()
            loss.backward()

    for name, fn in (("plain", plain), ("two_pass", two_pass), ("fused", fused)):
        fn()
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.reps):
            fn()
        s1.record()
        torch.cuda.synchronize()
        ms = s0.elapsed_time(s1) / (a.reps * a.cams)
        # per-stage device times of one more pass (live HIP events)
        _lib.timing_enable(True)
        fn()
        torch.cuda.synchronize()
        st = {k: round(v[0] / a.cams, 4) for k, v in _lib.timing_read().items() if v[1]}
        _lib.timing_enable(False)
        print(json.dumps({"mode": name, "ms_per_camera": round(ms, 4), "stages_ms_per_camera": st,
                          "gaussians": a.gaussians, "features": a.features, "W": W, "H": H, "cams": a.cams,
                          "reps": a.reps}), flush=True)


if __name__ == "__main__":
    main()
