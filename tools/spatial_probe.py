#!/usr/bin/env python3
"""Probe: does a spatially coherent Gaussian order speed up the binning
passes?  The tile plan and bucket passes walk the Gaussians in index order,
TB_BLOCKS contiguous slices per camera; with the scene in random order every
slice touches the whole screen, so each block's per-tile runs are a few keys
long (the bucket pass's stores scatter; at configs[4] its keys exceed the LDS
and every key is its own store).  Here the same scene is rendered in its own
order and permuted into 3-D Morton order of the means (30-bit codes, torch
argsort), interleaved, and the live stage times compared.  Results do not
depend on the order (the tile sort orders every list by the unique
(depth bits, id) key), so only the timing moves.

    python tools/spatial_probe.py [--gaussians 300000 --cams 27 --width 800 --height 800 --features 32]
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
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings,  # noqa: E402
                                               GaussianRasterizerBatch)
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def morton_perm(means):
    lo, hi = means.min(0).values, means.max(0).values
    q = ((means - lo) / (hi - lo).clamp_min(1e-12) * 1023).long().clamp(0, 1023)

    def spread(v):
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        return (v | (v << 2)) & 0x09249249
    return torch.argsort(spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300_000)
    ap.add_argument("--cams", type=int, default=27)
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    W, H, C = a.width, a.height, a.cams
    g = make_gaussians(a.gaussians, F=a.features, seed=0, device=dev)
    keys = ["means3D", "colors", "opacities", "scales", "rotations"] + (["semantic_feature"] if a.features else [])
    perm = morton_perm(g["means3D"])
    scenes = {"index_order": {k: g[k].contiguous() for k in keys},
              "morton_order": {k: g[k][perm].contiguous() for k in keys}}
    bg = torch.zeros(3, device=dev)
    sets = [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y, bg=bg,
        viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference") for c in camera_rig(C, W, H)]
    gen = torch.Generator(device=dev).manual_seed(1)
    up = [torch.randn(C, 3, H, W, device=dev, generator=gen), torch.randn(C, 1, H, W, device=dev, generator=gen)]
    if a.features:
        up.append(torch.randn(C, a.features, H, W, device=dev, generator=gen))
    label = torch.ones(a.gaussians, device=dev)
    # the library's own form: the index-order scene, the binning passes
    # walking it in Morton order (GaussianRasterizerBatch(spatial_order=True))
    scenes["walk_order"] = scenes["index_order"]
    ras = {name: GaussianRasterizerBatch(sets, spatial_order=(name == "walk_order")) for name in scenes}
    assert ras["index_order"].spatial_order is False

    def step(name):
        s = scenes[name]
        leaves = {k: s[k].detach().requires_grad_(True) for k in keys}
        kw = dict(means3D=leaves["means3D"], means2D=torch.zeros(a.gaussians, 3, device=dev),
                  opacities=leaves["opacities"], colors_precomp=leaves["colors"], scales=leaves["scales"],
                  rotations=leaves["rotations"], label=label)
        if a.features:
            im, _, feat, depth, _ = ras[name](semantic_feature=leaves["semantic_feature"], **kw)
            torch.autograd.backward([im, depth, feat], up)
        else:
            im, _, depth, _ = ras[name](**kw)
            torch.autograd.backward([im, depth], up[:2])
        return im

    out = {name: [] for name in scenes}
    imgs = {}
    for name in scenes:  # warm-up (kernel loads, binning capacity)
        for _ in range(2):
            imgs[name] = step(name).detach()
    torch.cuda.synchronize()
    same = {"morton_order": bool(torch.equal(imgs["index_order"], imgs["morton_order"])),
            "walk_order": bool(torch.equal(imgs["index_order"], imgs["walk_order"]))}
    for _ in range(a.reps):
        for name in scenes:
            torch.cuda.synchronize()
            _lib.timing_enable(True)
            for _ in range(a.steps):
                step(name)
            torch.cuda.synchronize()
            st = _lib.timing_read()
            _lib.timing_enable(False)
            out[name].append({k: round(v[0] / a.steps, 4) for k, v in st.items() if v[1]})
    print(json.dumps({"gaussians": a.gaussians, "cams": C, "size": [W, H], "features": a.features,
                      "images_identical": same, "stage_ms_per_step": out}))


if __name__ == "__main__":
    main()
