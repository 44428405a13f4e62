#!/usr/bin/env python3
"""Host time per phase of one bench training step (BASELINE configs[1] shape
by default: 100k Gaussians, one 800x800 camera, F = 0), measured on the host
clock without synchronising between phases: where a single-camera step that
is host-bound spends its time.  The forward's phase includes the plan's
device->host read, i.e. waiting for the GPU.

    python tools/host_step.py [--gaussians 100000] [--cams 1] [--features 0] [--mode batch|percam]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.optim import FusedAdam  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: E402
                                               GaussianRasterizerBatch)
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=100_000)
    ap.add_argument("--cams", type=int, default=1)
    ap.add_argument("--features", type=int, default=0)
    ap.add_argument("--size", type=int, default=800)
    ap.add_argument("--mode", default="batch", choices=["batch", "percam"])
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    W = H = a.size
    g = make_gaussians(a.gaussians, F=a.features, seed=0, device=dev)
    bg = torch.zeros(3, device=dev)
    sets = [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y, bg=bg,
        viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference") for c in camera_rig(a.cams, W, H)]
    # the bench's parameterisation (dyn_train.py:117-129): logit opacities, log scales
    params = {"means3D": g["means3D"].clone(), "colors": g["colors"].clone(), "opacities": torch.logit(g["opacities"]),
              "scales": torch.log(g["scales"]), "rotations": g["rotations"].clone()}
    params = {k: v.requires_grad_(True) for k, v in params.items()}
    if a.features:
        params["semantic_feature"] = g["semantic_feature"].clone().requires_grad_(True)
    opt = FusedAdam([{"params": [p], "lr": 1e-3} for p in params.values()], lr=0.0, eps=1e-15)
    label = torch.ones(a.gaussians, device=dev)
    gen = torch.Generator(device=dev).manual_seed(1)
    C = a.cams
    upc = torch.randn(C, 3, H, W, device=dev, generator=gen)
    upd = torch.randn(C, 1, H, W, device=dev, generator=gen)
    upf = torch.randn(C, a.features, H, W, device=dev, generator=gen) if a.features else None
    batch = GaussianRasterizerBatch(sets)
    rasters = [GaussianRasterizer(s) for s in sets]
    phases = {"zero_grad": 0.0, "activations": 0.0, "forward": 0.0, "backward": 0.0, "adam": 0.0}

    def step(rec: bool):
        t = [time.perf_counter()]
        opt.zero_grad(set_to_none=True)
        t.append(time.perf_counter())
        rv = dict(means3D=params["means3D"], colors_precomp=params["colors"],
                  opacities=torch.sigmoid(params["opacities"]), scales=torch.exp(params["scales"]),
                  rotations=torch.nn.functional.normalize(params["rotations"]),
                  means2D=torch.zeros_like(params["means3D"]), label=label)
        if a.features:
            rv["semantic_feature"] = params["semantic_feature"]
        t.append(time.perf_counter())
        if a.mode == "batch":
            outs = batch(**rv)
            o, gr = [outs[0], outs[-2]], [upc, upd]
            if a.features:
                o.append(outs[2])
                gr.append(upf)
        else:
            o, gr = [], []
            for i, r in enumerate(rasters):
                outs = r(**rv)
                o += [outs[0], outs[-2]]
                gr += [upc[i], upd[i]]
                if a.features:
                    o.append(outs[2])
                    gr.append(upf[i])
        t.append(time.perf_counter())
        torch.autograd.backward(o, gr)
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        if rec:
            for k, (t0, t1) in zip(phases, zip(t, t[1:])):
                phases[k] += t1 - t0

    for _ in range(20):
        step(False)
    torch.cuda.synchronize()
    if os.environ.get("HOST_STEP_PROFILE"):
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            for _ in range(20):
                step(False)
            torch.cuda.synchronize()
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30), flush=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    out = {k: round(v / a.steps * 1e3, 4) for k, v in phases.items()}
    print({"mode": a.mode, "cams": C, "gaussians": a.gaussians, "features": a.features, "step_ms": round(wall, 4),
           "host_ms_per_phase": out}, flush=True)


if __name__ == "__main__":
    main()
