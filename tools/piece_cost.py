#!/usr/bin/env python3
"""Measured cost of one more camera piece in a rank's batch (the fixed cost
per piece of distributed.shard_camera_windows' balance model; VERDICT r04
item 1 asked for it measured instead of guessed).

A piece is a (camera, tile window) entry of the rank's camera batch: its
projection of every Gaussian, its plan and binning launches' share, and the
launch tails of its windows.  Same scene and rig as bench.py (300k Gaussians,
800x800, F = 32, raw parameters); forward + backward of one batch per step,
interleaved windows of STEPS steps:
  A  cameras 0-2 whole + camera 3 whole                (4 pieces)
  B  cameras 0-2 whole + camera 3 as 2 row bands        (5 pieces, same pixels)
  C  cameras 0-2 whole + camera 3 as 3 row bands        (6 pieces, same pixels)
  D  cameras 0-2 whole                                   (3 pieces: one camera fewer)
piece = (B - A + C - B) / 2, camera = A - D; fraction = piece / camera.

    python tools/piece_cost.py [--reps 3] [--steps 100]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizerBatch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--gaussians", type=int, default=300_000)
    a = ap.parse_args()
    args = argparse.Namespace(gaussians=a.gaussians, features=32, seed=0, compat="reference")
    dev = torch.device("cuda", 0)
    params, label = bench.make_params(args, dev)
    W = H = 800
    rig = camera_rig(27, W, H)
    gy = (H + 15) // 16
    gx = (W + 15) // 16

    def bands(k):
        cuts = [round(i * gy / k) for i in range(k + 1)]
        return [(0, cuts[i], gx, cuts[i + 1]) for i in range(k)]

    layouts = {
        "A": [(c, None) for c in range(4)],
        "B": [(c, None) for c in range(3)] + [(3, w) for w in bands(2)],
        "C": [(c, None) for c in range(3)] + [(3, w) for w in bands(3)],
        "D": [(c, None) for c in range(3)],
    }
    m2 = torch.zeros_like(params["means3D"])
    gen = torch.Generator(device=dev).manual_seed(1)
    up_c = torch.randn(3, H, W, device=dev, generator=gen)
    up_d = torch.randn(1, H, W, device=dev, generator=gen)
    up_f = torch.randn(32, H, W, device=dev, generator=gen)
    runs = {}
    for name, lay in layouts.items():
        sets = bench.make_settings([rig[c] for c, _ in lay], dev, "reference", None, [w for _, w in lay])
        ras = GaussianRasterizerBatch(sets, raw_params=True)
        n = len(lay)
        ups = [up_c.expand(n, -1, -1, -1).contiguous(), up_d.expand(n, -1, -1, -1).contiguous(),
               up_f.expand(n, -1, -1, -1).contiguous()]
        runs[name] = (ras, ups)

    def step(name):
        ras, ups = runs[name]
        for p in params.values():
            p.grad = None
        rv = bench.raw_rendervar(params, label, m2)
        im, _, feat, depth, _ = ras(**rv)
        torch.autograd.backward([im, depth, feat], [ups[0], ups[1], ups[2]])

    res = {k: [] for k in layouts}
    for _ in range(a.reps):
        for name in layouts:
            for _ in range(10):
                step(name)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(name)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / a.steps * 1e3)
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    piece = ((med["B"] - med["A"]) + (med["C"] - med["B"])) / 2
    camera = med["A"] - med["D"]
    out = {"ms_per_step": {k: [round(x, 4) for x in v] for k, v in res.items()},
           "median_ms": {k: round(v, 4) for k, v in med.items()},
           "piece_ms": round(piece, 4), "camera_ms": round(camera, 4),
           "piece_fraction_of_camera": round(piece / camera, 4),
           "layouts": {k: [[c, w] for c, w in v] for k, v in layouts.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
