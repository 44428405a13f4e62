#!/usr/bin/env python3
"""Multi-stream camera overlap (bench.py step) vs one stream: the summed
per-camera gradients on the shared leaves must agree to fp32 atomic order."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizer  # noqa: E402


class A:
    gaussians, features, seed, cams, width, height = 300000, 32, 0, 8, 800, 800


def grads(n_streams):
    dev = torch.device("cuda", 0)
    params, label = bench.make_params(A, dev)
    settings = bench.make_settings(camera_rig(A.cams, A.width, A.height, seed=A.seed), dev, "reference")
    g = torch.Generator(device=dev).manual_seed(1)
    up_c = torch.randn(3, A.height, A.width, device=dev, generator=g)
    up_d = torch.randn(1, A.height, A.width, device=dev, generator=g)
    up_f = torch.randn(A.features, A.height, A.width, device=dev, generator=g)
    rv = bench.params2rendervar(params, label)
    leaves = {k: v.detach().requires_grad_(True) for k, v in rv.items() if isinstance(v, torch.Tensor) and v.requires_grad}
    rvl = dict(rv, **leaves)
    main = torch.cuda.current_stream(dev)
    streams = [main] + [torch.cuda.Stream(device=dev) for _ in range(n_streams - 1)]
    for st in streams:
        st.wait_stream(main)
    for i, s in enumerate(settings):
        with torch.cuda.stream(streams[i % n_streams]):
            im, radius, feat, depth, _ = GaussianRasterizer(s)(**rvl)
            torch.autograd.backward([im, depth, feat], [up_c, up_d, up_f])
    for st in streams:
        main.wait_stream(st)
    torch.cuda.synchronize()
    return {k: v.grad.clone() for k, v in leaves.items()}


a, b = grads(1), grads(4)
worst = 0.0
for k in a:
    rel = ((a[k] - b[k]).norm() / a[k].norm().clamp_min(1e-30)).item()
    worst = max(worst, rel)
    print(k, f"{rel:.2e}")
print("max rel L2", f"{worst:.2e}")
assert worst < 1e-4
print("ok")
