#!/usr/bin/env python3
"""Where the host time of one camera goes (tiny scene, GPU time negligible):
time inside _RasterizeGaussians.forward / .backward (Python wrapper + C ABI
calls) vs the whole fwd+bwd (autograd engine, dispatch), with and without a
GradientSink."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd import _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: E402
                                               GradientSink, _RasterizeGaussians)
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402

acc = {"fwd": 0.0, "bwd": 0.0}
for name in ("forward", "backward"):
    orig = getattr(_RasterizeGaussians, name)

    def wrap(*a, _orig=orig, _k="bwd" if name == "backward" else "fwd"):
        t0 = time.perf_counter()
        r = _orig(*a)
        acc[_k] += time.perf_counter() - t0
        return r
    setattr(_RasterizeGaussians, name, staticmethod(wrap))


def main():
    _lib.load()
    dev = "cuda"
    P, W, H, F = 1000, 64, 64, 32
    g = make_gaussians(P, F=F, device=dev)
    c = camera_rig(27, W, H)[0]
    for sink in (None, GradientSink()):
        s = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
            bg=torch.zeros(3, device=dev), scale_modifier=1.0,
            viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
            projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
            campos=torch.from_numpy(c.campos.copy()).to(dev), prefiltered=False, debug=False, grad_sink=sink)
        leaves = {k: v.clone().requires_grad_(True) for k, v in
                  dict(means3D=g["means3D"], colors_precomp=g["colors"], opacities=g["opacities"],
                       scales=g["scales"], rotations=g["rotations"],
                       semantic_feature=g["semantic_feature"]).items()}
        means2D = torch.zeros_like(g["means3D"], requires_grad=True)
        label = torch.ones(P, device=dev)
        up = [torch.randn(3, H, W, device=dev), torch.randn(1, H, W, device=dev), torch.randn(F, H, W, device=dev)]
        ras = GaussianRasterizer(s)

        def cam():
            im, radius, feat, depth, _ = ras(means2D=means2D, label=label, **leaves)
            torch.autograd.backward([im, depth, feat], up)

        for _ in range(20):
            cam()
        torch.cuda.synchronize()
        acc["fwd"] = acc["bwd"] = 0.0
        n = 300
        t0 = time.perf_counter()
        for _ in range(n):
            cam()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / n * 1e6
        print(f"sink={sink is not None}: per camera {t:.1f} us; inside forward {acc['fwd'] / n * 1e6:.1f} us, "
              f"inside backward {acc['bwd'] / n * 1e6:.1f} us", flush=True)


if __name__ == "__main__":
    main()
