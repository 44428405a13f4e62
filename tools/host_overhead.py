#!/usr/bin/env python3
"""Host-side cost of one camera through the drop-in path (tiny scene: GPU time
negligible): raw _C forward+backward, and GaussianRasterizer autograd."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd import _C, _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer  # noqa: E402
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def main():
    _lib.load()
    dev = "cuda"
    P, W, H, F = 1000, 64, 64, 32
    g = make_gaussians(P, F=F, device=dev)
    c = camera_rig(27, W, H)[0]
    s = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.zeros(3, device=dev), scale_modifier=1.0,
        viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(dev), prefiltered=False, debug=False)
    leaves = {k: v.clone().requires_grad_(True) for k, v in
              dict(means3D=g["means3D"], colors_precomp=g["colors"], opacities=g["opacities"],
                   scales=g["scales"], rotations=g["rotations"],
                   semantic_feature=g["semantic_feature"]).items()}
    means2D = torch.zeros_like(g["means3D"], requires_grad=True)
    label = torch.ones(P, device=dev)
    up = [torch.randn(3, H, W, device=dev), torch.randn(1, H, W, device=dev),
          torch.randn(F, H, W, device=dev)]
    ras = GaussianRasterizer(s)

    def cam():
        im, radius, feat, depth, _ = ras(means2D=means2D, label=label, **leaves)
        torch.autograd.backward([im, depth, feat], up)

    for _ in range(20):
        cam()
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        cam()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    _lib.timing_enable(False)
    print(f"drop-in autograd fwd+bwd per camera: {(t1 - t0) / n * 1e6:.1f} us (P={P}, {W}x{H})")
    # forward only
    t0 = time.perf_counter()
    with torch.no_grad():
        for _ in range(n):
            ras(means2D=means2D, label=label, **leaves)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"drop-in forward only per camera: {(t1 - t0) / n * 1e6:.1f} us")


if __name__ == "__main__":
    main()


def raw():
    """Raw _C calls (no autograd) on the tiny scene."""
    dev = "cuda"
    P, W, H, F = 1000, 64, 64, 32
    g = make_gaussians(P, F=F, device=dev)
    c = camera_rig(27, W, H)[0]
    e = torch.Tensor([])
    bg = torch.zeros(3, device=dev)
    view = torch.from_numpy(c.viewmatrix.copy()).to(dev)
    proj = torch.from_numpy(c.projmatrix.copy()).to(dev)
    campos = torch.from_numpy(c.campos.copy()).to(dev)
    dc, dd, da = torch.randn(3, H, W, device=dev), torch.randn(1, H, W, device=dev), torch.zeros(1, H, W, device=dev)
    df = torch.randn(F, H, W, device=dev)
    sem = g["semantic_feature"]

    def fwd():
        return _C.rasterize_gaussians(bg, g["means3D"], g["colors"], sem, g["opacities"], g["scales"],
                                      g["rotations"], 1.0, e, view, proj, c.c_x, c.c_y, c.tanfovx,
                                      c.tanfovy, H, W, e, 0, campos, False, False)

    def bwd(o):
        L, color, feat, depth, alpha, radii, geom, binning, img = o
        return _C.rasterize_gaussians_backward(bg, g["means3D"], radii, g["colors"], sem, g["scales"],
                                               g["rotations"], 1.0, e, view, proj, c.tanfovx, c.tanfovy,
                                               c.c_x, c.c_y, dc, df, dd, da, e, 0, campos, geom, L,
                                               binning, img, alpha, False)
    o = fwd()
    for _ in range(20):
        bwd(o)
    torch.cuda.synchronize()
    n = 300
    t0 = time.perf_counter()
    for _ in range(n):
        o = fwd()
    t1 = time.perf_counter()
    for _ in range(n):
        bwd(o)
    t2 = time.perf_counter()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    print(f"raw _C forward: {(t1 - t0) / n * 1e6:.1f} us; raw _C backward (host, async): "
          f"{(t2 - t1) / n * 1e6:.1f} us; drain {(t3 - t2) * 1e6:.0f} us")


if __name__ == "__main__" and os.environ.get("RAW"):
    raw()
