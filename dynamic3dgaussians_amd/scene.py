"""Seeded synthetic scenes for tests and the benchmark.

There is no network and no dataset in this environment, so the benchmark uses
synthetic Gaussians with the statistics of a trained Panoptic scene:
means ~ U(box), log-scales ~ N(log(0.01 * extent), 0.5), random unit
quaternions, opacity ~ U(0.05, 0.95), colours ~ U(0, 1), SH (deg 3) ~ N(0, 0.2)
with the DC term from the colour, features ~ N(0, 1).  Parameters are built
the way Dynamic3DGaussians' params2rendervar does (helpers.py:98-107).
"""
from __future__ import annotations

import math

import numpy as np
import torch

SH_C0 = 0.28209479177387814


def make_gaussians(P: int, F: int = 0, sh_degree: int = 0, extent: float = 1.0, seed: int = 0,
                   scale_mult: float = 1.0, device="cpu") -> dict:
    """Return a dict of float32 tensors on `device`:
    means3D [P,3], rotations [P,4] (unit), scales [P,3], opacities [P,1],
    colors [P,3], shs [P,(D+1)^2,3], semantic_feature [P,F] (if F > 0)."""
    g = torch.Generator().manual_seed(seed)
    means = (torch.rand(P, 3, generator=g) * 2 - 1) * extent
    log_scales = torch.randn(P, 3, generator=g) * 0.5 + math.log(0.01 * extent * scale_mult)
    quats = torch.randn(P, 4, generator=g)
    quats = torch.nn.functional.normalize(quats, dim=1)
    opac = torch.rand(P, 1, generator=g) * 0.9 + 0.05
    colors = torch.rand(P, 3, generator=g)
    M = (sh_degree + 1) ** 2
    shs = torch.randn(P, max(M, 1), 3, generator=g) * 0.2
    shs[:, 0, :] = (colors - 0.5) / SH_C0
    out = dict(means3D=means, rotations=quats, scales=torch.exp(log_scales), opacities=opac,
               colors=colors, shs=shs)
    if F > 0:
        out["semantic_feature"] = torch.randn(P, F, generator=g)
    return {k: v.float().contiguous().to(device) for k, v in out.items()}


def camera_tensors(cam, device="cpu", bg=(0.0, 0.0, 0.0)) -> dict:
    """Torch tensors of a camera.CameraParams in the raster-settings layout."""
    return dict(image_height=cam.H, image_width=cam.W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy,
                c_x=cam.c_x, c_y=cam.c_y,
                bg=torch.tensor(bg, dtype=torch.float32, device=device),
                viewmatrix=torch.from_numpy(np.ascontiguousarray(cam.viewmatrix)).to(device),
                projmatrix=torch.from_numpy(np.ascontiguousarray(cam.projmatrix)).to(device),
                campos=torch.from_numpy(np.ascontiguousarray(cam.campos)).to(device))
