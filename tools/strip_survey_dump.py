#!/usr/bin/env python3
"""Dump the bench scene's camera-0 screen-space Gaussians and tile lists
(gs_debug_export), with the per-pixel last-contributor counts, for an offline
survey of strip-culling granularity (tools/strip_survey.py, quad_survey.py).

    python tools/strip_survey_dump.py [camera]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd import _C  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402
from tests import _harness as Hh  # noqa: E402

dev = "cuda"
P, W, H = 300000, 800, 800
g = make_gaussians(P, F=0, seed=0, device=dev)
cam = int(sys.argv[1]) if len(sys.argv) > 1 else 0
c = camera_rig(27, W, H)[cam]
e = torch.Tensor([])
o = _C.rasterize_gaussians(torch.zeros(3, device=dev), g["means3D"], g["colors"], None, g["opacities"],
                           g["scales"], g["rotations"], 1.0, e, torch.from_numpy(c.viewmatrix.copy()).to(dev),
                           torch.from_numpy(c.projmatrix.copy()).to(dev), c.c_x, c.c_y, c.tanfovx, c.tanfovy,
                           H, W, e, 0, torch.from_numpy(c.campos.copy()).to(dev), False, False)
st = Hh.export_state(P, W, H, o)
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/strip_survey{'' if cam == 0 else cam}.npz", means2D=st["means2D"],
                    conic_opacity=st["conic_opacity"], point_list=st["point_list"], ranges=st["ranges"],
                    n_contrib=st["n_contrib"])
print("ok", len(st["point_list"]))
