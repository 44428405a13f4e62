#!/usr/bin/env python3
"""Forward outputs of the bench scene with the default build vs a variant
(e.g. exp_boxcull) saved to gpurun_out for a bitwise comparison, plus the
oracle's colour image PSNR for camera 0."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamic3dgaussians_amd import _C, _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def main():
    tag = os.environ.get("GSPLAT_VARIANT", "") or "default"
    _lib.load(auto_build=False)
    dev = "cuda"
    g = make_gaussians(300000, F=32, seed=0, device=dev)
    out = {}
    for ci in (0, 5, 13):
        c = camera_rig(27, 800, 800)[ci]
        e = torch.Tensor([])
        o = _C.rasterize_gaussians(torch.zeros(3, device=dev), g["means3D"], g["colors"],
                                   g["semantic_feature"], g["opacities"], g["scales"], g["rotations"], 1.0,
                                   e, torch.from_numpy(c.viewmatrix.copy()).to(dev),
                                   torch.from_numpy(c.projmatrix.copy()).to(dev), c.c_x, c.c_y, c.tanfovx,
                                   c.tanfovy, 800, 800, e, 0, torch.from_numpy(c.campos.copy()).to(dev),
                                   False, False)
        out[f"color{ci}"] = o[1].cpu().numpy()
        out[f"feat{ci}"] = o[2][:, ::8, ::8].contiguous().cpu().numpy()
        out[f"depth{ci}"] = o[3].cpu().numpy()
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/cull_{tag}.npz", **out)
    print("saved", tag)


if __name__ == "__main__":
    main()
