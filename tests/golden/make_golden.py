#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own
Python code (run in the dev container, where /root/reference exists; the
fixtures -- data only -- are committed, the reference never travels).

1. sh_eval.npz -- the reference's SH evaluator utils/sh_utils.py:eval_sh
   (the Python twin of CR/forward.cu:20-71 computeColorFromSH) on seeded
   directions/coefficients, degrees 0..3, plus the clamp(+0.5) colour rule
   of CR/forward.cu:63-70 and gaussian_renderer/__init__.py:86.  Pins the
   oracle's and the HIP kernel's SH colour path.

2. boundary_conventions.json -- the reference autograd wrapper
   DGR/diff_gaussian_rasterization/__init__.py driven with a recording stand-in
   for its compiled `_C` module: which value lands in which positional slot
   of `_C.rasterize_gaussians` / `_C.rasterize_gaussians_backward` (including
   the swapped camera scalars, Q2), what the wrapper returns, and how it
   masks the gradients with `label` (Q12).  The stand-in replaces only the
   missing extension; nothing of the reference is built.

Usage: python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _load_module(name, path, package_dir=None):
    spec = importlib.util.spec_from_file_location(
        name, path, submodule_search_locations=[package_dir] if package_dir else None)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def make_sh(ref):
    sh_utils = _load_module("ref_sh_utils", os.path.join(ref, "utils", "sh_utils.py"))
    g = torch.Generator().manual_seed(0)
    P = 256
    means = torch.randn(P, 3, generator=g)
    campos = torch.tensor([0.3, -0.2, -4.0])
    shs = torch.randn(P, 16, 3, generator=g) * 0.4
    out = {"means3D": means.numpy(), "campos": campos.numpy(), "shs": shs.numpy()}
    for deg in range(4):
        dirs = means - campos
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        # eval_sh takes [..., C, coeffs]
        val = sh_utils.eval_sh(deg, shs.transpose(1, 2).contiguous(), dirs)
        rgb = torch.clamp_min(val + 0.5, 0.0)
        out[f"rgb_deg{deg}"] = rgb.numpy().astype(np.float32)
        out[f"clamped_deg{deg}"] = (val + 0.5 < 0).numpy()
    np.savez_compressed(os.path.join(HERE, "sh_eval.npz"), **out)


class Recorder(types.ModuleType):
    """Stand-in for the compiled `_C`: records calls, returns seeded tensors."""

    def __init__(self):
        super().__init__("_C")
        self.fwd_args = None
        self.bwd_args = None

    @staticmethod
    def _enc(x):
        if isinstance(x, torch.Tensor):
            return {"tensor": x.detach().cpu().double().reshape(-1).tolist(), "shape": list(x.shape)}
        return x

    def rasterize_gaussians(self, *args, **kw):
        self.fwd_args = [self._enc(a) for a in args]
        means3D = args[1]
        P = means3D.shape[0]
        H, W = int(args[15]), int(args[16])
        g = torch.Generator().manual_seed(11)
        color = torch.randn(3, H, W, generator=g)
        feat = torch.randn(32, H, W, generator=g)
        depth = torch.randn(1, H, W, generator=g)
        alpha = torch.zeros(1, H, W)
        radii = torch.arange(P, dtype=torch.int32)
        buf = torch.zeros(4, dtype=torch.uint8)
        return (123, color, feat, depth, alpha, radii, buf, buf.clone(), buf.clone())

    def rasterize_gaussians_backward(self, *args, **kw):
        self.bwd_args = [self._enc(a) for a in args]
        P = args[1].shape[0]
        M = args[19].shape[1] if args[19].numel() else 0
        g = torch.Generator().manual_seed(12)
        r = lambda *s: torch.randn(*s, generator=g)  # noqa: E731
        out = [r(P, 3), r(P, 3), r(P, 32), r(P, 1), r(P, 3), r(P, 6), r(P, M, 3), r(P, 3), r(P, 4)]
        m = kw.get("grad_mask")  # our binding's fused label mask (never passed by the reference)
        if m is not None:
            m = m.float().reshape(-1)
            for i in (1, 3, 4, 5, 7, 8):
                out[i] = out[i] * m[:, None]
            out[6] = out[6] * m[:, None, None]
        return tuple(out)

    def mark_visible(self, *args):
        return torch.ones(args[0].shape[0], dtype=torch.bool)


def conventions_case():
    """Inputs of the recorded call (also rebuilt by the test)."""
    g = torch.Generator().manual_seed(5)
    P, H, W = 6, 4, 5
    t = dict(
        means3D=torch.randn(P, 3, generator=g), colors_precomp=torch.rand(P, 3, generator=g),
        opacities=torch.rand(P, 1, generator=g), scales=torch.rand(P, 3, generator=g),
        rotations=torch.randn(P, 4, generator=g), semantic_feature=torch.randn(P, 32, generator=g),
        label=torch.tensor([1.0, 0.0, 1.0, 1.0, 0.0, 1.0]))
    settings = dict(image_height=H, image_width=W, tanfovx=0.61, tanfovy=0.47, c_x=2.25, c_y=1.75,
                    bg=torch.tensor([0.1, 0.2, 0.3]), scale_modifier=1.5,
                    viewmatrix=torch.arange(16, dtype=torch.float32).reshape(4, 4),
                    projmatrix=torch.arange(16, 32, dtype=torch.float32).reshape(4, 4),
                    sh_degree=0, campos=torch.tensor([0.5, 0.25, -3.0]), prefiltered=False,
                    debug=False, confidence=torch.ones(P, 1))
    return t, settings


def run_wrapper(module, recorder, tensors, settings_kw):
    """Drive a wrapper module (reference or ours) exactly like dyn_train.py:244."""
    t = {k: v.clone().requires_grad_(k != "label") for k, v in tensors.items()}
    means2D = torch.zeros_like(t["means3D"], requires_grad=True)
    s = module.GaussianRasterizationSettings(**settings_kw)
    out = module.GaussianRasterizer(raster_settings=s)(
        means3D=t["means3D"], means2D=means2D, opacities=t["opacities"],
        colors_precomp=t["colors_precomp"], semantic_feature=t["semantic_feature"],
        scales=t["scales"], rotations=t["rotations"], label=t["label"])
    color, radii, feat, depth, alpha = out
    loss = color.sum() * 0.5 + feat.mean() + depth.sum() * 2.0 + alpha.sum()
    loss.backward()
    grads = {k: (v.grad.double().reshape(-1).tolist() if v.grad is not None else None)
             for k, v in t.items() if k != "label"}
    grads["means2D"] = means2D.grad.double().reshape(-1).tolist()
    return {"forward_args": recorder.fwd_args, "backward_args": recorder.bwd_args,
            "n_outputs": len(out), "radii": radii.tolist(), "grads": grads}


def make_conventions(ref):
    dgr = os.path.join(ref, "submodules_fsgs", "diff-gaussian-rasterization-confidence",
                       "diff_gaussian_rasterization")
    rec = Recorder()
    sys.modules["ref_dgr._C"] = rec
    mod = _load_module("ref_dgr", os.path.join(dgr, "__init__.py"), package_dir=dgr)
    tensors, settings = conventions_case()
    res = run_wrapper(mod, rec, tensors, settings)
    res["settings_fields"] = list(mod.GaussianRasterizationSettings._fields)
    with open(os.path.join(HERE, "boundary_conventions.json"), "w") as f:
        json.dump(res, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    make_sh(a.reference)
    make_conventions(a.reference)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
