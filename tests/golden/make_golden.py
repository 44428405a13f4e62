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

3. cov3d.npz -- the reference's 3D covariance in Python: utils/general_utils.py
   build_rotation / build_scaling_rotation / strip_symmetric (:78-110), composed
   as scene/gaussian_model.py:40-44 (build_covariance_from_scaling_rotation:
   L = R S, Sigma = L L^T, upper triangle), the Python twin of
   CR/forward.cu:129-163 computeCov3D.  The module hard-codes device="cuda";
   here its `torch` is a view of torch whose zeros() drop the device argument
   (there is no GPU in the dev container) -- nothing else is changed.  Its
   build_rotation normalises the quaternion; the CUDA kernel does not (Q7):
   the fixture holds raw and normalised quaternions so the test can show both.

4. cameras.npz -- the 3DGS camera matrices: utils/graphics_utils.py
   getWorld2View2 / getProjectionMatrix (:38-71), composed as
   scene/cameras.py:49-52 (world_view_transform, full_proj_transform,
   camera_center; the .cuda() moves left out), for seeded R, T and fields of
   view.  Pins camera.setup_camera (the helpers.py:68-95 form every G1 caller
   uses) at a centred principal point, where the two forms must agree.

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


class _TorchOnCPU(types.ModuleType):
    """torch as utils/general_utils.py sees it, with the hard-coded
    device="cuda" of its zeros() calls redirected to the CPU."""

    def __getattr__(self, k):
        return getattr(torch, k)

    @staticmethod
    def zeros(*a, **kw):
        kw.pop("device", None)
        return torch.zeros(*a, **kw)


def make_cov3d(ref):
    gu = _load_module("ref_general_utils", os.path.join(ref, "utils", "general_utils.py"))
    gu.torch = _TorchOnCPU("torch")
    g = torch.Generator().manual_seed(3)
    P = 512
    scales = torch.exp(torch.randn(P, 3, generator=g) * 0.7 - 3.0)
    rot_raw = torch.randn(P, 4, generator=g) * torch.exp(0.5 * torch.randn(P, 1, generator=g))
    rot_unit = rot_raw / rot_raw.norm(dim=1, keepdim=True)
    out = {"scales": scales.numpy(), "rotations_raw": rot_raw.numpy(), "rotations_unit": rot_unit.numpy()}
    for tag, mod in (("1", 1.0), ("0p7", 0.7)):
        # scene/gaussian_model.py:40-44 build_covariance_from_scaling_rotation
        L = gu.build_scaling_rotation(mod * scales, rot_raw)
        cov = L @ L.transpose(1, 2)
        out[f"cov3D_mod{tag}"] = gu.strip_symmetric(cov).numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "cov3d.npz"), **out)


def make_cameras(ref):
    gr = _load_module("ref_graphics_utils", os.path.join(ref, "utils", "graphics_utils.py"))
    rng = np.random.default_rng(4)
    n = 16
    Rs, Ts, fx, fy, Ws, Hs, wvt, full, centre = [], [], [], [], [], [], [], [], []
    for i in range(n):
        q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
        if np.linalg.det(q) < 0:
            q[:, 0] = -q[:, 0]
        R = q.astype(np.float64)
        T = rng.uniform(-3, 3, 3)
        W, H = int(rng.integers(64, 1921)), int(rng.integers(64, 1081))
        fovx = float(rng.uniform(0.5, 1.6))
        fovy = 2 * np.arctan(np.tan(fovx / 2) * H / W)
        # scene/cameras.py:49-52
        w = torch.tensor(gr.getWorld2View2(R, T)).transpose(0, 1)
        p = gr.getProjectionMatrix(znear=0.01, zfar=100.0, fovX=fovx, fovY=fovy).transpose(0, 1)
        f = w.unsqueeze(0).bmm(p.unsqueeze(0)).squeeze(0)
        c = w.inverse()[3, :3]
        Rs.append(R); Ts.append(T); fx.append(fovx); fy.append(fovy); Ws.append(W); Hs.append(H)  # noqa: E702
        wvt.append(w.numpy()); full.append(f.numpy()); centre.append(c.numpy())  # noqa: E702
    np.savez_compressed(os.path.join(HERE, "cameras.npz"), R=np.array(Rs), T=np.array(Ts), fovx=np.array(fx),
                        fovy=np.array(fy), W=np.array(Ws), H=np.array(Hs), world_view_transform=np.array(wvt),
                        full_proj_transform=np.array(full), camera_center=np.array(centre))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    make_sh(a.reference)
    make_conventions(a.reference)
    make_cov3d(a.reference)
    make_cameras(a.reference)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
