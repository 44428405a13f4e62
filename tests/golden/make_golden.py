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

5. train_helpers.npz -- the training loop's own helpers around the
   rasterizer, from helpers.py and external.py: setup_camera (helpers.py:
   68-95, the camera every Dynamic3DGaussians caller builds, here with
   off-centre principal points), params2rendervar (:98-107, the activations
   GS_FLAG_ACTIVATE folds into the kernels), l1_loss_v1/v2 and
   weighted_l2_loss_v1/v2 (:110-122), quat_mult (:124-133), build_rotation
   (external.py:61-78), calc_psnr (external.py:85-87), and the neighbour
   losses composed from them exactly as train.py:256-270 does (rigid, rot,
   iso).  Both files import Open3D at module level (for o3d_knn, which is not
   called); Open3D is absent here, so an EMPTY placeholder module is
   registered under that name while they load -- none of the functions used
   touches it.  helpers.py's `Camera` (the rasterizer's settings tuple) is
   replaced by a recorder of its keyword arguments, its `.cuda()` moves are
   identity and its / external.py's hard-coded device="cuda" goes to the CPU
   (there is no GPU here); nothing else is changed.

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


class _RecordCamera:
    """helpers.py's `Camera` (GaussianRasterizationSettings): keeps the
    keyword arguments setup_camera computes."""

    def __init__(self, **kw):
        self.kw = kw


def _load_with_placeholders(name, path):
    """Load a reference module whose top level imports Open3D (absent) and
    the rasterizer package: both names point at inert placeholders while it
    loads."""
    saved = {k: sys.modules.get(k) for k in ("open3d", "diff_gaussian_rasterization")}
    sys.modules["open3d"] = types.ModuleType("open3d")
    dgr = types.ModuleType("diff_gaussian_rasterization")
    dgr.GaussianRasterizationSettings = _RecordCamera
    dgr.GaussianRasterizer = None
    sys.modules["diff_gaussian_rasterization"] = dgr
    try:
        return _load_module(name, path)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


class _TorchOnCPUAll(_TorchOnCPU):
    """_TorchOnCPU plus zeros_like / ones / tensor without their device."""

    @staticmethod
    def zeros_like(*a, **kw):
        kw.pop("device", None)
        return torch.zeros_like(*a, **kw)

    @staticmethod
    def ones(*a, **kw):
        kw.pop("device", None)
        return torch.ones(*a, **kw)

    @staticmethod
    def tensor(*a, **kw):
        kw.pop("device", None)
        return torch.tensor(*a, **kw)


def make_train_helpers(ref):
    hp = _load_with_placeholders("ref_helpers", os.path.join(ref, "helpers.py"))
    ex = _load_with_placeholders("ref_external", os.path.join(ref, "external.py"))
    hp.torch = _TorchOnCPUAll("torch")
    ex.torch = _TorchOnCPUAll("torch")
    cuda0 = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **kw: self  # the .cuda() moves of setup_camera
    out = {}
    try:
        rng = np.random.default_rng(7)
        cams = {k: [] for k in ("w", "h", "k", "w2c", "viewmatrix", "projmatrix", "campos", "tanfovx", "tanfovy",
                                "c_x", "c_y")}
        for i in range(12):
            w, h = int(rng.integers(64, 1921)), int(rng.integers(64, 1081))
            fx, fy = float(rng.uniform(0.6, 1.6) * w), float(rng.uniform(0.6, 1.6) * w)
            cx, cy = float(w / 2 + rng.uniform(-0.2, 0.2) * w), float(h / 2 + rng.uniform(-0.2, 0.2) * h)
            if i == 0:
                cx, cy = w / 2, h / 2
            K = [[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]]
            q, _ = np.linalg.qr(rng.standard_normal((3, 3)))
            if np.linalg.det(q) < 0:
                q[:, 0] = -q[:, 0]
            w2c = np.eye(4)
            w2c[:3, :3], w2c[:3, 3] = q, rng.uniform(-3, 3, 3)
            cam = hp.setup_camera(w, h, K, w2c.tolist())
            kw = cam.kw
            for k, v in (("w", w), ("h", h), ("k", np.array(K)), ("w2c", w2c),
                         ("viewmatrix", kw["viewmatrix"].reshape(4, 4).numpy()),
                         ("projmatrix", kw["projmatrix"].reshape(4, 4).numpy()), ("campos", kw["campos"].numpy()),
                         ("tanfovx", kw["tanfovx"]), ("tanfovy", kw["tanfovy"]), ("c_x", kw["c_x"]),
                         ("c_y", kw["c_y"])):
                cams[k].append(v)
        for k, v in cams.items():
            out[f"cam_{k}"] = np.array(v)
        g = torch.Generator().manual_seed(8)
        P = 2000
        params = {"means3D": torch.randn(P, 3, generator=g), "rgb_colors": torch.rand(P, 3, generator=g),
                  "unnorm_rotations": torch.randn(P, 4, generator=g) * torch.exp(torch.randn(P, 1, generator=g)),
                  "logit_opacities": torch.randn(P, 1, generator=g) * 3,
                  "log_scales": torch.randn(P, 3, generator=g) - 4}
        rv = hp.params2rendervar(params)
        for k, v in params.items():
            out[f"p_{k}"] = v.numpy()
        for k in ("rotations", "opacities", "scales"):
            out[f"rv_{k}"] = rv[k].numpy()
        x, y = torch.randn(64, 3, generator=g), torch.randn(64, 3, generator=g)
        wt = torch.rand(64, 1, generator=g)
        out.update(loss_x=x.numpy(), loss_y=y.numpy(), loss_w=wt.numpy(),
                   l1_v1=hp.l1_loss_v1(x, y).numpy(), l1_v2=hp.l1_loss_v2(x, y).numpy(),
                   wl2_v1=hp.weighted_l2_loss_v1(x, y, wt).numpy(), wl2_v2=hp.weighted_l2_loss_v2(x, y, wt[:, 0]).numpy())
        img1, img2 = torch.rand(3, 48, 40, generator=g), torch.rand(3, 48, 40, generator=g)
        out.update(psnr_img1=img1.numpy(), psnr_img2=img2.numpy(), psnr=ex.calc_psnr(img1, img2).numpy())
        # the neighbour losses as train.py:256-270 composes them
        N, K = 400, 10
        fg_pts = torch.randn(N, 3, generator=g)
        fg_rot = torch.nn.functional.normalize(torch.randn(N, 4, generator=g))
        prev_inv = torch.nn.functional.normalize(torch.randn(N, 4, generator=g))
        nbr = (torch.arange(N)[:, None] + torch.randint(1, N, (N, K), generator=g)) % N
        nw = torch.rand(N, K, generator=g)
        prev_off = torch.randn(N, K, 3, generator=g) * 0.3
        ndist = torch.rand(N, K, generator=g)
        rel_rot = hp.quat_mult(fg_rot, prev_inv)
        rot = ex.build_rotation(rel_rot)
        neighbor_pts = fg_pts[nbr]
        curr_offset = neighbor_pts - fg_pts[:, None]
        cop = (rot.transpose(2, 1)[:, None] @ curr_offset[:, :, :, None]).squeeze(-1)
        rigid = hp.weighted_l2_loss_v2(cop, prev_off, nw)
        rot_l = hp.weighted_l2_loss_v2(rel_rot[nbr], rel_rot[:, None], nw)
        mag = torch.sqrt((curr_offset ** 2).sum(-1) + 1e-20)
        iso = hp.weighted_l2_loss_v1(mag, ndist, nw)
        out.update(nb_fg_pts=fg_pts.numpy(), nb_fg_rot=fg_rot.numpy(), nb_prev_inv_rot=prev_inv.numpy(),
                   nb_indices=nbr.numpy(), nb_weight=nw.numpy(), nb_prev_offset=prev_off.numpy(),
                   nb_dist=ndist.numpy(), nb_rel_rot=rel_rot.numpy(), nb_rot=rot.numpy(),
                   nb_rigid=rigid.numpy(), nb_rot_loss=rot_l.numpy(), nb_iso=iso.numpy())
    finally:
        torch.Tensor.cuda = cuda0
    np.savez_compressed(os.path.join(HERE, "train_helpers.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    a = ap.parse_args()
    make_sh(a.reference)
    make_conventions(a.reference)
    make_cov3d(a.reference)
    make_cameras(a.reference)
    make_train_helpers(a.reference)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
