"""Shared test harness: run the HIP rasterizer and the CPU oracle on the same
seeded inputs and compare.  The oracle is used here only as the checker."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from dynamic3dgaussians_amd import _C, _lib
from dynamic3dgaussians_amd.camera import camera_rig, intrinsics, look_at_w2c, setup_camera
from dynamic3dgaussians_amd.scene import make_gaussians
from oracle import oracle as O

DEV = "cuda"


def scene(P=2000, F=0, sh_degree=0, seed=0, W=128, H=96, cam_index=0, use_sh=False,
          use_cov=False, scale_mult=3.0, n_cams=27, bg=(0.0, 0.0, 0.0), cx=None, cy=None):
    """Inputs for one camera as numpy-friendly CPU tensors + camera params."""
    g = make_gaussians(P, F=F, sh_degree=sh_degree, seed=seed, scale_mult=scale_mult)
    if cx is None and cy is None:
        cam = camera_rig(n_cams, W, H)[cam_index]
    else:
        eye = np.array([0.3, -1.2, 2.2]) * 1.0
        cam = setup_camera(W, H, intrinsics(W, H, 60.0, cx=cx, cy=cy), look_at_w2c(eye))
    inputs = dict(
        bg=torch.tensor(bg, dtype=torch.float32),
        means3D=g["means3D"],
        colors=None if use_sh else g["colors"],
        semantic_feature=g.get("semantic_feature"),
        opacity=g["opacities"],
        scales=None if use_cov else g["scales"],
        rotations=None if use_cov else g["rotations"],
        scale_modifier=1.0,
        cov3D_precomp=None,
        viewmatrix=torch.from_numpy(cam.viewmatrix.copy()),
        projmatrix=torch.from_numpy(cam.projmatrix.copy()),
        c_x=cam.c_x, c_y=cam.c_y, tan_fovx=cam.tanfovx, tan_fovy=cam.tanfovy,
        image_height=H, image_width=W,
        sh=g["shs"][:, : (sh_degree + 1) ** 2].contiguous() if use_sh else None,
        degree=sh_degree,
        campos=torch.from_numpy(cam.campos.copy()),
    )
    if use_cov:
        # Sigma = (S R)^T (S R) computed in float64, handed over precomputed
        q = torch.nn.functional.normalize(g["rotations"].double(), dim=1)
        r, x, y, z = q.unbind(1)
        R = torch.stack([
            torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
            torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
            torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)
        M = torch.diag_embed(g["scales"].double()) @ R
        S = M.transpose(1, 2) @ M
        inputs["cov3D_precomp"] = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1],
                                               S[:, 1, 2], S[:, 2, 2]], 1).float().contiguous()
    return inputs


FWD_ORDER = ["bg", "means3D", "colors", "semantic_feature", "opacity", "scales", "rotations",
             "scale_modifier", "cov3D_precomp", "viewmatrix", "projmatrix", "c_x", "c_y",
             "tan_fovx", "tan_fovy", "image_height", "image_width", "sh", "degree", "campos"]


def _to(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(dev)
    if x is None:
        return torch.Tensor([]).to(dev) if dev != "cpu" else None
    return x


def fwd_args(inp, dev):
    return [_to(inp[k], dev) for k in FWD_ORDER] + [False, False]


def gpu_forward(inp, compat="reference"):
    out = _C.rasterize_gaussians(*fwd_args(inp, DEV), compat=compat)
    torch.cuda.synchronize()
    return out


def oracle_forward(inp, compat="reference"):
    args = [inp[k] for k in FWD_ORDER]
    return O.rasterize_gaussians(*args, prefiltered=False, debug=False, compat=compat)


def upstream_grads(H, W, F, seed=1, alpha_grad=True):
    g = torch.Generator().manual_seed(seed)
    dc = torch.randn(3, H, W, generator=g)
    df = torch.randn(F, H, W, generator=g) if F else torch.zeros(0, H, W)
    dd = torch.randn(1, H, W, generator=g) * 0.1
    da = torch.randn(1, H, W, generator=g) if alpha_grad else torch.zeros(1, H, W)
    return dc, df, dd, da


def bwd_cam4(inp, swap):
    """Camera scalars in the binding's (c_x, c_y, tan_fovx, tan_fovy) slots;
    `swap` reproduces the reference Python wrapper's ordering (Q2)."""
    if swap:
        return inp["tan_fovx"], inp["tan_fovy"], inp["c_x"], inp["c_y"]
    return inp["c_x"], inp["c_y"], inp["tan_fovx"], inp["tan_fovy"]


def gpu_backward(inp, fwd, grads, compat="reference", swap=None):
    if swap is None:
        swap = compat == "reference"
    num_rendered, color, feat, depth, alpha, radii, geom, binning, img = fwd
    dc, df, dd, da = [t.to(DEV) for t in grads]
    d = lambda k: _to(inp[k], DEV)  # noqa: E731
    out = _C.rasterize_gaussians_backward(
        d("bg"), d("means3D"), radii, d("colors"), d("semantic_feature"), d("scales"),
        d("rotations"), inp["scale_modifier"], d("cov3D_precomp"), d("viewmatrix"),
        d("projmatrix"), *bwd_cam4(inp, swap), dc, df, dd, da, d("sh"), inp["degree"],
        d("campos"), geom, num_rendered, binning, img, alpha, False, compat=compat)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in out]


def oracle_backward(inp, ofwd, grads, compat="reference", swap=None, pixel_order=None):
    if swap is None:
        swap = compat == "reference"
    L, color, feat, depth, alpha, radii, st = ofwd
    dc, df, dd, da = [t.numpy() for t in grads]
    return O.rasterize_gaussians_backward(
        inp["bg"], inp["means3D"], radii, inp["colors"], inp["semantic_feature"], inp["scales"],
        inp["rotations"], inp["scale_modifier"], inp["cov3D_precomp"], inp["viewmatrix"],
        inp["projmatrix"], *bwd_cam4(inp, swap), dc, df, dd, da, inp["sh"], inp["degree"],
        inp["campos"], st, L, None, None, alpha, compat=compat, pixel_order=pixel_order)


def export_state(P, W, H, fwd):
    """Per-stage GPU state via gs_debug_export (for stage-level parity).  The
    tile lists hold num_instances (<= num_rendered) entries: read the ranges
    first, then the lists."""
    L_ = _lib.load()
    num_rendered, color, feat, depth, alpha, radii, geom, binning, img = fwd
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    f = lambda *s: torch.empty(*s, dtype=torch.float32, device=DEV)  # noqa: E731
    u = lambda *s: torch.empty(*s, dtype=torch.int32, device=DEV)  # noqa: E731
    s = torch.cuda.current_stream().cuda_stream
    rg = u(tiles, 2)
    _lib.check(L_.gs_debug_export(P, W, H, geom.data_ptr(), None, img.data_ptr(), 0, None, None, None, None,
                                  None, None, rg.data_ptr(), None, s), "debug export")
    torch.cuda.synchronize()
    n_inst = int(rg.view(torch.int64).cpu().numpy().view(np.uint32).reshape(-1, 2)[:, 1].max()) if tiles else 0
    st = dict(means2D=f(P, 2), depths=f(P), conic_opacity=f(P, 4), rgb=f(P, 3), tiles=u(P),
              point_list=u(max(n_inst, 1)), ranges=u(tiles, 2), n_contrib=u(H * W))
    _lib.check(L_.gs_debug_export(P, W, H, geom.data_ptr(), binning.data_ptr() if binning.numel() else None,
                                  img.data_ptr(), n_inst, st["means2D"].data_ptr(),
                                  st["depths"].data_ptr(), st["conic_opacity"].data_ptr(),
                                  st["rgb"].data_ptr(), st["tiles"].data_ptr(),
                                  st["point_list"].data_ptr(), st["ranges"].data_ptr(),
                                  st["n_contrib"].data_ptr(), s), "debug export")
    torch.cuda.synchronize()
    out = {k: v.cpu().numpy() for k, v in st.items()}
    out["point_list"] = out["point_list"][:n_inst].view(np.uint32)
    out["tiles"] = out["tiles"].view(np.uint32)
    out["ranges"] = out["ranges"].view(np.uint32).reshape(-1)
    out["n_contrib"] = out["n_contrib"].view(np.uint32)
    out["num_instances"] = n_inst
    return out


def check_tile_lists(st_g, st_o, W, H):
    """The binned tile lists against the reference's: every tile's list is the
    reference's list (same (depth, index) order) minus instances whose
    Gaussian reaches alpha >= 1/255 at no pixel of the tile (checked in float64
    at every pixel centre, CR/forward.cu:350-360).  Also maps each pixel's
    last contributor back to a Gaussian id and compares it with the
    reference's.  Returns the fraction of instances dropped."""
    rg = st_g["ranges"].reshape(-1, 2).astype(np.int64)
    ro = np.asarray(st_o.ranges, np.int64).reshape(-1, 2)
    pg, po = st_g["point_list"], np.asarray(st_o.point_list)
    m2 = np.asarray(st_o.means2D, np.float64)
    co = np.asarray(st_o.conic_opacity, np.float64)
    gx = (W + 15) // 16
    dropped = 0
    for t in range(rg.shape[0]):
        lo_list = po[ro[t, 0]:ro[t, 1]]
        g_list = pg[rg[t, 0]:rg[t, 1]]
        keep = np.isin(lo_list, g_list)
        assert keep.sum() == len(g_list), f"tile {t}: instances not in the reference's list"
        np.testing.assert_array_equal(lo_list[keep], g_list)
        drop = lo_list[~keep].astype(np.int64)
        dropped += len(drop)
        if len(drop):
            tx, ty = t % gx, t // gx
            xs = np.arange(tx * 16, min(tx * 16 + 16, W), dtype=np.float64)
            ys = np.arange(ty * 16, min(ty * 16 + 16, H), dtype=np.float64)
            px, py = np.meshgrid(xs, ys)
            dx = m2[drop, 0, None, None] - px[None]
            dy = m2[drop, 1, None, None] - py[None]
            a, b, c, op = (co[drop, k, None, None] for k in range(4))
            power = -0.5 * (a * dx * dx + c * dy * dy) - b * dx * dy
            alpha = np.minimum(0.99, op * np.exp(power))
            blends = (power <= 0) & (alpha >= 1.0 / 255.0)
            assert not blends.any(), f"tile {t}: a dropped instance blends"
    assert flipped_pixels(st_g, st_o, W, H).size <= 1e-3 * W * H
    return dropped / max(len(po), 1)


def _last_ids(n, ranges, plist, W, H):
    gx = (W + 15) // 16
    pix = np.arange(W * H)
    tile = (pix // W // 16) * gx + (pix % W) // 16
    if len(plist) == 0:
        return np.full(W * H, -1, np.int64)
    return np.where(n > 0, plist[np.clip(ranges[tile, 0] + n - 1, 0, len(plist) - 1)], -1)


def flipped_pixels(st_g, st_o, W, H):
    """Pixels whose last contributor, as a Gaussian id, differs between the
    GPU and the oracle: a termination / alpha-threshold decision flipped by
    the ulp difference of v_exp_f32 vs libm expf.  (n_contrib itself is a
    position in a list, and the GPU lists are pruned.)"""
    rg = st_g["ranges"].reshape(-1, 2).astype(np.int64)
    ro = np.asarray(st_o.ranges, np.int64).reshape(-1, 2)
    gid_g = _last_ids(st_g["n_contrib"].astype(np.int64), rg, st_g["point_list"].astype(np.int64), W, H)
    gid_o = _last_ids(np.asarray(st_o.n_contrib, np.int64), ro, np.asarray(st_o.point_list, np.int64), W, H)
    return np.nonzero(gid_g != gid_o)[0]


def covers_pixels(st_o, radii, pixels, W):
    """Gaussians whose screen footprint (the reference's radius square around
    means2D) contains any of `pixels`."""
    m2 = np.asarray(st_o.means2D, np.float64)
    r = np.asarray(radii, np.float64)
    hit = np.zeros(len(r), bool)
    for p in pixels:
        px, py = float(p % W), float(p // W)
        hit |= (r > 0) & (np.abs(m2[:, 0] - px) <= r + 1) & (np.abs(m2[:, 1] - py) <= r + 1)
    return hit


def psnr(a, b, peak=1.0):
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return float("inf") if mse == 0 else 10 * np.log10(peak * peak / mse)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / den) if den > 0 else float(np.linalg.norm(a - b))
