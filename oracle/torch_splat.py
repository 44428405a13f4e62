"""Naive dense PyTorch splat -- TEST INFRASTRUCTURE ONLY (and the shape of
BASELINE.json configs[0], "naive PyTorch CPU splat").

Only tests/ may import this module, as a checker.  It restates the
rasterizer's forward -- preprocess (CR/forward.cu:174-260: projection,
computeCov3D :129-163, computeCov2D :75-124, getRect CR/auxiliary.h:46-56)
and the per-pixel front-to-back blend (CR/forward.cu:330-380) -- as dense
float64 tensor algebra over every (pixel, Gaussian) pair of each 16x16 tile
and its tile list, so that torch autograd differentiates it.  That gives gradients derived independently of
both the reference's hand-written backward (CR/backward.cu) and the C oracle
(oracle/gs_oracle.c): `tests/test_gpu_autograd.py` checks the HIP backward
against them.

Semantics follow compat="fixed" (the reference's quirks that only change
gradients -- Q2 swapped camera arguments, Q3 x_grad_mul, Q5 dead feature
term -- are the ones "fixed" removes; the forward quirks Q7 unnormalised
quaternion, Q8 z <= 0 culling, Q9 asymmetric clamp, Q14 unnormalised depth
are reproduced).  Discrete decisions (tile membership by the radius rect,
alpha >= 1/255, the T < 1e-4 stop) are made without gradient, like the
reference.  Autograd keeps every tile's pairs: O(256 x tile instances)
memory, small scenes only.
"""
from __future__ import annotations

import torch

TILE = 16
# CR/auxiliary.h:22-39
SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435)


def sh_colors(means3D, shs, degree, campos):
    """computeColorFromSH (CR/forward.cu:20-71): shs [P, M, 3] -> rgb [P, 3],
    clamped at 0 after the +0.5 (autograd zeroes the clamped channels, as the
    reference's backward does with its clamped flags)."""
    d = means3D - campos.to(means3D.dtype)[None]
    d = d / torch.sqrt((d * d).sum(1, keepdim=True))
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    S = lambda i: shs[:, i, :]  # noqa: E731
    res = SH_C0 * S(0)
    if degree > 0:
        res = res - SH_C1 * y * S(1) + SH_C1 * z * S(2) - SH_C1 * x * S(3)
        if degree > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            res = (res + SH_C2[0] * xy * S(4) + SH_C2[1] * yz * S(5) + SH_C2[2] * (2.0 * zz - xx - yy) * S(6)
                   + SH_C2[3] * xz * S(7) + SH_C2[4] * (xx - yy) * S(8))
            if degree > 2:
                res = (res + SH_C3[0] * y * (3.0 * xx - yy) * S(9) + SH_C3[1] * xy * z * S(10)
                       + SH_C3[2] * y * (4.0 * zz - xx - yy) * S(11)
                       + SH_C3[3] * z * (2.0 * zz - 3.0 * xx - 3.0 * yy) * S(12)
                       + SH_C3[4] * x * (4.0 * zz - xx - yy) * S(13) + SH_C3[5] * z * (xx - yy) * S(14)
                       + SH_C3[6] * x * (xx - 3.0 * yy) * S(15))
    return torch.clamp(res + 0.5, min=0.0)


def _quat_cols(q):
    """CR/forward.cu:137-149 (glm columns; Q7: not normalised).  -> [P, 3, 3]
    with R[:, c, k] = column c, row k."""
    r, x, y, z = q.unbind(1)
    return torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], 1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], 1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1)], 1)


def preprocess(means3D, scales, rotations, view, proj, tanfovx, tanfovy, cx, cy, W, H, scale_modifier=1.0,
               means2D_ndc_offset=None):
    """Per-Gaussian screen quantities (float64, differentiable) and the
    detached rect / visibility."""
    P = means3D.shape[0]
    hom = torch.cat([means3D, torch.ones(P, 1, dtype=means3D.dtype)], 1)
    Vm = view.reshape(4, 4).to(means3D.dtype)   # column-major: o_j = sum_i p_i m[4i + j]
    Pm = proj.reshape(4, 4).to(means3D.dtype)
    pv = (hom @ Vm)[:, :3]
    ph = hom @ Pm
    pw = 1.0 / (ph[:, 3] + 1e-7)
    pp = ph[:, :2] * pw[:, None]
    if means2D_ndc_offset is not None:   # the reference's means2D leaf: gradient = dL/d(NDC mean)
        pp = pp + means2D_ndc_offset[:, :2]
    # Sigma = M M^T with M[c][k] = s_k R[c][k]
    Rc = _quat_cols(rotations)
    M = Rc * (scale_modifier * scales)[:, None, :]
    Sigma = M @ M.transpose(1, 2)
    fx, fy = W / (2.0 * tanfovx), H / (2.0 * tanfovy)
    tz = pv[:, 2]
    lxp, lxn = (W - cx) / fx + 0.3 * tanfovx, cx / fx + 0.3 * tanfovx
    lyp, lyn = (H - cy) / fy + 0.3 * tanfovy, cy / fy + 0.3 * tanfovy
    tx = torch.clamp(pv[:, 0] / tz, -lxn, lxp) * tz
    ty = torch.clamp(pv[:, 1] / tz, -lyn, lyp) * tz
    j00, j02 = fx / tz, -(fx * tx) / (tz * tz)
    j11, j12 = fy / tz, -(fy * ty) / (tz * tz)
    # rows of J W: a0[r] = view[4r] j00 + view[2+4r] j02, a1[r] = view[1+4r] j11 + view[2+4r] j12
    v = view.reshape(-1).to(means3D.dtype)
    a0 = torch.stack([v[4 * r] * j00 + v[2 + 4 * r] * j02 for r in range(3)], 1)
    a1 = torch.stack([v[1 + 4 * r] * j11 + v[2 + 4 * r] * j12 for r in range(3)], 1)
    ca = torch.einsum("pi,pij,pj->p", a0, Sigma, a0) + 0.3
    cb = torch.einsum("pi,pij,pj->p", a1, Sigma, a0)
    cc = torch.einsum("pi,pij,pj->p", a1, Sigma, a1) + 0.3
    det = ca * cc - cb * cb
    conic = torch.stack([cc / det, -cb / det, ca / det], 1)
    px = ((pp[:, 0] + 1.0) * W - 1.0) * 0.5
    py = ((pp[:, 1] + 1.0) * H - 1.0) * 0.5
    with torch.no_grad():
        mid = 0.5 * (ca + cc)
        l1 = mid + torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        l2 = mid - torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
        rad = torch.ceil(3.0 * torch.sqrt(torch.maximum(l1, l2)))
        gx, gy = (W + TILE - 1) // TILE, (H + TILE - 1) // TILE
        pxf, pyf = px.float(), py.float()
        rmin_x = torch.clamp(((pxf - rad) / TILE).trunc(), 0, gx)
        rmin_y = torch.clamp(((pyf - rad) / TILE).trunc(), 0, gy)
        rmax_x = torch.clamp((((pxf + rad) + TILE) - 1.0).div(TILE).trunc(), 0, gx)
        rmax_y = torch.clamp((((pyf + rad) + TILE) - 1.0).div(TILE).trunc(), 0, gy)
        visible = (tz > 0) & (det != 0) & ((rmax_x - rmin_x) * (rmax_y - rmin_y) > 0)
    return dict(px=px, py=py, depth=tz, conic=conic, rect=(rmin_x, rmin_y, rmax_x, rmax_y), visible=visible,
                radius=rad)


def render(means3D, colors, opacity, scales, rotations, view, proj, tanfovx, tanfovy, cx, cy, W, H, bg,
           features=None, means2D=None, scale_modifier=1.0, tiles=None):
    """-> (color [3,H,W], depth [1,H,W], features [F,H,W] or None,
    alpha = 1 - T_final [1,H,W]) in the inputs' float dtype (float64 for the
    gradient checks, float32 for bench.py's CPU baseline), differentiable in
    every float input (means2D: the NDC offset leaf).  `tiles` (an iterable
    of (tx, ty)) renders only those 16x16 tiles; the rest of the image stays
    zero (a bounded sample of a large render)."""
    pre = preprocess(means3D, scales, rotations, view, proj, tanfovx, tanfovy, cx, cy, W, H, scale_modifier,
                     means2D)
    vis = pre["visible"]
    idx = torch.nonzero(vis).squeeze(1)
    # front-to-back: (depth, index) -- the reference's stable tile order
    order = idx[torch.argsort(pre["depth"][idx].detach().float(), stable=True)]
    px, py, z = pre["px"][order], pre["py"][order], pre["depth"][order]
    con = pre["conic"][order]
    op = opacity.reshape(-1)[order]
    col = colors[order]
    feat = features[order] if features is not None else None
    rmin_x, rmin_y, rmax_x, rmax_y = (r[order] for r in pre["rect"])
    # per 16x16 tile: the tile's pixels against the Gaussians whose rect
    # contains it (the reference's tile lists), dense over those pairs
    gx, gy = (W + TILE - 1) // TILE, (H + TILE - 1) // TILE
    Fd = feat.shape[1] if feat is not None else 0
    fmap = None
    rows_c, rows_d, rows_a, rows_f, where = [], [], [], [], []
    dt = means3D.dtype
    bg = bg.to(dt)
    tile_iter = tiles if tiles is not None else [(tx, ty) for ty in range(gy) for tx in range(gx)]
    for tx, ty in tile_iter:
        x0, y0 = tx * TILE, ty * TILE
        x1, y1 = min(x0 + TILE, W), min(y0 + TILE, H)
        ys, xs = torch.meshgrid(torch.arange(y0, y1, dtype=dt),
                                torch.arange(x0, x1, dtype=dt), indexing="ij")
        qx, qy = xs.reshape(-1, 1), ys.reshape(-1, 1)
        m = torch.nonzero((tx >= rmin_x) & (tx < rmax_x) & (ty >= rmin_y) & (ty < rmax_y)).squeeze(1)
        if m.numel() == 0:
            c = bg[None].expand(qx.shape[0], 3)
            rows_c.append(c); rows_d.append(torch.zeros(qx.shape[0], dtype=means3D.dtype))
            rows_a.append(torch.zeros(qx.shape[0], dtype=means3D.dtype))
            if feat is not None:
                rows_f.append(torch.zeros(qx.shape[0], Fd, dtype=means3D.dtype))
            where.append((x0, y0, x1, y1))
            continue
        dx, dy = px[m][None] - qx, py[m][None] - qy
        cm = con[m]
        power = -0.5 * (cm[:, 0] * dx * dx + cm[:, 2] * dy * dy) - cm[:, 1] * dx * dy
        alpha = torch.clamp(op[m][None] * torch.exp(power), max=0.99)
        with torch.no_grad():
            valid = (power <= 0) & (alpha >= 1.0 / 255.0)
        a = torch.where(valid, alpha, torch.zeros_like(alpha))
        one_m = 1.0 - a
        T_excl = torch.cumprod(torch.cat([torch.ones_like(one_m[:, :1]), one_m[:, :-1]], 1), 1)
        with torch.no_grad():
            stop = valid & (T_excl * one_m < 1e-4)
            keep = torch.cumsum(stop.int(), 1) == 0
        w = a * T_excl * keep
        T_final = torch.prod(torch.where(keep, one_m, torch.ones_like(one_m)), 1)
        rows_c.append(w @ col[m] + T_final[:, None] * bg[None])
        rows_d.append(w @ z[m])
        rows_a.append(1.0 - T_final)
        if feat is not None:
            rows_f.append(w @ feat[m])
        where.append((x0, y0, x1, y1))
    # assemble (index_put keeps the graph)
    pix = torch.cat([(torch.arange(y0, y1)[:, None] * W + torch.arange(x0, x1)[None]).reshape(-1)
                     for (x0, y0, x1, y1) in where])
    color = torch.zeros(H * W, 3, dtype=means3D.dtype).index_put((pix,), torch.cat(rows_c, 0)).T.reshape(3, H, W)
    depth = torch.zeros(H * W, dtype=means3D.dtype).index_put((pix,), torch.cat(rows_d, 0)).reshape(1, H, W)
    alpha = torch.zeros(H * W, dtype=means3D.dtype).index_put((pix,), torch.cat(rows_a, 0)).reshape(1, H, W)
    if feat is not None:
        fmap = torch.zeros(H * W, Fd, dtype=means3D.dtype).index_put((pix,), torch.cat(rows_f, 0)).T.reshape(
            Fd, H, W)
    return color, depth, fmap, alpha
