"""Fused colour + seg pass against the reference's
two-pass rendering (train.py:145 colour, train.py:246-249 seg with
colors_precomp = seg_colors), both through the drop-in GaussianRasterizer."""
from __future__ import annotations

import pytest
import torch

from tests import _harness as H
from dynamic3dgaussians_amd.fused import render_colour_and_seg
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer

pytestmark = pytest.mark.gpu


def _setup(bg, F=0, P=3000, seed=0, compat="reference"):
    inp = H.scene(P=P, F=F, seed=seed, bg=bg)
    d = lambda k: inp[k].to(H.DEV)  # noqa: E731
    rs = GaussianRasterizationSettings(
        image_height=inp["image_height"], image_width=inp["image_width"], tanfovx=inp["tan_fovx"],
        tanfovy=inp["tan_fovy"], c_x=inp["c_x"], c_y=inp["c_y"], bg=d("bg"), scale_modifier=1.0,
        viewmatrix=d("viewmatrix"), projmatrix=d("projmatrix"), sh_degree=0, campos=d("campos"),
        prefiltered=False, debug=False, compat=compat)
    P = inp["means3D"].size(0)
    g = torch.Generator().manual_seed(seed + 11)
    seg = (torch.rand(P, 3, generator=g) > 0.5).float()  # binary seg colours like the reference
    leaves = dict(means3D=d("means3D"), colors_precomp=d("colors"), opacities=d("opacity"),
                  scales=d("scales"), rotations=d("rotations"), seg_colors=seg.to(H.DEV))
    if F:
        leaves["semantic_feature"] = d("semantic_feature")
    leaves = {k: v.clone().requires_grad_(True) for k, v in leaves.items()}
    return rs, leaves


def _means2D(leaves):
    return torch.zeros_like(leaves["means3D"], requires_grad=True)


@pytest.mark.parametrize("bg", [(0.0, 0.0, 0.0), (1.0, 0.25, 0.5)])
def test_fused_colour_seg_matches_two_passes(bg):
    rs, lv = _setup(bg)
    m2a, m2b, m2c = _means2D(lv), _means2D(lv), _means2D(lv)
    ras = GaussianRasterizer(rs)
    geo = dict(means3D=lv["means3D"], opacities=lv["opacities"], scales=lv["scales"],
               rotations=lv["rotations"])
    im, radius, depth = ras(means2D=m2a, colors_precomp=lv["colors_precomp"], **geo)
    seg2, _, _ = ras(means2D=m2b, colors_precomp=lv["seg_colors"], **geo)
    im_f, radius_f, depth_f, seg_f = render_colour_and_seg(
        rs, means2D=m2c, colors_precomp=lv["colors_precomp"], seg_colors=lv["seg_colors"], **geo)
    torch.cuda.synchronize()
    # forward: the same fp32 fma chain per pixel -> bit-identical
    assert torch.equal(im_f, im)
    assert torch.equal(depth_f, depth)
    assert torch.equal(radius_f, radius)
    assert torch.equal(seg_f, seg2)
    assert seg_f.shape == (3, rs.image_height, rs.image_width)


@pytest.mark.parametrize("compat", ["reference", "fixed"])
def test_fused_colour_seg_gradients(compat):
    """Colour + depth + seg loss through the fused pass.  dL/dseg_colors equals
    the seg render's dL/dcolors_precomp in both modes.  Geometry: reference
    numerics drop the feature term of dL/dalpha (Q5), so the fused geometry
    gradients equal the colour render's alone (the reference's densification
    intent, train.py:245); fixed numerics give the full two-pass sum.  All up to
    fp32 atomic / summation order."""
    rs, lv = _setup((0.0, 0.0, 0.0), compat=compat)
    ras = GaussianRasterizer(rs)
    geo_keys = ("means3D", "opacities", "scales", "rotations")
    g = torch.Generator(device=H.DEV).manual_seed(5)
    Wc = torch.randn(3, rs.image_height, rs.image_width, device=H.DEV, generator=g)
    Ws = torch.randn(3, rs.image_height, rs.image_width, device=H.DEV, generator=g)
    Wd = torch.randn(1, rs.image_height, rs.image_width, device=H.DEV, generator=g)

    def grads(loss, extra, keep=False):
        ts = [lv[k] for k in geo_keys] + [lv["colors_precomp"], lv["seg_colors"]] + extra
        return torch.autograd.grad(loss, ts, allow_unused=True, retain_graph=keep)

    geo = {k: lv[k] for k in geo_keys}
    m2a, m2b = _means2D(lv), _means2D(lv)
    im, _, depth = ras(means2D=m2a, colors_precomp=lv["colors_precomp"], **geo)
    seg, _, _ = ras(means2D=m2b, colors_precomp=lv["seg_colors"], **geo)
    col_loss = (im * Wc).sum() + (depth * Wd).sum()
    colour_only = grads(col_loss, [m2a], keep=True)
    two = grads(col_loss + (seg * Ws).sum(), [m2a, m2b])
    m2c = _means2D(lv)
    im_f, _, depth_f, seg_f = render_colour_and_seg(
        rs, means2D=m2c, colors_precomp=lv["colors_precomp"], seg_colors=lv["seg_colors"], **geo)
    one = grads((im_f * Wc).sum() + (seg_f * Ws).sum() + (depth_f * Wd).sum(), [m2c])
    rel = lambda a, b: H.rel_l2(a.cpu().numpy(), b.cpu().numpy())  # noqa: E731
    assert colour_only[5] is None                # seg_colors unused by the colour loss
    assert rel(one[4], two[4]) <= 1e-5            # colors_precomp
    assert rel(one[5], two[5]) <= 1e-5            # seg_colors
    if compat == "reference":
        for i, name in enumerate(geo_keys):
            assert rel(one[i], colour_only[i]) <= 1e-5, name
        assert rel(one[6], colour_only[6]) <= 1e-5   # means2D
    else:
        for i, name in enumerate(geo_keys):
            assert rel(one[i], two[i]) <= 1e-4, name
        assert rel(one[6], two[6] + two[7]) <= 1e-4  # means2D of both renders


def test_fused_colour_seg_with_semantic_feature():
    """With the caller's own semantic features the layout is [features, seg,
    ones] (fused.py): the caller's channels keep their indices, and the
    user's feature map comes back bit-identical to a plain render's (the
    same fp32 fma chain per channel), the seg image to the seg render's."""
    rs, lv = _setup((0.0, 0.0, 0.0), F=8)
    geo = dict(means3D=lv["means3D"], opacities=lv["opacities"], scales=lv["scales"],
               rotations=lv["rotations"])
    ras = GaussianRasterizer(rs)
    label = torch.ones(lv["means3D"].size(0), device=H.DEV)
    im, radius, feat, depth, _ = ras(means2D=_means2D(lv), colors_precomp=lv["colors_precomp"],
                                     semantic_feature=lv["semantic_feature"], label=label, **geo)
    seg2, _, _ = ras(means2D=_means2D(lv), colors_precomp=lv["seg_colors"], **geo)
    im_f, radius_f, depth_f, seg_f, feat_f = render_colour_and_seg(
        rs, means2D=_means2D(lv), colors_precomp=lv["colors_precomp"], seg_colors=lv["seg_colors"],
        semantic_feature=lv["semantic_feature"], **geo)
    torch.cuda.synchronize()
    assert torch.equal(im_f, im) and torch.equal(depth_f, depth) and torch.equal(radius_f, radius)
    assert torch.equal(seg_f, seg2)
    assert torch.equal(feat_f, feat)


def test_fused_colour_seg_f32_against_oracle():
    """The G3 fused pass at BASELINE configs[2] full size (300k Gaussians,
    800x800, the caller's 32 semantic channels + seg: the F = 36 kernels)
    against the oracle's two renders of the reference step: the colour render
    (F = 32, dyn_train.py:244) and the seg render (colors_precomp =
    seg_colors, train.py:246-249), reference numerics, non-zero background.
    Images: the criteria of tests/test_gpu_parity.py (>= 99.9 % of pixels
    within 1e-5); gradients dL/dcolors, dL/dsemantic (colour render) and
    dL/dseg_colors (seg render's dL/dcolors) relative L2 <= 1e-4."""
    import numpy as np
    inp = H.scene(P=300_000, F=32, W=800, H=800, scale_mult=1.0, bg=(0.3, 0.2, 0.1))
    P, Hh, W = inp["means3D"].shape[0], inp["image_height"], inp["image_width"]
    g = torch.Generator().manual_seed(17)
    seg_colors = (torch.rand(P, 3, generator=g) > 0.5).float()
    d = lambda k: inp[k].to(H.DEV)  # noqa: E731
    rs = GaussianRasterizationSettings(
        image_height=Hh, image_width=W, tanfovx=inp["tan_fovx"], tanfovy=inp["tan_fovy"], c_x=inp["c_x"],
        c_y=inp["c_y"], bg=d("bg"), scale_modifier=1.0, viewmatrix=d("viewmatrix"), projmatrix=d("projmatrix"),
        sh_degree=0, campos=d("campos"), prefiltered=False, debug=False, compat="reference")
    lv = {k: v.clone().requires_grad_(True) for k, v in dict(
        colors_precomp=d("colors"), seg_colors=seg_colors.to(H.DEV), semantic_feature=d("semantic_feature")).items()}
    geo = dict(means3D=d("means3D"), opacities=d("opacity"), scales=d("scales"), rotations=d("rotations"))
    im, radii, depth, seg, feat = render_colour_and_seg(
        rs, means2D=torch.zeros(P, 3, device=H.DEV), label=torch.ones(P, device=H.DEV), **lv, **geo)
    gr = torch.Generator().manual_seed(23)
    dc, dseg = torch.randn(3, Hh, W, generator=gr), torch.randn(3, Hh, W, generator=gr)
    df, dd = torch.randn(32, Hh, W, generator=gr), torch.randn(1, Hh, W, generator=gr) * 0.1
    loss = ((im * dc.to(H.DEV)).sum() + (seg * dseg.to(H.DEV)).sum() + (feat * df.to(H.DEV)).sum()
            + (depth * dd.to(H.DEV)).sum())
    gcol, gseg, gsem = torch.autograd.grad(loss, [lv["colors_precomp"], lv["seg_colors"], lv["semantic_feature"]])
    # the oracle's two renders
    oc = H.oracle_forward(inp)
    inp_s = dict(inp, colors=seg_colors, semantic_feature=None)
    os_ = H.oracle_forward(inp_s)
    for a, b in ((im, oc[1]), (feat, oc[2]), (depth, oc[3]), (seg, os_[1])):
        a = a.detach().cpu().numpy()
        assert a.shape == b.shape
        assert np.mean(np.abs(a - b) <= 1e-5 * max(1.0, np.abs(b).max() if b is oc[3] else 1.0)) >= 0.999
    np.testing.assert_array_equal(radii.cpu().numpy(), oc[5])
    ob = H.oracle_backward(inp, oc, (dc, df, dd, torch.zeros(1, Hh, W)))
    osb = H.oracle_backward(inp_s, os_, (dseg, torch.zeros(0, Hh, W), torch.zeros(1, Hh, W), torch.zeros(1, Hh, W)))
    # over the Gaussians whose footprint holds no pixel whose
    # last contributor flipped (v_exp_f32 vs libm expf; in reference numerics
    # the backward starts from T = 1, Q1, so one flipped termination rescales
    # its pixel's whole gradient -- test_gpu_fullsize.py)
    st_g = H.export_state(P, W, Hh, H.gpu_forward(inp))
    flipped = H.flipped_pixels(st_g, oc[6], W, Hh)
    keep = ~H.covers_pixels(oc[6], oc[5], flipped, W)
    assert keep.mean() >= 0.99
    for name, a, b in (("colors", gcol, ob[1]), ("semantic", gsem, ob[2]), ("seg_colors", gseg, osb[1])):
        a = a.cpu().numpy()
        err = H.rel_l2(a[keep], b[keep])
        assert err <= 1e-4, (name, err, flipped.size)
