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
    """With the caller's own semantic features the seg channels go first (they
    receive the reference's background quirk, Q4) and the user's feature map is
    returned unchanged: equal to a plain render's feature map."""
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
