"""GS_FLAG_ACTIVATE (GaussianRasterizerBatch(raw_params=True)): the
Dynamic3DGaussians activations of helpers.py:98-107 (params2rendervar:
sigmoid of the logit opacities, exp of the log scales, F.normalize of the
unnormalised rotations) applied inside the preprocess kernels, forward and
backward.  The step must equal the one torch gives with the activations as
its own ops in front of the rasterizer: same images and radii, and the raw
parameters' gradients equal autograd's through torch's activations.

The forward activations follow torch's GPU operation order, including the
pairwise squared-norm sum of its reduction kernel (tools/act_probe.py), so
the render records -- and with them radii and images -- are bit-identical to
the torch path's (asserted on the records).  The gradients go through
autograd's formulas in a fixed order of our own (the 4-term sum of the
normalize backward), so they are held to relative L2 <= 1e-4, the
full-size bar of tests/test_gpu_fullsize.py; images to >= 99.9 % of pixels
within 1e-5 and radii to >= 99.9 % equal, should the torch build change."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizerBatch
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _settings(cams, W, H, compat, sh_degree=0):
    return [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.tensor([0.1, 0.2, 0.3], device=DEV),
        viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=sh_degree,
        campos=torch.from_numpy(c.campos.copy()).to(DEV), compat=compat) for c in cams]


def _raw_scene(P, F, use_sh, seed):
    """Raw parameters as dyn_train.py / train.py hold them (helpers.py:98-107),
    with genuinely unnormalised rotations."""
    g = make_gaussians(P, F=F, seed=seed, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(seed + 101)
    qs = torch.exp(0.6 * torch.randn(P, 1, device=DEV, generator=gen))
    raw = {"means3D": g["means3D"], "logit_opacities": torch.logit(g["opacities"]),
           "log_scales": torch.log(g["scales"]), "unnorm_rotations": g["rotations"] * qs}
    if use_sh:
        raw["shs"] = torch.randn(P, 16, 3, device=DEV, generator=gen) * 0.2
    else:
        raw["rgb_colors"] = g["colors"]
    if F:
        raw["semantic_feature"] = g["semantic_feature"]
    return raw


def _kw(leaves, raw):
    kw = {"means3D": leaves["means3D"]}
    if "shs" in leaves:
        kw["shs"] = leaves["shs"]
    else:
        kw["colors_precomp"] = leaves["rgb_colors"]
    if "semantic_feature" in leaves:
        kw["semantic_feature"] = leaves["semantic_feature"]
    if raw:
        kw.update(opacities=leaves["logit_opacities"], scales=leaves["log_scales"],
                  rotations=leaves["unnorm_rotations"])
    else:
        kw.update(opacities=torch.sigmoid(leaves["logit_opacities"]), scales=torch.exp(leaves["log_scales"]),
                  rotations=torch.nn.functional.normalize(leaves["unnorm_rotations"]))
    return kw


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _close_frac(a, b, tol=1e-5):
    return float(((a - b).abs() <= tol).float().mean().item())


@pytest.mark.parametrize("F,use_sh,label_kind,compat", [(32, False, "ones", "reference"),
                                                         (0, True, "mask", "reference"),
                                                         (8, False, None, "fixed")])
def test_raw_params_match_torch_activations(F, use_sh, label_kind, compat, P=20000, W=176, H=144, C=4):
    raw = _raw_scene(P, F, use_sh, seed=31 + F)
    sets = _settings(camera_rig(C, W, H), W, H, compat, sh_degree=3 if use_sh else 0)
    gen = torch.Generator(device=DEV).manual_seed(7)
    label = None
    if label_kind == "ones":
        label = torch.ones(P, device=DEV)
    elif label_kind == "mask":
        label = (torch.rand(P, device=DEV, generator=gen) > 0.3).float()
    ups = [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen)]
    if F:
        ups.append(torch.randn(C, F, H, W, device=DEV, generator=gen))
    outs, grads = {}, {}
    for mode in ("torch", "raw"):
        leaves = {k: v.clone().requires_grad_(True) for k, v in raw.items()}
        ras = GaussianRasterizerBatch(sets, raw_params=mode == "raw")
        extra = {} if label is None else {"label": label}
        out = ras(means2D=torch.zeros(P, 3, device=DEV), **extra, **_kw(leaves, mode == "raw"))
        # arity by the G1-G4 dispatch: colour, radii, depth (+ feature, alpha)
        if label is not None and F:
            im, radii, feat, depth, alpha = out
        elif label is not None:
            im, radii, depth, alpha = out
            feat = None
        elif F:
            im, feat, radii, depth = out
        else:
            im, radii, depth = out
            feat = None
        outs[mode] = (im.detach(), radii, depth.detach(), None if feat is None else feat.detach())
        ts, gs = [im, depth], ups[:2]
        if F:
            ts.append(feat)
            gs = ups
        torch.autograd.backward(ts, gs)
        grads[mode] = {k: leaves[k].grad for k in leaves}
    (im0, r0, d0, f0), (im1, r1, d1, f1) = outs["torch"], outs["raw"]
    same_img = torch.equal(im0, im1)
    print(f"F={F} sh={use_sh}: images bit-identical {same_img}, radii equal "
          f"{float((r0 == r1).float().mean()):.6f}")
    assert float((r0 == r1).float().mean()) >= 0.999
    assert _close_frac(im0, im1) >= 0.999 and _close_frac(d0, d1, 1e-5 * float(d0.abs().max())) >= 0.999
    if F:
        assert _close_frac(f0, f1) >= 0.999
    for k in raw:
        g0, g1 = grads["torch"][k], grads["raw"][k]
        assert g1 is not None, k
        assert _rel(g1, g0) <= 1e-4, (k, _rel(g1, g0))
    if label_kind == "mask":
        off = label == 0
        for k in ("logit_opacities", "log_scales", "unnorm_rotations", "means3D"):
            assert torch.all(grads["raw"][k][off] == 0), k


def test_raw_params_render_records_match_torch_activations(P=30000, W=160, H=128):
    """The activated opacity in the render record (and the conic built from
    exp(scale) and the normalised rotation) against the torch path's, per
    Gaussian: reports the bit-identical fraction and holds every difference
    to a few ulps."""
    from dynamic3dgaussians_amd import _C
    from tests import _harness as Hh
    raw = _raw_scene(P, 0, False, seed=5)
    s = _settings(camera_rig(1, W, H), W, H, "reference")[0]
    recs = {}
    for mode in ("torch", "raw"):
        kw = _kw(raw, mode == "raw")
        out = _C.rasterize_gaussians_batch(
            s.bg, kw["means3D"], kw["colors_precomp"], None, kw["opacities"], kw["scales"], kw["rotations"], 1.0,
            torch.Tensor([]), s.viewmatrix.reshape(1, 16), s.projmatrix.reshape(1, 16), [s.c_x], [s.c_y],
            [s.tanfovx], [s.tanfovy], H, W, torch.Tensor([]), 0, s.campos.reshape(1, 3), False, False,
            compat="reference", activate=mode == "raw")
        torch.cuda.synchronize()
        nr, color, feat, depth, alpha, radii, geom, binning, img, ni = out
        st = Hh.export_state(P, W, H, (nr[0], color[0], feat[0], depth[0], alpha[0], radii[0], geom, binning, img))
        recs[mode] = (radii[0].cpu().numpy(), st["conic_opacity"])
    r0, c0 = recs["torch"]
    r1, c1 = recs["raw"]
    vis = (r0 > 0) & (r1 > 0)
    op_eq = float(np.mean(c0[vis, 3] == c1[vis, 3]))
    con_eq = float(np.mean(np.all(c0[vis, :3] == c1[vis, :3], axis=1)))
    print(f"records: opacity bit-identical {op_eq:.6f}, conic bit-identical {con_eq:.6f} over {int(vis.sum())}")
    assert op_eq == 1.0 and con_eq == 1.0, (op_eq, con_eq)
    np.testing.assert_allclose(c1[vis, 3], c0[vis, 3], rtol=4e-7, atol=0)
    scale = np.maximum(np.abs(c0[vis, 0]), np.abs(c0[vis, 2]))[:, None]
    assert np.all(np.abs(c1[vis, :3] - c0[vis, :3]) <= 1e-5 * scale)
    assert float(np.mean(r0 == r1)) >= 0.999


@pytest.mark.parametrize("raw_params,F", [(True, 32), (False, 35)])
def test_native_batch_binding_matches_ctypes_binding(raw_params, F, P=12000, W=144, H=112, C=3):
    """The C++ batch fast path (lib/_gs_native.so forward_batch /
    backward_batch) and the ctypes batch binding drive the same C ABI:
    identical forward outputs and the same gradients (label mask, densify
    statistics, a padded feature width 35 -> 36, raw parameters)."""
    from dynamic3dgaussians_amd import _C
    assert _C.native_loaded()
    raw = _raw_scene(P, F, False, seed=77)
    sets = _settings(camera_rig(C, W, H), W, H, "reference")
    gen = torch.Generator(device=DEV).manual_seed(9)
    label = (torch.rand(P, device=DEV, generator=gen) > 0.2).float()
    ups = [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen),
           torch.randn(C, F, H, W, device=DEV, generator=gen)]
    res = {}
    keep = _C._native
    try:
        for mode in ("native", "ctypes"):
            _C._native = keep if mode == "native" else None
            leaves = {k: v.clone().requires_grad_(True) for k, v in raw.items()}
            ras = GaussianRasterizerBatch(sets, track_densify=True, raw_params=raw_params)
            im, radii, feat, depth, alpha = ras(means2D=torch.zeros(P, 3, device=DEV), label=label,
                                                **_kw(leaves, raw_params))
            torch.autograd.backward([im, depth, feat], ups)
            torch.cuda.synchronize()
            res[mode] = ([t.detach().cpu().numpy() for t in (im, radii, feat, depth, alpha)],
                         {k: v.grad.cpu().numpy() for k, v in leaves.items()},
                         {k: v.cpu().numpy() for k, v in ras.densify_stats.items()})
    finally:
        _C._native = keep
    (fa, ga, sa), (fb, gb, sb) = res["native"], res["ctypes"]
    for a, b in zip(fa, fb):
        np.testing.assert_array_equal(a, b)
    for k in ga:  # fp32 atomics: the summation order may differ between runs
        assert np.linalg.norm(ga[k] - gb[k]) <= 1e-5 * max(np.linalg.norm(gb[k]), 1e-30), k
    for k in sa:
        np.testing.assert_allclose(sa[k], sb[k], rtol=1e-5, atol=1e-7)
