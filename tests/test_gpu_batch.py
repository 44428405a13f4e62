"""Camera batches (gs_*_batch, GaussianRasterizerBatch): one launch per stage
for the C cameras of a multi-camera step.  Camera c's forward outputs must be
bit-identical to the per-camera drop-in rasterizer's, and the backward must
equal the sum of the per-camera gradients (autograd's accumulation) up to
fp32 summation order."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,
                                               GaussianRasterizerBatch)
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _settings(cams, W, H, compat, sh_degree=0, bg=None):
    bg = torch.zeros(3, device=DEV) if bg is None else bg
    return [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y, bg=bg,
        viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=sh_degree,
        campos=torch.from_numpy(c.campos.copy()).to(DEV), compat=compat) for c in cams]


def _scene(P, F, use_sh, seed=0):
    g = make_gaussians(P, F=F, seed=seed, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(seed + 11)
    src = dict(means3D=g["means3D"], opacities=g["opacities"], scales=g["scales"], rotations=g["rotations"])
    if F:
        src["semantic_feature"] = g["semantic_feature"]
    if use_sh:
        src["shs"] = torch.randn(P, 16, 3, device=DEV, generator=gen) * 0.2
    else:
        src["colors_precomp"] = g["colors"]
    return src


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("F,use_sh,compat", [(0, False, "reference"), (32, False, "reference"),
                                             (8, True, "fixed"), (32, False, "fixed"), (16, True, "reference")])
def test_batch_matches_per_camera(F, use_sh, compat, P=15000, W=176, H=144, C=5):
    src = _scene(P, F, use_sh, seed=F + (7 if use_sh else 0))
    rig = camera_rig(C, W, H)
    sets = _settings(rig, W, H, compat, sh_degree=3 if use_sh else 0)
    gen = torch.Generator(device=DEV).manual_seed(3)
    label = (torch.rand(P, device=DEV, generator=gen) > 0.25).float()
    up_c = torch.randn(C, 3, H, W, device=DEV, generator=gen)
    up_d = torch.randn(C, 1, H, W, device=DEV, generator=gen)
    up_f = torch.randn(C, F, H, W, device=DEV, generator=gen) if F else None
    up_a = torch.randn(C, 1, H, W, device=DEV, generator=gen)
    names = list(src)

    # per camera (the drop-in), autograd sums over the cameras
    leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
    m2 = torch.zeros(P, 3, device=DEV, requires_grad=True)
    ref = []
    for c in range(C):
        out = GaussianRasterizer(sets[c])(means2D=m2, label=label, **leaves)
        if F:
            im, radius, feat, depth, alpha = out
        else:
            im, radius, depth, alpha = out
            feat = None
        ref.append((im.detach(), radius, None if feat is None else feat.detach(), depth.detach(), alpha.detach()))
        outs, gr = [im, depth, alpha], [up_c[c], up_d[c], up_a[c]]
        if F:
            outs.append(feat)
            gr.append(up_f[c])
        torch.autograd.backward(outs, gr)
    ref_grads = {k: leaves[k].grad.clone() for k in names}
    ref_grads["means2D"] = m2.grad.clone()

    # the batch
    leaves_b = {k: v.clone().requires_grad_(True) for k, v in src.items()}
    m2b = torch.zeros(P, 3, device=DEV, requires_grad=True)
    out = GaussianRasterizerBatch(sets)(means2D=m2b, label=label, **leaves_b)
    if F:
        im, radius, feat, depth, alpha = out
    else:
        im, radius, depth, alpha = out
        feat = None
    assert im.shape == (C, 3, H, W) and radius.shape == (C, P) and depth.shape == (C, 1, H, W)
    for c in range(C):
        r_im, r_rad, r_feat, r_depth, r_alpha = ref[c]
        assert torch.equal(im[c], r_im), c
        assert torch.equal(radius[c], r_rad), c
        assert torch.equal(depth[c], r_depth), c
        assert torch.equal(alpha[c], r_alpha), c
        if F:
            assert torch.equal(feat[c], r_feat), c
    outs, gr = [im, depth, alpha], [up_c, up_d, up_a]
    if F:
        outs.append(feat)
        gr.append(up_f)
    torch.autograd.backward(outs, gr)
    for k in names:
        assert leaves_b[k].grad is not None, k
        assert _rel(leaves_b[k].grad, ref_grads[k]) < 1e-5, (k, _rel(leaves_b[k].grad, ref_grads[k]))
    assert _rel(m2b.grad, ref_grads["means2D"]) < 1e-5
    # label masking: masked Gaussians get exactly zero (Q12)
    off = label == 0
    assert torch.all(leaves_b["means3D"].grad[off] == 0)


def test_batch_of_two_camera_groups_matches_per_camera():
    """11 cameras: the blend launches deal the first 8 one per XCD and the
    last 3 as a smaller group (cam_slot, GS_CAM_GROUP = 8); every camera's
    outputs stay bit-identical to its per-camera render and the gradients
    the per-camera sum."""
    test_batch_matches_per_camera(32, False, "reference", P=9000, W=112, H=96, C=11)


def test_batch_of_one_is_the_single_camera_call(P=12000, W=128, H=96):
    src = _scene(P, 32, False, seed=2)
    rig = camera_rig(3, W, H)
    sets = _settings(rig[1:2], W, H, "reference")
    a = GaussianRasterizer(sets[0])(means2D=torch.zeros(P, 3, device=DEV), label=torch.ones(P, device=DEV), **src)
    b = GaussianRasterizerBatch(sets)(means2D=torch.zeros(P, 3, device=DEV), label=torch.ones(P, device=DEV), **src)
    for x, y in zip(a, b):
        assert torch.equal(x, y[0])


def test_batch_with_empty_and_partial_views(P=8000, W=160, H=112):
    """A camera that sees nothing (every list empty) next to ones that do."""
    src = _scene(P, 8, False, seed=4)
    rig = camera_rig(3, W, H)
    sets = _settings(rig, W, H, "reference")
    # camera 1 looks away from the scene: view matrix of camera 0 turned around
    v = sets[0].viewmatrix.clone()
    v[:, 2] = -v[:, 2]
    v[:, 0] = -v[:, 0]
    sets[1] = sets[1]._replace(viewmatrix=v, projmatrix=sets[1].projmatrix)
    leaves = {k: t.clone().requires_grad_(True) for k, t in src.items()}
    m2 = torch.zeros(P, 3, device=DEV, requires_grad=True)
    im, radius, feat, depth, alpha = GaussianRasterizerBatch(sets)(means2D=m2, label=torch.ones(P, device=DEV),
                                                                    **leaves)
    ref = GaussianRasterizer(sets[1])(means2D=torch.zeros(P, 3, device=DEV), label=torch.ones(P, device=DEV), **src)
    assert torch.equal(im[1], ref[0]) and torch.equal(radius[1], ref[1])
    (im.sum() + feat.sum() + depth.sum()).backward()
    assert all(torch.isfinite(t.grad).all() for t in leaves.values())


def test_batch_densify_stats_match_reference_bookkeeping(P=12000, W=144, H=112, C=4):
    src = _scene(P, 0, False, seed=6)
    rig = camera_rig(C, W, H)
    sets = _settings(rig, W, H, "reference")
    gen = torch.Generator(device=DEV).manual_seed(5)
    up = torch.randn(C, 3, H, W, device=DEV, generator=gen)
    acc, den, mx = torch.zeros(P, device=DEV), torch.zeros(P, device=DEV), torch.zeros(P, device=DEV)
    for c in range(C):
        m2 = torch.zeros(P, 3, device=DEV, requires_grad=True)
        im, radius, depth = GaussianRasterizer(sets[c])(means2D=m2, **src)
        im.backward(up[c])
        seen = radius > 0
        mx[seen] = torch.max(radius[seen].float(), mx[seen])
        acc[seen] += torch.norm(m2.grad[seen, :2], dim=-1)
        den[seen] += 1
    ras = GaussianRasterizerBatch(sets, track_densify=True)
    m2 = torch.zeros(P, 3, device=DEV, requires_grad=True)
    im, radius, depth = ras(means2D=m2, **src)
    im.backward(up)
    st = ras.densify_stats
    torch.testing.assert_close(st["denom"], den, rtol=0, atol=0)
    torch.testing.assert_close(st["max_2D_radius"], mx, rtol=0, atol=0)
    torch.testing.assert_close(st["means2D_gradient_accum"], acc, rtol=1e-5, atol=1e-6)


def _batch_grads(src, sets, ups, label):
    """Gradients of one GaussianRasterizerBatch step over `sets` (G3 call)."""
    leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
    im, radius, feat, depth, alpha = GaussianRasterizerBatch(sets)(
        means2D=torch.zeros(src["means3D"].shape[0], 3, device=DEV), label=label, **leaves)
    torch.autograd.backward([im, depth, feat], list(ups))
    return {k: leaves[k].grad for k in leaves}


@pytest.mark.parametrize("world", [2, 3, 4])
def test_camera_shards_sum_to_the_full_batch(world, P=15000, W=128, H=96, C=27):
    """BASELINE configs[3]: the 27-camera step split over N ranks (camera c
    on rank c mod N, distributed.shard_cameras).  The per-shard batch
    gradients summed over the shards equal the 27-camera batch's (fp32
    summation order only), and a bound GradBucket accumulating the shards'
    backward passes in place holds that same sum."""
    from dynamic3dgaussians_amd.distributed import GradBucket, shard_cameras
    src = _scene(P, 32, False, seed=9)
    rig = camera_rig(C, W, H)
    sets = _settings(rig, W, H, "reference")
    gen = torch.Generator(device=DEV).manual_seed(21)
    up_c = torch.randn(C, 3, H, W, device=DEV, generator=gen)
    up_d = torch.randn(C, 1, H, W, device=DEV, generator=gen)
    up_f = torch.randn(C, 32, H, W, device=DEV, generator=gen)
    label = torch.ones(P, device=DEV)
    full = _batch_grads(src, sets, (up_c, up_d, up_f), label)
    shards = [shard_cameras(C, r, world) for r in range(world)]
    assert sorted(c for s in shards for c in s) == list(range(C))
    total = {k: torch.zeros_like(v) for k, v in full.items()}
    for cams in shards:
        g = _batch_grads(src, [sets[c] for c in cams], (up_c[cams], up_d[cams], up_f[cams]), label)
        for k in total:
            total[k] += g[k]
    for k in full:
        assert _rel(total[k], full[k]) <= 1e-5, (k, _rel(total[k], full[k]))
    # the bench's path: leaves whose .grad are views into one bucket, every
    # shard's backward accumulating into it
    leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
    bucket = GradBucket(leaves, bind_grads=True)
    bucket.zero_grad()
    for cams in shards:
        out = GaussianRasterizerBatch([sets[c] for c in cams])(
            means2D=torch.zeros(P, 3, device=DEV), label=label, **leaves)
        torch.autograd.backward([out[0], out[3], out[2]], [up_c[cams], up_d[cams], up_f[cams]])
    bucket.all_reduce()  # no process group: a no-op that checks the views
    for k in full:
        assert leaves[k].grad.data_ptr() == bucket._views[list(leaves).index(k)].data_ptr()
        assert _rel(leaves[k].grad, full[k]) <= 1e-5, (k, _rel(leaves[k].grad, full[k]))


def test_batch_sort_classes_with_long_and_short_cameras(P=20000, W=160, H=128):
    """The batch merges the cameras' tile-sort class extents (gs_api.hip: max
    of the long-class prefixes, min of the short-class one): a camera with
    tiles longer than SORT_SMALL (1024) and TS_CAP (4096) next to cameras
    whose tiles are all short must still sort every list.  A dense cluster of
    Gaussians just in front of camera 0 makes its long tiles; the batch's
    outputs must be bit-identical to the per-camera calls."""
    from tests import _harness as Hh
    rig = camera_rig(27, W, H)
    cams = [rig[0], rig[9], rig[18]]
    sets = _settings(cams, W, H, "reference")
    src = _scene(P, 8, False, seed=12)
    c0 = cams[0]
    fwd0 = torch.from_numpy(c0.viewmatrix[:3, 2].copy()).float().to(DEV)  # camera 0's viewing axis (w2c row 2)
    pos0 = torch.from_numpy(c0.campos.copy()).float().to(DEV)
    gen = torch.Generator(device=DEV).manual_seed(5)
    n_cl = 12000
    cl = pos0 + 0.6 * fwd0 + 0.01 * torch.randn(n_cl, 3, device=DEV, generator=gen)
    means = src["means3D"].clone()
    means[:n_cl] = cl
    src["means3D"] = means
    src["scales"] = src["scales"].clone()
    src["scales"][:n_cl] = 0.004
    label = torch.ones(P, device=DEV)
    per = [GaussianRasterizer(s)(means2D=torch.zeros(P, 3, device=DEV), label=label, **src) for s in sets]
    # precondition: camera 0 has tiles past both class limits, another camera has only short tiles
    maxlen = []
    for s in sets:
        out = _C_forward(src, s)
        st = Hh.export_state(P, W, H, out)
        rg = st["ranges"].reshape(-1, 2).astype(np.int64)
        maxlen.append(int((rg[:, 1] - rg[:, 0]).max()))
    assert maxlen[0] > 4096, maxlen
    assert min(maxlen[1:]) <= 1024, maxlen
    bat = GaussianRasterizerBatch(sets)(means2D=torch.zeros(P, 3, device=DEV), label=label, **src)
    for c in range(len(sets)):
        for x, y in zip(per[c], bat):
            assert torch.equal(x, y[c]), (c, maxlen)


def _C_forward(src, s):
    from dynamic3dgaussians_amd import _C
    out = _C.rasterize_gaussians(
        s.bg, src["means3D"], src["colors_precomp"], src.get("semantic_feature"), src["opacities"],
        src["scales"], src["rotations"], 1.0, torch.Tensor([]), s.viewmatrix, s.projmatrix, s.c_x, s.c_y,
        s.tanfovx, s.tanfovy, s.image_height, s.image_width, torch.Tensor([]), 0, s.campos, False, False)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("F", [0, 32, 36])
def test_forward_zeroed_scratch_and_a_second_backward(F, P=12000, W=160, H=128, C=4):
    """The batch forward zeroes the backward's scratch inside its blend
    (gs_gaussians.zero_fill, ABI 13) and the first backward skips its fill
    (GS_FLAG_SCRATCH_ZEROED) -- test_batch_matches_per_camera holds those
    gradients to the per-camera calls, which zero their own scratch.  A
    second backward of the same forward (retain_graph), whose scratch the
    first one wrote, must zero it again: it adds the same gradients."""
    src = _scene(P, F, False, seed=5 + F)
    sets = _settings(camera_rig(C, W, H), W, H, "reference")
    gen = torch.Generator(device=DEV).manual_seed(9)
    ups = [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen)]
    if F:
        ups.append(torch.randn(C, F, H, W, device=DEV, generator=gen))

    def run(twice):
        leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
        out = GaussianRasterizerBatch(sets)(means2D=torch.zeros(P, 3, device=DEV), label=torch.ones(P, device=DEV),
                                            **leaves)
        outs = [out[0], out[3], out[2]] if F else [out[0], out[2]]
        torch.autograd.backward(outs, ups, retain_graph=twice)
        first = {k: v.grad.clone() for k, v in leaves.items()}
        if twice:
            torch.autograd.backward(outs, ups)
        return first, {k: v.grad.clone() for k, v in leaves.items()}

    g1, _ = run(False)
    g2, both = run(True)
    for k in g1:
        assert _rel(g2[k], g1[k]) < 1e-5, (k, _rel(g2[k], g1[k]))
        assert _rel(both[k], 2 * g1[k]) < 1e-5, (k, _rel(both[k], 2 * g1[k]))


def test_misaligned_zero_fill_is_refused_and_the_next_call_renders(monkeypatch, P=4000, W=96, H=64, C=2):
    """A zero_fill region that is not 16-B aligned is refused by the C ABI
    (status -1, gs_render_impl) after the plan kernels were enqueued; the
    header slot that call leased goes back to the pool once its stream is
    drained, and the next call on the same device renders the same images
    as a call with the fill turned off."""
    import dynamic3dgaussians_amd._C as C_
    src = _scene(P, 32, False, seed=13)
    sets = _settings(camera_rig(C, W, H), W, H, "reference")
    make = C_.batch_backward_scratch

    def render():
        leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
        return GaussianRasterizerBatch(sets)(means2D=torch.zeros(P, 3, device=DEV),
                                             label=torch.ones(P, device=DEV), **leaves)

    monkeypatch.setattr(C_, "batch_backward_scratch", lambda *a: make(*a)[1:])
    with pytest.raises(Exception, match="zero_fill"):
        render()
    monkeypatch.setattr(C_, "batch_backward_scratch", make)
    out = render()
    monkeypatch.setenv("GS_FORWARD_ZERO_SCRATCH", "0")
    ref = render()
    torch.cuda.synchronize()
    for a, b in zip(out[:5], ref[:5]):
        if torch.is_tensor(a) and a.is_floating_point():
            assert torch.equal(a, b)
