"""The sync-free batch forward (gs_forward_batch, ABI 11; VERDICT r04 item 2,
SURVEY.md 7(d)): the binning buffer is sized from the previous call's list
lengths and the plan headers are read after every stage is enqueued.  Its
outputs must be bit-identical to the reference's two-phase order (plan, host
read of the counts, render) whether the first attempt fits or not:
  * steady state: capacity and sort extents from the previous call, no retry;
  * a forced overflow of one camera's binning buffer: the kernels store
    nothing past it and the call re-renders with the exact lengths;
  * a stale sort hint (a tile outside the hinted class launches): re-rendered;
  * a scene that changes between calls (capacities adapt);
  * the ctypes binding as well as the native one.
Gradients through the backward (which takes the forward's binning layout)
equal the two-phase path's up to fp32 atomic order (1e-5 relative L2)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from dynamic3dgaussians_amd import _C
from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizerBatch
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _settings(cams, W, H, compat="reference", windows=None):
    windows = windows or [None] * len(cams)
    return [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.tensor([0.1, 0.2, 0.3], device=DEV), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(DEV), compat=compat, tile_window=w)
        for c, w in zip(cams, windows)]


def _scene(P, F, seed=0):
    g = make_gaussians(P, F=F, seed=seed, device=DEV)
    return {"means3D": g["means3D"], "colors_precomp": g["colors"], "opacities": g["opacities"],
            "scales": g["scales"], "rotations": g["rotations"], "semantic_feature": g["semantic_feature"]}


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _run(ras, src, ups, lab):
    leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
    P = src["means3D"].shape[0]
    im, radii, feat, depth, alpha = ras(means2D=torch.zeros(P, 3, device=DEV), label=lab, **leaves)
    torch.autograd.backward([im, depth, feat], ups)
    torch.cuda.synchronize()
    return [t.detach().clone() for t in (im, radii, feat, depth, alpha)], {k: v.grad for k, v in leaves.items()}


def _same(outs_a, outs_b, grads_a, grads_b):
    for a, b in zip(outs_a, outs_b):
        assert torch.equal(a, b)
    for k in grads_b:
        assert _rel(grads_a[k], grads_b[k]) <= 1e-5, (k, _rel(grads_a[k], grads_b[k]))


def _ups(C, F, W, H, seed=1):
    gen = torch.Generator(device=DEV).manual_seed(seed)
    return [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen),
            torch.randn(C, F, H, W, device=DEV, generator=gen)]


@pytest.mark.parametrize("compat", ["reference", "fixed"])
@pytest.mark.parametrize("binding", ["native", "ctypes"])
def test_sync_free_steady_state_matches_two_phase(compat, binding, P=20000, W=208, H=160, F=32, C=6):
    src = _scene(P, F, seed=2)
    rig = camera_rig(C, W, H)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    sets = _settings(rig, W, H, compat, windows=[None, None, None, (0, 2, gx, gy - 3), None, (1, 0, gx - 2, gy)])
    ups = _ups(C, F, W, H)
    lab = torch.ones(P, device=DEV)
    assert _C.native_loaded(), "the native binding did not load"
    keep = _C._native
    try:
        _C._native = keep if binding == "native" else None
        ref_o, ref_g = _run(GaussianRasterizerBatch(sets, sync_free=False), src, ups, lab)
        ras = GaussianRasterizerBatch(sets)
        for it in range(3):
            o, g = _run(ras, src, ups, lab)
            _same(o, ref_o, g, ref_g)
    finally:
        _C._native = keep
    # the first call has no capacity (its attempt renders nothing and retries);
    # the later ones fit
    assert ras.plan.calls == 3 and ras.plan.retries == 0, (ras.plan.calls, ras.plan.retries)
    assert all(c >= n for c, n in zip(ras.plan.capacity, ras.plan.num_instances))


def test_forced_overflow_and_stale_hint_retry_bit_identical(P=30000, W=240, H=176, F=32, C=5):
    src = _scene(P, F, seed=4)
    sets = _settings(camera_rig(C, W, H), W, H)
    ups = _ups(C, F, W, H, seed=3)
    lab = torch.ones(P, device=DEV)
    ref_o, ref_g = _run(GaussianRasterizerBatch(sets, sync_free=False), src, ups, lab)
    ras = GaussianRasterizerBatch(sets)
    _run(ras, src, ups, lab)  # first call: capacities and hint
    exact = list(ras.plan.num_instances)
    assert min(exact) > 100
    # one camera's binning buffer 100 instances short, another's exact
    cap = [n + 4096 for n in exact]
    cap[2] = exact[2] - 100
    cap[4] = exact[4]
    ras.plan.force_capacity = cap
    o, g = _run(ras, src, ups, lab)
    _same(o, ref_o, g, ref_g)
    assert ras.plan.retries == 1
    # exact capacities fit
    ras.plan.force_capacity = exact
    o, g = _run(ras, src, ups, lab)
    _same(o, ref_o, g, ref_g)
    assert ras.plan.retries == 1
    # a stale sort hint: the long-tile class launches left out
    valid, p1, q1, p2, max_len, total = ras.plan.hint
    assert valid == 1
    ras.plan.hint = [1, 0, 1 << 20, 0, 16, total]
    o, g = _run(ras, src, ups, lab)
    _same(o, ref_o, g, ref_g)
    assert ras.plan.retries == 2
    o, g = _run(ras, src, ups, lab)  # and back to the steady state
    _same(o, ref_o, g, ref_g)
    assert ras.plan.retries == 2


def test_scene_growing_between_calls(P=20000, W=192, H=144, F=8, C=4):
    """The Gaussians grow every call (more instances than the last call's
    capacity margin): every call still matches the two-phase render."""
    base = _scene(P, F, seed=6)
    sets = _settings(camera_rig(C, W, H), W, H)
    ras = GaussianRasterizerBatch(sets)
    lab = torch.ones(P, device=DEV)
    ups = _ups(C, F, W, H, seed=5)
    grown = 0
    for it, s in enumerate((1.0, 1.05, 1.6, 2.4, 2.4, 1.0)):
        src = dict(base, scales=base["scales"] * s)
        ref_o, ref_g = _run(GaussianRasterizerBatch(sets, sync_free=False), src, ups, lab)
        before = ras.plan.retries
        o, g = _run(ras, src, ups, lab)
        _same(o, ref_o, g, ref_g)
        grown += ras.plan.retries - before
    assert grown >= 1  # the large growth steps outgrew the capacity and re-rendered


def test_sync_free_empty_and_debug_paths(W=96, H=80, C=3):
    """A batch whose cameras see nothing (lists empty, capacity 0 fits) and
    the debug flag (the two-phase path with its checks) behave as before."""
    src = _scene(500, 4, seed=8)
    src["opacities"] = torch.full_like(src["opacities"], 1e-5)  # projected, but no alpha >= 1/255 anywhere
    sets = _settings(camera_rig(C, W, H), W, H)
    ras = GaussianRasterizerBatch(sets)
    lab = torch.ones(500, device=DEV)
    for _ in range(2):
        im, radii, feat, depth, alpha = ras(means2D=torch.zeros(500, 3, device=DEV), label=lab, **src)
        assert int(radii.count_nonzero()) > 0
        assert ras.plan.num_instances == [0] * C
        np.testing.assert_array_equal(im[:, 0].cpu().numpy(), np.float32(0.1))
    assert ras.plan.retries == 0
    dbg = [s_._replace(debug=True) for s_ in _settings(camera_rig(C, W, H), W, H)]
    src2 = _scene(3000, 4, seed=9)
    r_dbg = GaussianRasterizerBatch(dbg)
    r_ref = GaussianRasterizerBatch(_settings(camera_rig(C, W, H), W, H), sync_free=False)
    lab = torch.ones(3000, device=DEV)
    a = r_dbg(means2D=torch.zeros(3000, 3, device=DEV), label=lab, **src2)
    b = r_ref(means2D=torch.zeros(3000, 3, device=DEV), label=lab, **src2)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert r_dbg.plan.calls == 0  # debug runs the two-phase path
