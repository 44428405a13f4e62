"""The sharded optimizer step on the GPU (distributed.ShardedAdam, ZeRO
stage 1) and the camera batch's gradient destinations (grad_into):

* at one rank ShardedAdam's update is FusedAdam's, bit for bit (the same HIP
  kernel over the flat storage);
* N ranks each updating their own 1/N slice from the same summed gradients
  (no collective: the slices are assembled here) give FusedAdam's full
  update, bit for bit -- the sharding moves no arithmetic;
* GaussianRasterizerBatch(...)(..., grad_into=views) writes the gradients the
  autograd path returns (to the float-atomic sums' run-to-run noise,
  relative L2 <= 1e-6) into the caller's buffer, every element, and leaves
  .grad untouched (None), for the G3 (label + features) and G2 calls; a
  destination of the wrong size is refused.
The exchange itself (reduce-scatter / all-gather over a process group) is
covered over gloo in tests/test_sharded_adam.py; bench.py runs it over RCCL
(GS_BENCH_ZERO=force at one rank)."""
from __future__ import annotations

import pytest
import torch

from dynamic3dgaussians_amd import _lib
from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.distributed import ShardedAdam
from dynamic3dgaussians_amd.optim import FusedAdam
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizerBatch
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
LRS = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
       "log_scales": 1e-3, "semantic_feature": 1e-3}


def _raw_params(P, F, seed=0):
    g = make_gaussians(P, F=F, seed=seed, device=DEV)
    p = {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
         "logit_opacities": torch.logit(g["opacities"]), "log_scales": torch.log(g["scales"])}
    if F:
        p["semantic_feature"] = g["semantic_feature"]
    return {k: torch.nn.Parameter(v.detach().clone().contiguous()) for k, v in p.items()}


def _grad_seq(params, steps, seed=7):
    gen = torch.Generator(device=DEV).manual_seed(seed)
    return [{k: torch.randn(p.shape, device=DEV, generator=gen) for k, p in params.items()} for _ in range(steps)]


def _fused_reference(P, F, grads):
    params = _raw_params(P, F)
    opt = FusedAdam([{"params": [p], "lr": LRS[k], "name": k} for k, p in params.items()], lr=0.0, eps=1e-15)
    for g in grads:
        for k, p in params.items():
            p.grad = g[k].clone()
        opt.step()
    return params


@pytest.mark.parametrize("P,F", [(1000, 0), (4099, 32)])
def test_one_rank_update_is_fused_adams(P, F):
    grads = _grad_seq(_raw_params(P, F), 4)
    ref = _fused_reference(P, F, grads)
    params = _raw_params(P, F)
    opt = ShardedAdam(params, LRS, rank=0, world=1, eps=1e-15)
    for g in grads:
        for k, v in opt.grad_views(0).items():
            v.copy_(g[k])
        opt.step(0)
    torch.cuda.synchronize()
    for k in params:
        assert torch.equal(params[k].detach(), ref[k].detach()), k


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ranks_slices_assemble_to_the_full_update(world):
    P, F = 3001, 32
    grads = _grad_seq(_raw_params(P, F), 3)
    ref = _fused_reference(P, F, grads)
    ref_flat = torch.cat([ref[k].detach().reshape(-1) for k in ref])
    got = torch.empty_like(ref_flat)
    covered = torch.zeros_like(ref_flat, dtype=torch.int32)
    for r in range(world):
        params = _raw_params(P, F)
        opt = ShardedAdam(params, LRS, rank=r, world=world, eps=1e-15, collectives=False)
        for g in grads:
            for k, v in opt.grad_views(0).items():
                v.copy_(g[k])
            opt.step(0)
        hi = min(opt.hi, opt.total)
        if opt.lo < hi:
            got[opt.lo:hi] = opt.param_flat[opt.lo:hi]
            covered[opt.lo:hi] += 1
    torch.cuda.synchronize()
    assert bool((covered == 1).all())
    assert torch.equal(got, ref_flat)


def _cams(n, W, H, windows=None):
    out = []
    for i, c in enumerate(camera_rig(n, W, H, seed=3)):
        kw = {} if windows is None or windows[i] is None else {"tile_window": windows[i]}
        out.append(GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
            bg=torch.tensor([0.1, 0.2, 0.3], device=DEV),
            viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
            projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=0,
            campos=torch.from_numpy(c.campos.copy()).to(DEV), **kw))
    return out


_ARG = {"means3D": "means3D", "rgb_colors": "colors_precomp", "unnorm_rotations": "rotations",
        "logit_opacities": "opacities", "log_scales": "scales", "semantic_feature": "semantic_feature"}


def _step(ras, params, label, ups, grad_into=None):
    kw = {_ARG[k]: p for k, p in params.items()}
    m2 = torch.zeros_like(params["means3D"])
    if "semantic_feature" in params:
        im, _, feat, depth, _ = ras(means2D=m2, label=label, grad_into=grad_into, **kw)
        torch.autograd.backward([im, depth, feat], ups)
    else:
        im, _, depth, _ = ras(means2D=m2, label=label, grad_into=grad_into, **kw)
        torch.autograd.backward([im, depth], ups[:2])


@pytest.mark.parametrize("F,binding,windows", [(0, "native", False), (32, "native", False),
                                               (32, "ctypes", False), (32, "native", True)])
def test_grad_into_writes_autograds_gradients(F, binding, windows):
    from dynamic3dgaussians_amd import _C
    P, W, H, C = 6000, 160, 128, 3
    sets = _cams(C, W, H, [None, (0, 2, 10, 6), (3, 0, 10, 8)] if windows else None)
    assert _C.native_loaded(), "the native binding did not load"
    keep = _C._native
    try:
        _C._native = keep if binding == "native" else None
        _grad_into_case(sets, P, W, H, C, F)
    finally:
        _C._native = keep


def _grad_into_case(sets, P, W, H, C, F):
    gen = torch.Generator(device=DEV).manual_seed(11)
    ups = [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen),
           torch.randn(C, F, H, W, device=DEV, generator=gen) if F else None]
    label = torch.ones(P, device=DEV)
    # autograd's gradients
    pa = _raw_params(P, F, seed=2)
    _step(GaussianRasterizerBatch(sets, raw_params=True), pa, label, ups)
    # the same step writing into a sharded optimizer's buffer (poisoned first:
    # every element must be written)
    pb = _raw_params(P, F, seed=2)
    opt = ShardedAdam(pb, LRS, rank=0, world=1)
    opt.grad_flat[0].fill_(float("nan"))
    dest = {_ARG[k]: v for k, v in opt.grad_views(0).items()}
    _step(GaussianRasterizerBatch(sets, raw_params=True), pb, label, ups, grad_into=dest)
    torch.cuda.synchronize()
    views = opt.grad_views(0)
    for k in pa:
        assert pb[k].grad is None, k
        assert bool(torch.isfinite(views[k]).all()), k  # every element written
        # the backward's float-atomic sums vary in their last bits run to run
        rel = ((views[k].double() - pa[k].grad.double()).norm() / pa[k].grad.double().norm()).item()
        assert rel <= 1e-6, (k, rel)
    # a destination of the wrong size is refused
    bad = dict(dest)
    bad["means3D"] = torch.empty(P - 1, 3, device=DEV)
    with pytest.raises((_lib.GsplatError, RuntimeError)):
        _step(GaussianRasterizerBatch(sets, raw_params=True), pb, label, ups, grad_into=bad)


def test_grad_into_refuses_a_feature_width_the_kernels_pad():
    # F = 35 runs the F = 36 kernels (padded rows): a P x 35 destination is
    # not the backward's P x 36 output and must be refused, not mis-strided
    P, W, H, C, F = 3000, 96, 80, 2, 35
    sets = _cams(C, W, H)
    gen = torch.Generator(device=DEV).manual_seed(3)
    ups = [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen),
           torch.randn(C, F, H, W, device=DEV, generator=gen)]
    params = _raw_params(P, F, seed=5)
    opt = ShardedAdam(params, LRS, rank=0, world=1)
    dest = {_ARG[k]: v for k, v in opt.grad_views(0).items()}
    with pytest.raises((_lib.GsplatError, RuntimeError)):
        _step(GaussianRasterizerBatch(sets, raw_params=True), params, torch.ones(P, device=DEV), ups, grad_into=dest)
