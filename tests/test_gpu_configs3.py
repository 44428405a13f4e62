"""BASELINE configs[3] at its real per-rank shape on one GPU: the
300k-Gaussian scene, the 27-camera 800x800 rig, F = 32, sharded 8 ways
(camera c on rank c mod 8, distributed.shard_cameras; train.py:392-432 is the
reference loop).  Each of the 8 shards' 3-4-camera batch backward, summed,
must equal the 27-camera batch gradients, and one TimestepDriver step of the
rig at that size -- run as 8 ranks one after the other in this process, their
bound gradients summed as the bucket's all-reduce would -- must equal the
reference's per-camera formulation (one GaussianRasterizer per camera,
autograd summing, the densification statistics camera by camera).
Tolerance: 1e-5 relative L2 (fp32 summation order of the gradient atomics
and of the camera sums)."""
from __future__ import annotations

import pytest
import torch

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.distributed import shard_cameras
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings, GaussianRasterizer,
                                               GaussianRasterizerBatch)
from dynamic3dgaussians_amd.scene import make_gaussians
from dynamic3dgaussians_amd.timesteps import TimestepDriver, batch_renderer, params2rendervar

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
P, W, H, C, F, WORLD = 300_000, 800, 800, 27, 32, 8


def _settings():
    return [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.zeros(3, device=DEV), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(DEV), compat="reference") for c in camera_rig(C, W, H)]


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def test_eight_way_shards_sum_to_the_full_rig():
    g = make_gaussians(P, F=F, seed=0, device=DEV)
    src = {"means3D": g["means3D"], "colors_precomp": g["colors"], "opacities": g["opacities"],
           "scales": g["scales"], "rotations": g["rotations"], "semantic_feature": g["semantic_feature"]}
    sets = _settings()
    gen = torch.Generator(device=DEV).manual_seed(3)
    up_c = torch.randn(C, 3, H, W, device=DEV, generator=gen)
    up_d = torch.randn(C, 1, H, W, device=DEV, generator=gen)
    up_f = torch.randn(C, F, H, W, device=DEV, generator=gen)
    label = torch.ones(P, device=DEV)

    def grads(cams):
        leaves = {k: v.clone().requires_grad_(True) for k, v in src.items()}
        im, radius, feat, depth, _ = GaussianRasterizerBatch([sets[c] for c in cams])(
            means2D=torch.zeros(P, 3, device=DEV), label=label, **leaves)
        torch.autograd.backward([im, depth, feat], [up_c[cams], up_d[cams], up_f[cams]])
        return {k: v.grad for k, v in leaves.items()}

    full = grads(list(range(C)))
    shards = [shard_cameras(C, r, WORLD) for r in range(WORLD)]
    assert sorted(len(s) for s in shards) == [3, 3, 3, 3, 3, 4, 4, 4]
    total = {k: torch.zeros_like(v) for k, v in full.items()}
    for cams in shards:
        for k, v in grads(cams).items():
            total[k] += v
    for k in full:
        assert _rel(total[k], full[k]) <= 1e-5, (k, _rel(total[k], full[k]))


def test_eight_rank_driver_step_matches_per_camera_autograd():
    settings = _settings()
    g = make_gaussians(P, seed=1, device=DEV)
    base = {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
            "logit_opacities": torch.logit(g["opacities"]), "log_scales": torch.log(g["scales"])}
    tg = torch.rand(C, 3, H, W, device=DEV, generator=torch.Generator(device=DEV).manual_seed(7))
    render = batch_renderer(settings)
    # 8 ranks one after the other: each renders its shard, its bound .grad
    # views hold its share; their sum is what the bucket's all-reduce gives
    tot = {k: torch.zeros_like(v) for k, v in base.items()}
    stats = {k: torch.zeros(P, device=DEV) for k in ("means2D_gradient_accum", "denom", "max_2D_radius")}
    loss = 0.0
    for r in range(WORLD):
        params = {k: torch.nn.Parameter(v.clone()) for k, v in base.items()}
        opt = torch.optim.SGD([{"params": [params[k]], "name": k, "lr": 0.0} for k in params], lr=0.0)
        # the plain bucket path (its bound .grad views are what this test sums)
        drv = TimestepDriver(params, {}, opt, C, render, rank=r, world=WORLD, sharded=False)
        assert len(drv.cams) in (3, 4)
        loss += drv.step(tg)
        for k in tot:
            tot[k] += params[k].grad
        v = drv.variables
        stats["means2D_gradient_accum"] += v["means2D_gradient_accum"]
        stats["denom"] += v["denom"]
        torch.maximum(stats["max_2D_radius"], v["max_2D_radius"], out=stats["max_2D_radius"])
    # the reference formulation, camera by camera
    ref = {k: torch.nn.Parameter(v.clone()) for k, v in base.items()}
    accum, denom, maxr = (torch.zeros(P, device=DEV) for _ in range(3))
    ref_loss = 0.0
    for c, s in enumerate(settings):
        rv = params2rendervar(ref)
        im, radius, _ = GaussianRasterizer(s)(**rv)
        lc = torch.abs(im - tg[c]).mean() / C
        lc.backward()
        ref_loss += float(lc)
        seen = radius > 0
        accum[seen] += torch.norm(rv["means2D"].grad[seen, :2] * C, dim=-1)
        denom[seen] += 1
        maxr[seen] = torch.max(radius[seen].float(), maxr[seen])
    assert abs(loss - ref_loss) <= 1e-5 * abs(ref_loss)
    for k in base:
        assert _rel(tot[k], ref[k].grad) <= 1e-5, (k, _rel(tot[k], ref[k].grad))
    assert torch.equal(stats["denom"], denom)
    assert torch.equal(stats["max_2D_radius"], maxr)
    assert _rel(stats["means2D_gradient_accum"], accum) <= 1e-5
