"""The per-timestep driver on the HIP batch renderer (GPU): one driver step
equals the reference's per-camera formulation of the same loss -- one
GaussianRasterizer per camera, autograd summing the cameras' gradients, the
densification statistics accumulated camera by camera as
external.py:136-140 / train.py:288-290 do -- and a short two-timestep run
trains (the timestep-0 fit loss falls, timestep 1 starts from the
constant-velocity initialisation)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.optim import FusedAdam
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
from dynamic3dgaussians_amd.scene import make_gaussians
from dynamic3dgaussians_amd.timesteps import TimestepDriver, batch_renderer, params2rendervar

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
N_CAMS, W, H, P = 5, 160, 128, 6000
LRS = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
       "log_scales": 1e-3}


def _settings():
    return [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.zeros(3, device=DEV), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(DEV), compat="reference")
        for c in camera_rig(N_CAMS, W, H, seed=3)]


def _params(seed=0):
    g = make_gaussians(P, seed=seed, device=DEV)
    return {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
            "logit_opacities": torch.logit(g["opacities"]), "log_scales": torch.log(g["scales"])}


def _leaf(p):
    return {k: torch.nn.Parameter(v.clone()) for k, v in p.items()}


def _targets(seed):
    return torch.rand(N_CAMS, 3, H, W, device=DEV, generator=torch.Generator(device=DEV).manual_seed(seed))


def _rel(a, b):
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def test_driver_step_matches_per_camera_autograd():
    settings = _settings()
    tg = _targets(7)
    # the driver: one batch launch per stage, the bucket's bound gradients
    params = _leaf(_params())
    opt = torch.optim.SGD([{"params": [params[k]], "name": k, "lr": 0.0} for k in LRS], lr=0.0)
    drv = TimestepDriver(params, {}, opt, N_CAMS, batch_renderer(settings))
    loss = drv.step(tg)
    grads = {k: params[k].grad.detach().clone() for k in LRS}
    v = drv.variables
    # the reference's formulation: camera by camera
    ref = _leaf(_params())
    accum = torch.zeros(P, device=DEV)
    denom = torch.zeros(P, device=DEV)
    maxr = torch.zeros(P, device=DEV)
    ref_loss = 0.0
    for c, s in enumerate(settings):
        rv = params2rendervar(ref)
        im, radius, _ = GaussianRasterizer(s)(**rv)
        lc = torch.abs(im - tg[c]).mean() / N_CAMS
        lc.backward()
        ref_loss += float(lc)
        seen = radius > 0
        # the reference's per-view statistic: the norm of the means2D gradient
        # of its one-camera loss, N_CAMS x this camera's share of the rig mean
        accum[seen] += torch.norm(rv["means2D"].grad[seen, :2] * N_CAMS, dim=-1)
        denom[seen] += 1
        maxr[seen] = torch.max(radius[seen].float(), maxr[seen])
    np.testing.assert_allclose(loss, ref_loss, rtol=1e-5)
    for k in LRS:
        assert _rel(grads[k], ref[k].grad) < 1e-5, (k, _rel(grads[k], ref[k].grad))
    assert torch.equal(v["denom"], denom)
    assert torch.equal(v["max_2D_radius"], maxr)
    assert _rel(v["means2D_gradient_accum"], accum) < 1e-5


def test_two_timesteps_fit():
    settings = _settings()
    render = batch_renderer(settings)
    with torch.no_grad():
        tg0, _ = render(params2rendervar(_params()), list(range(N_CAMS)))
        tg0 = tg0.detach().clone()
    params = _leaf(_params())
    with torch.no_grad():
        params["rgb_colors"].add_(0.3 * torch.randn_like(params["rgb_colors"])).clamp_(0, 1)
    opt = FusedAdam([{"params": [params[k]], "name": k, "lr": lr * 4} for k, lr in LRS.items()], lr=0.0, eps=1e-15)
    drv = TimestepDriver(params, {}, opt, N_CAMS, render)
    losses = drv.run(2, lambda t: 12 if t == 0 else 3, lambda t: tg0)
    assert losses[0][-1] < 0.7 * losses[0][0], losses[0]
    # timestep 1: means started from 2 x (end of t0) - (start of t1's prev) = constant velocity
    v = drv.variables
    assert "prev_pts" in v and v["prev_pts"].shape == (P, 3)
    assert all(np.isfinite(losses[1]))
    for k in LRS:
        assert torch.isfinite(drv.params[k]).all()
