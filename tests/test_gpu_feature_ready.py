"""gs_gaussians.feature_ready (ABI 10): the forward blend waits for an event
recorded on another stream before it reads semantic_feature -- bench.py's
overlapped feature all-reduce + optimizer step (N > 1) writes the features on
a side stream while the next step's preprocess / sort already run.

The side stream sleeps ~tens of ms before it writes the features, so a blend
that did not wait would read the stale (zero) buffer; the feature map must
equal a synchronous render of the written features.  F = 32 hands the event
to the kernels; F = 35 (padded to a compiled width by the binding) waits on
the calling stream before the pad copy."""
from __future__ import annotations

import pytest
import torch

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizerBatch
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _settings(cams, W, H):
    return [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.zeros(3, device=DEV), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(DEV)) for c in cams]


@pytest.mark.parametrize("F", [32, 35])
def test_forward_waits_for_feature_ready(F, P=20000, W=160, H=128, C=3):
    g = make_gaussians(P, F=F, seed=3, device=DEV)
    kw = dict(means3D=g["means3D"], colors_precomp=g["colors"], opacities=g["opacities"], scales=g["scales"],
              rotations=g["rotations"])
    ras = GaussianRasterizerBatch(_settings(camera_rig(C, W, H), W, H))
    target = g["semantic_feature"].contiguous()
    im_ref, feat_ref, _, _ = ras(means2D=torch.zeros(P, 3, device=DEV), semantic_feature=target, **kw)
    torch.cuda.synchronize()
    buf = torch.zeros_like(target)
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    ev = torch.cuda.Event()
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)  # ~0.1 s at the shader clock
        buf.copy_(target)
        ev.record(side)
    buf.record_stream(side)
    im, feat, _, _ = ras(means2D=torch.zeros(P, 3, device=DEV), semantic_feature=buf, feature_ready=ev, **kw)
    torch.cuda.synchronize()
    assert torch.equal(im, im_ref)
    assert float(feat_ref.abs().max()) > 0
    assert torch.equal(feat, feat_ref)
