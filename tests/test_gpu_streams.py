"""Cameras rendered on several HIP streams (bench.py's step) give the same
summed gradients as one stream, up to fp32 atomic order: the library keeps
no cross-call device state, and each forward/backward pair stays on its
stream."""
from __future__ import annotations

import pytest
import torch

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizer
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu


def _grads(n_streams, P=20000, W=160, H=128, cams=6, F=8):
    dev = torch.device("cuda", 0)
    g = make_gaussians(P, F=F, seed=0, device=dev)
    leaves = {k: g[k].clone().requires_grad_(True)
              for k in ("means3D", "colors", "opacities", "scales", "rotations", "semantic_feature")}
    gen = torch.Generator(device=dev).manual_seed(1)
    up = [torch.randn(3, H, W, device=dev, generator=gen), torch.randn(1, H, W, device=dev, generator=gen),
          torch.randn(F, H, W, device=dev, generator=gen)]
    main = torch.cuda.current_stream(dev)
    streams = [main] + [torch.cuda.Stream(device=dev) for _ in range(n_streams - 1)]
    for st in streams:
        st.wait_stream(main)
    for i, c in enumerate(camera_rig(cams, W, H)):
        rs = GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
            bg=torch.zeros(3, device=dev), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
            projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
            campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference")
        with torch.cuda.stream(streams[i % n_streams]):
            m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
            im, radius, feat, depth, _ = GaussianRasterizer(rs)(
                means3D=leaves["means3D"], means2D=m2, opacities=leaves["opacities"],
                colors_precomp=leaves["colors"], scales=leaves["scales"], rotations=leaves["rotations"],
                semantic_feature=leaves["semantic_feature"], label=torch.ones(P, device=dev))
            torch.autograd.backward([im, depth, feat], up)
    for st in streams:
        main.wait_stream(st)
    torch.cuda.synchronize()
    return {k: v.grad.clone() for k, v in leaves.items()}


def test_multi_stream_cameras_match_one_stream():
    a, b = _grads(1), _grads(4)
    for k in a:
        rel = ((a[k] - b[k]).norm() / a[k].norm().clamp_min(1e-30)).item()
        assert rel < 1e-5, (k, rel)


def _sink_vs_autograd(n_streams, use_sh, P=12000, W=144, H=112, cams=5, F=32):
    """Summed gradients of `cams` cameras: GradientSink (in-kernel
    accumulation) vs autograd's accumulation on the leaves."""
    from dynamic3dgaussians_amd.rasterizer import GradientSink
    dev = torch.device("cuda", 0)
    g = make_gaussians(P, F=F, seed=3, device=dev)
    gen = torch.Generator(device=dev).manual_seed(2)
    sh = torch.randn(P, 16, 3, device=dev, generator=gen) * 0.2
    label = (torch.rand(P, device=dev, generator=gen) > 0.3).float()
    up = [torch.randn(3, H, W, device=dev, generator=gen), torch.randn(1, H, W, device=dev, generator=gen),
          torch.randn(F, H, W, device=dev, generator=gen)]
    rig = camera_rig(cams, W, H)
    main = torch.cuda.current_stream(dev)
    streams = [main] + [torch.cuda.Stream(device=dev) for _ in range(n_streams - 1)]
    names = ["means3D", "opacities", "scales", "rotations", "semantic_feature"] + (["shs"] if use_sh else ["colors_precomp"])
    src = dict(means3D=g["means3D"], opacities=g["opacities"], scales=g["scales"], rotations=g["rotations"],
               semantic_feature=g["semantic_feature"], shs=sh, colors_precomp=g["colors"])
    out = {}
    sink = GradientSink()
    for mode in ("autograd", "sink"):
        leaves = {k: src[k].clone().requires_grad_(True) for k in names}
        m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
        for st in streams:
            st.wait_stream(main)
        sink.reset()
        for i, c in enumerate(rig):
            rs = GaussianRasterizationSettings(
                image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
                bg=torch.zeros(3, device=dev), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
                projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=3 if use_sh else 0,
                campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference",
                grad_sink=sink if mode == "sink" else None)
            with torch.cuda.stream(streams[i % n_streams]):
                im, radius, feat, depth, _ = GaussianRasterizer(rs)(means2D=m2, label=label, **leaves)
                torch.autograd.backward([im, depth, feat], up)
        for st in streams:
            main.wait_stream(st)
        if mode == "sink":
            gr = sink.gradients()
            out[mode] = {k: gr[k].clone() for k in names + ["means2D"]}
            assert all(leaves[k].grad is None for k in names)  # autograd added nothing
        else:
            out[mode] = {k: leaves[k].grad.clone() for k in names}
            out[mode]["means2D"] = m2.grad.clone()
    torch.cuda.synchronize()
    return out["autograd"], out["sink"]


@pytest.mark.parametrize("n_streams,use_sh", [(1, False), (3, False), (2, True)])
def test_gradient_sink_matches_autograd_sum(n_streams, use_sh):
    a, b = _sink_vs_autograd(n_streams, use_sh)
    for k in a:
        assert a[k].shape == b[k].shape, k
        rel = ((a[k] - b[k]).norm() / a[k].norm().clamp_min(1e-30)).item()
        assert rel < 1e-5, (k, rel)


@pytest.mark.parametrize("n_streams", [1, 3])
def test_gradient_sink_densify_stats_match_reference_bookkeeping(n_streams, P=12000, W=144, H=112, cams=5):
    """With a sink, means2D.grad is not populated; the per-camera statistics
    the reference derives from it (accumulate_mean2d_gradient,
    external.py:136-140, and max_2D_radius, train.py:288-290) come out of the
    backward kernel: equal to the reference's per-camera updates (norm of each
    camera's own means2D gradient) up to fp32 summation order."""
    from dynamic3dgaussians_amd.rasterizer import GradientSink
    dev = torch.device("cuda", 0)
    g = make_gaussians(P, F=0, seed=5, device=dev)
    gen = torch.Generator(device=dev).manual_seed(4)
    up = [torch.randn(3, H, W, device=dev, generator=gen), torch.randn(1, H, W, device=dev, generator=gen)]
    rig = camera_rig(cams, W, H)
    names = ["means3D", "opacities", "scales", "rotations", "colors_precomp"]
    src = dict(means3D=g["means3D"], opacities=g["opacities"], scales=g["scales"], rotations=g["rotations"],
               colors_precomp=g["colors"])

    def settings(c, sink=None):
        return GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
            bg=torch.zeros(3, device=dev), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
            projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
            campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference", grad_sink=sink)

    # the reference: one camera at a time, statistics from means2D.grad
    variables = {"means2D_gradient_accum": torch.zeros(P, device=dev), "denom": torch.zeros(P, device=dev),
                 "max_2D_radius": torch.zeros(P, device=dev)}
    for c in rig:
        leaves = {k: src[k].clone().requires_grad_(True) for k in names}
        m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
        im, radius, depth, _ = GaussianRasterizer(settings(c))(means2D=m2, label=torch.ones(P, device=dev),
                                                               **leaves)
        torch.autograd.backward([im, depth], up)
        seen = radius > 0
        variables["max_2D_radius"][seen] = torch.max(radius[seen], variables["max_2D_radius"][seen])
        variables["means2D_gradient_accum"][seen] += torch.norm(m2.grad[seen, :2], dim=-1)
        variables["denom"][seen] += 1
    # the sink, cameras over n_streams streams
    sink = GradientSink()
    mine = {k: torch.zeros(P, device=dev) for k in variables}
    mine["means2D_gradient_accum"] += 0.25  # running totals from earlier steps are kept
    main = torch.cuda.current_stream(dev)
    streams = [main] + [torch.cuda.Stream(device=dev) for _ in range(n_streams - 1)]
    for st in streams:
        st.wait_stream(main)
    sink.reset()
    leaves = {k: src[k].clone().requires_grad_(True) for k in names}
    m2 = torch.zeros_like(leaves["means3D"], requires_grad=True)
    with pytest.warns(RuntimeWarning, match="means2D.grad is not populated"):
        for i, c in enumerate(rig):
            with torch.cuda.stream(streams[i % n_streams]):
                im, radius, depth, _ = GaussianRasterizer(settings(c, sink))(
                    means2D=m2, label=torch.ones(P, device=dev), **leaves)
                torch.autograd.backward([im, depth], up)
    for st in streams:
        main.wait_stream(st)
    assert m2.grad is None
    sink.update_densify_stats(mine)
    torch.cuda.synchronize()
    assert int((variables["denom"] > 0).sum()) > P // 4  # the scene is seen
    torch.testing.assert_close(mine["denom"], variables["denom"], rtol=0, atol=0)
    torch.testing.assert_close(mine["max_2D_radius"], variables["max_2D_radius"], rtol=0, atol=0)
    torch.testing.assert_close(mine["means2D_gradient_accum"] - 0.25, variables["means2D_gradient_accum"],
                               rtol=1e-5, atol=1e-6)
