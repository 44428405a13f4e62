"""The binning passes' walk order (gs_gaussians.walk_order, ABI 12): the tile
histogram and bucket passes may walk the Gaussians in any permutation, and
the forward's outputs must not depend on it -- every tile list is sorted by
its unique (depth bits, id) keys, so the lists, and with them the images,
radii and the reference's counts, are bit-identical to the id-order walk;
gradients equal it up to fp32 atomic order.  Covered: the spatial (Morton)
order of GaussianRasterizerBatch(spatial_order=True) and an arbitrary
permutation, the sync-free and the two-phase forward, tile windows, both
bindings; _C.spatial_order is a permutation in non-decreasing Morton code;
debug mode refuses a walk order that is not a permutation."""
from __future__ import annotations

import pytest
import torch

from dynamic3dgaussians_amd import _C, _lib
from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizerBatch, rasterize_gaussians_batch

from .test_gpu_sync_free import _run, _same, _scene, _settings, _ups

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _morton(means):
    lo, hi = means.min(0).values, means.max(0).values
    ext = hi - lo
    q = torch.where(ext > 0, (means - lo) / ext * 1023.0, torch.zeros_like(means)).clamp(0, 1023).to(torch.int64)

    def spread(v):
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        return (v | (v << 2)) & 0x09249249
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)


def test_spatial_order_is_a_morton_sorted_permutation():
    P = 50_001
    means = make_means(P)
    order = _C.spatial_order(means)
    torch.cuda.synchronize()
    assert order.dtype == torch.int32 and order.numel() == P
    assert torch.equal(torch.sort(order.long()).values, torch.arange(P, device=DEV))
    codes = _morton(means)[order.long()]
    assert bool((codes[1:] >= codes[:-1]).all())


def make_means(P):
    g = torch.Generator(device=DEV).manual_seed(3)
    return (torch.randn(P, 3, device=DEV, generator=g) * torch.tensor([2.0, 1.0, 0.5], device=DEV)).contiguous()


@pytest.mark.parametrize("binding", ["native", "ctypes"])
@pytest.mark.parametrize("sync_free", [True, False])
def test_spatial_walk_gives_the_id_order_outputs(binding, sync_free, P=20000, W=208, H=160, F=32, C=5):
    src = _scene(P, F, seed=4)
    rig = camera_rig(C, W, H)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    sets = _settings(rig, W, H, windows=[None, (0, 2, gx, gy - 3), None, None, (1, 0, gx - 2, gy)])
    ups = _ups(C, F, W, H)
    lab = torch.ones(P, device=DEV)
    assert _C.native_loaded(), "the native binding did not load"
    keep = _C._native
    try:
        _C._native = keep if binding == "native" else None
        ref_o, ref_g = _run(GaussianRasterizerBatch(sets, sync_free=sync_free), src, ups, lab)
        ras = GaussianRasterizerBatch(sets, sync_free=sync_free, spatial_order=True, order_refresh=2)
        for _ in range(3):  # the order computed, reused, recomputed
            o, g = _run(ras, src, ups, lab)
            _same(o, ref_o, g, ref_g)
        assert ras._walk is not None and ras._walk.numel() == P
    finally:
        _C._native = keep


def test_any_permutation_gives_the_id_order_outputs(P=15000, W=160, H=128, F=32, C=3):
    src = _scene(P, F, seed=6)
    sets = _settings(camera_rig(C, W, H), W, H)
    lab = torch.ones(P, device=DEV)

    def forward(walk):
        out = rasterize_gaussians_batch(src["means3D"], torch.zeros(P, 3, device=DEV), None, src["colors_precomp"],
                                        src["semantic_feature"], src["opacities"], src["scales"],
                                        src["rotations"], None, sets, label=lab, walk_order=walk)
        torch.cuda.synchronize()
        return [t.detach().clone() for t in out]
    ref = forward(None)
    g = torch.Generator(device=DEV).manual_seed(9)
    for walk in (torch.arange(P - 1, -1, -1, device=DEV, dtype=torch.int32),
                 torch.randperm(P, device=DEV, generator=g).to(torch.int32)):
        for a, b in zip(forward(walk.contiguous()), ref):
            assert torch.equal(a, b)


def test_debug_mode_refuses_a_walk_that_is_not_a_permutation(P=4000, W=96, H=80, F=0, C=2):
    src = _scene(P, 32, seed=7)
    sets = _settings(camera_rig(C, W, H), W, H)
    sets = [s._replace(debug=True) for s in sets]
    walk = torch.arange(P, device=DEV, dtype=torch.int32)
    walk[5] = 7  # id 7 twice, id 5 never
    with pytest.raises((_lib.GsplatError, RuntimeError), match="walk order"):
        rasterize_gaussians_batch(src["means3D"], torch.zeros(P, 3, device=DEV), None, src["colors_precomp"],
                                  None, src["opacities"], src["scales"], src["rotations"], None, sets,
                                  walk_order=walk)


@pytest.mark.parametrize("P", [1, 2, 63, 64, 65, 257])
def test_spatial_order_small_and_degenerate(P):
    means = make_means(P)
    if P > 2:
        means[: P // 2] = means[0]  # repeated points: equal codes keep id order (stable sort)
    order = _C.spatial_order(means)
    torch.cuda.synchronize()
    assert torch.equal(torch.sort(order.long()).values, torch.arange(P, device=DEV))
    codes = _morton(means)[order.long()]
    assert bool((codes[1:] >= codes[:-1]).all())
    eq = codes[1:] == codes[:-1]
    assert bool((order[1:][eq] > order[:-1][eq]).all())  # ties in id order
    assert _C.spatial_order(torch.zeros(0, 3, device=DEV)).numel() == 0
