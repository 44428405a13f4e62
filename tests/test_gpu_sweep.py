"""Seeded sweep of small random configurations: the HIP forward and backward
against the CPU oracle at the tolerances of test_gpu_parity.py (SURVEY.md
8(c)).  Each case draws image size (odd sizes, not multiples of the 16-pixel
tile), scene size and Gaussian extent, scene seed, camera of the 27-camera
rig or an off-centre principal point, feature width (every instantiation:
plain VALU widths, the padded ones, the matrix-core 32/64 and the fused 36),
SH degree or precomputed colours, scale modifier, background and compat mode
from one fixed generator, so the case list is the same on every run.  A
second sweep holds random camera batches (2-6 rig cameras, the bench's
GaussianRasterizerBatch path) directly to the oracle: every camera's
forward, and the camera-summed backward against the summed oracle
backwards.

The reference's own entry points are the same for every case
(CR/rasterizer_impl.cu:195-357 forward, :359-433 backward); the sweep only
varies the inputs the reference's tests and callers vary (train.py:246-249,
external.py calc_psnr inputs, dyn_train.py F = 32)."""
import numpy as np
import pytest

from tests import _harness as H
from tests.test_gpu_parity import GRAD_NAMES, _cmp_forward

pytestmark = pytest.mark.gpu

_FWIDTHS = [0, 3, 5, 8, 16, 20, 32, 35, 36, 64]


def _cases(n=40, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        W = int(rng.integers(17, 200))
        Hh = int(rng.integers(15, 160))
        kw = dict(W=W, H=Hh, P=int(rng.integers(200, 5000)), seed=int(rng.integers(0, 1000)),
                  F=int(rng.choice(_FWIDTHS)), scale_mult=float(rng.uniform(1.0, 6.0)),
                  bg=tuple(float(x) for x in rng.uniform(0.0, 1.0, 3).round(3)))
        if rng.uniform() < 0.3:
            kw.update(cx=float(rng.uniform(0.2, 0.8) * W), cy=float(rng.uniform(0.2, 0.8) * Hh))
        else:
            kw["cam_index"] = int(rng.integers(0, 27))
        if rng.uniform() < 0.35:
            kw.update(use_sh=True, sh_degree=int(rng.integers(0, 4)))
        mod = float(rng.choice([1.0, 1.0, 0.6, 1.4]))
        compat = "fixed" if rng.uniform() < 0.4 else "reference"
        out.append(pytest.param(kw, mod, compat, id=f"case{i}"))
    return out


@pytest.mark.parametrize("kw,mod,compat", _cases())
def test_random_config_forward_backward(kw, mod, compat):
    inp = H.scene(**kw)
    inp["scale_modifier"] = mod
    F = kw["F"]
    g, o = _cmp_forward(inp, compat, F)
    grads = H.upstream_grads(inp["image_height"], inp["image_width"], F, seed=kw["seed"] + 1)
    gb = H.gpu_backward(inp, g, grads, compat)
    ob = H.oracle_backward(inp, o, grads, compat)
    for name, a, b in zip(GRAD_NAMES, gb, ob):
        assert a.shape == b.shape, name
        if b.size == 0 or not np.any(b):
            assert not np.any(a) or np.abs(a).max() < 1e-6, name
            continue
        assert H.rel_l2(a, b) <= 1e-4, (name, H.rel_l2(a, b))


def _batch_cases(n=8, seed=77):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kw = dict(W=int(rng.integers(40, 180)), H=int(rng.integers(30, 140)), P=int(rng.integers(500, 4000)),
                  seed=int(rng.integers(0, 1000)), F=int(rng.choice([0, 8, 32, 36])),
                  scale_mult=float(rng.uniform(1.5, 5.0)),
                  bg=tuple(float(x) for x in rng.uniform(0.0, 1.0, 3).round(3)))
        if rng.uniform() < 0.3:
            kw.update(use_sh=True, sh_degree=int(rng.integers(1, 4)))
        cams = sorted(int(c) for c in rng.choice(27, size=int(rng.integers(2, 7)), replace=False))
        compat = "fixed" if rng.uniform() < 0.4 else "reference"
        out.append(pytest.param(kw, cams, compat, id=f"batch{i}"))
    return out


@pytest.mark.parametrize("kw,cams,compat", _batch_cases())
def test_random_camera_batch_against_oracle(kw, cams, compat):
    """The bench's own path (one launch per stage for a camera batch) held
    directly to the oracle: camera c's forward outputs at the per-camera
    tolerances, and the batch backward's camera-summed gradients against
    the sum of the oracle's per-camera backwards (relative L2 <= 1e-4)."""
    import torch
    from dynamic3dgaussians_amd import _C
    dev = H.DEV
    F = kw["F"]
    inps = [H.scene(cam_index=c, **kw) for c in cams]
    i0 = inps[0]
    d = lambda k: H._to(i0[k], dev)  # noqa: E731
    st = lambda k: torch.stack([x[k] for x in inps]).to(dev)  # noqa: E731
    fl = lambda k: [float(x[k]) for x in inps]  # noqa: E731
    Hh, W = i0["image_height"], i0["image_width"]
    out = _C.rasterize_gaussians_batch(
        d("bg"), d("means3D"), d("colors"), d("semantic_feature"), d("opacity"), d("scales"), d("rotations"),
        i0["scale_modifier"], d("cov3D_precomp"), st("viewmatrix"), st("projmatrix"), fl("c_x"), fl("c_y"),
        fl("tan_fovx"), fl("tan_fovy"), Hh, W, d("sh"), i0["degree"], st("campos"), False, False, compat=compat)
    torch.cuda.synchronize()
    NR, color, feat, depth, alpha, radii, geom, binning, img, NI = out
    grads = [H.upstream_grads(Hh, W, F, seed=kw["seed"] + 1 + k) for k in range(len(cams))]
    osum = None
    for k, inp in enumerate(inps):
        o = H.oracle_forward(inp, compat)
        Lo, co, fo, do, ao, ro, _ = o
        assert NR[k] == Lo, (k, NR[k], Lo)
        np.testing.assert_array_equal(radii[k].cpu().numpy(), ro)
        cg = color[k].cpu().numpy()
        assert H.psnr(cg, co) >= 80.0
        assert np.mean(np.abs(cg - co) <= 1e-5) >= 0.999
        assert np.mean(np.abs(depth[k].cpu().numpy() - do) <= 1e-5 * max(1.0, np.abs(do).max())) >= 0.999
        assert np.mean(np.abs(alpha[k].cpu().numpy() - ao) <= 1e-5) >= 0.999
        if F:
            assert np.mean(np.abs(feat[k].cpu().numpy() - fo) <= 1e-5) >= 0.999
        ob = H.oracle_backward(inp, o, grads[k], compat)
        osum = [np.array(b, dtype=np.float64) for b in ob] if osum is None else \
            [s + b for s, b in zip(osum, ob)]
    swap = compat == "reference"
    cam4 = (fl("tan_fovx"), fl("tan_fovy"), fl("c_x"), fl("c_y")) if swap else \
        (fl("c_x"), fl("c_y"), fl("tan_fovx"), fl("tan_fovy"))
    up = [torch.stack([g[j] for g in grads]).to(dev) for j in range(4)]
    gb = _C.rasterize_gaussians_batch_backward(
        d("bg"), d("means3D"), radii, d("colors"), d("semantic_feature"), d("scales"), d("rotations"),
        i0["scale_modifier"], d("cov3D_precomp"), st("viewmatrix"), st("projmatrix"), *cam4,
        up[0], up[1] if F else None, up[2], up[3], d("sh"), i0["degree"], st("campos"), geom, NI, binning,
        img, alpha, False, compat=compat)
    torch.cuda.synchronize()
    for name, a, b in zip(GRAD_NAMES, gb, osum):
        a = a.cpu().numpy()
        assert a.shape == b.shape, name
        if b.size == 0 or not np.any(b):
            assert not np.any(a) or np.abs(a).max() < 1e-6, name
            continue
        assert H.rel_l2(a, b) <= 1e-4, (name, H.rel_l2(a, b))
