"""CPU tests of the oracle itself (no GPU): pinned against the reference's
own Python SH evaluator (golden fixture), closed-form known answers derived
from the reference formulas, finite differences in the "fixed" compat mode,
and the documented quirks of the "reference" mode."""
import os

import numpy as np
import pytest

from dynamic3dgaussians_amd.camera import camera_rig, setup_camera
from dynamic3dgaussians_amd.scene import make_gaussians
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _single(W=32, Hh=32, s=0.05, z=2.0, op=0.8, col=(1.0, 0.5, 0.25)):
    cam = setup_camera(W, Hh, np.array([[32, 0, 16], [0, 32, 16], [0, 0, 1.0]]), np.eye(4))
    out = O.rasterize_gaussians(np.zeros(3, np.float32), np.array([[0, 0, z]], np.float32),
                                np.array([col], np.float32), None, np.array([[op]], np.float32),
                                np.full((1, 3), s, np.float32), np.array([[1, 0, 0, 0]], np.float32),
                                1.0, None, cam.viewmatrix, cam.projmatrix, cam.c_x, cam.c_y,
                                cam.tanfovx, cam.tanfovy, Hh, W, None, 0, cam.campos)
    return cam, out


def test_single_gaussian_closed_form():
    """radius 4, xy (15.5, 15.5), conic 1/0.94 for s=0.05, z=2, f=32."""
    cam, (L, color, feat, depth, alpha, radii, st) = _single()
    assert radii[0] == 4 and L == 4  # 4 of the 2x2 tiles
    np.testing.assert_allclose(st.means2D[0], [15.5, 15.5])
    # cov2D = (f s / z)^2 + 0.3 = 0.64 + 0.3 -> conic 1/0.94
    np.testing.assert_allclose(st.conic_opacity[0], [1 / 0.94, 0, 1 / 0.94, 0.8], rtol=1e-6)
    ys, xs = np.mgrid[0:32, 0:32].astype(np.float64)
    q = ((xs - 15.5) ** 2 + (ys - 15.5) ** 2) / 0.94
    a = np.minimum(0.99, 0.8 * np.exp(-0.5 * q))
    a[a < 1 / 255] = 0
    np.testing.assert_allclose(color[0], a, atol=2e-7)
    np.testing.assert_allclose(color[1], 0.5 * a, atol=2e-7)
    np.testing.assert_allclose(depth[0], 2.0 * a, atol=5e-7)
    assert not alpha.any(), "Q1: the reference never writes out_alpha"


def test_fixed_alpha_and_background():
    cam, _ = _single()
    out = O.rasterize_gaussians(np.array([0.2, 0.4, 0.6], np.float32),
                                np.array([[0, 0, 2.0]], np.float32), np.array([[1, 1, 1]], np.float32),
                                None, np.array([[0.8]], np.float32), np.full((1, 3), 0.05, np.float32),
                                np.array([[1, 0, 0, 0]], np.float32), 1.0, None, cam.viewmatrix,
                                cam.projmatrix, 16, 16, cam.tanfovx, cam.tanfovy, 32, 32, None, 0,
                                cam.campos, compat="fixed")
    L, color, feat, depth, alpha, radii, st = out
    T = 1 - alpha[0]
    np.testing.assert_allclose(color[0], (1 - T) + 0.2 * T, atol=1e-6)
    np.testing.assert_allclose(color[2], (1 - T) + 0.6 * T, atol=1e-6)


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_colour_matches_reference_eval_sh(deg):
    """Golden: the reference's utils/sh_utils.py eval_sh (+0.5, clamp >= 0)."""
    gold = np.load(os.path.join(GOLD, "sh_eval.npz"))
    means = gold["means3D"]
    P = means.shape[0]
    M = (deg + 1) ** 2
    sh = np.ascontiguousarray(gold["shs"][:, :M])
    campos = gold["campos"]
    # a camera looking down +z from campos so that every point is in front of it
    w2c = np.eye(4, dtype=np.float32)
    w2c[:3, 3] = -campos
    cam = setup_camera(64, 64, np.array([[40, 0, 32], [0, 40, 32], [0, 0, 1.0]]), w2c)
    radii = np.zeros(P, np.int32)
    st = dict(means2D=np.zeros((P, 2), np.float32), depths=np.zeros(P, np.float32),
              cov3D=np.zeros((P, 6), np.float32), rgb=np.zeros((P, 3), np.float32),
              co=np.zeros((P, 4), np.float32), tiles=np.zeros(P, np.uint32),
              cl=np.zeros((P, 3), np.uint8))
    L_ = O.lib()
    p = O._p
    L_.or_preprocess(P, deg, M, p(means), p(np.full((P, 3), 0.1, np.float32)), 1.0,
                     p(np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1))),
                     p(np.full(P, 0.5, np.float32)), p(sh), None, None, p(cam.viewmatrix),
                     p(cam.projmatrix), p(campos.astype(np.float32)), 64, 64, 32.0, 32.0,
                     cam.tanfovx, cam.tanfovy, 0, p(radii, O._i), p(st["means2D"]), p(st["depths"]),
                     p(st["cov3D"]), p(st["rgb"]), p(st["co"]), p(st["tiles"], O._u32),
                     p(st["cl"], O._u8))
    vis = radii > 0
    assert vis.sum() > P // 2
    np.testing.assert_allclose(st["rgb"][vis], gold[f"rgb_deg{deg}"][vis], rtol=2e-6, atol=2e-6)
    np.testing.assert_array_equal(st["cl"][vis].astype(bool), gold[f"clamped_deg{deg}"][vis])


def test_higher_msb_values():
    """getHigherMsb end bits quoted in SURVEY.md 8(a)."""
    assert O.higher_msb(256) == 9
    assert O.higher_msb(2500) == 12
    assert O.higher_msb(8160) == 13


def test_binning_is_sorted_and_stable():
    g = make_gaussians(800, seed=3, scale_mult=3.0)
    cam = camera_rig(27, 96, 80)[2]
    L, *_, st = O.rasterize_gaussians(np.zeros(3, np.float32), g["means3D"], g["colors"], None,
                                      g["opacities"], g["scales"], g["rotations"], 1.0, None,
                                      cam.viewmatrix, cam.projmatrix, cam.c_x, cam.c_y, cam.tanfovx,
                                      cam.tanfovy, 80, 96, None, 0, cam.campos)
    k = st.keys
    assert np.all(np.diff(k.astype(np.float64)) >= 0) or np.all(k[1:] >= k[:-1])
    # ties (same tile, same depth) keep Gaussian-index order
    same = k[1:] == k[:-1]
    assert np.all(st.point_list[1:][same] > st.point_list[:-1][same])
    # ranges cover the list exactly
    r = st.ranges.reshape(-1, 2)
    assert r[:, 1].max() == L and np.sum(r[:, 1] - r[:, 0]) == L


def _smooth_scene(P=8, F=4, seed=3):
    """A few large, semi-transparent Gaussians covering the whole 40x32 image:
    every pixel passes alpha >= 1/255 for every Gaussian and T stays > 1e-4,
    so the rendered images are smooth in all parameters (no threshold jumps)
    and central differences are a valid check of the analytic gradients."""
    from dynamic3dgaussians_amd.camera import intrinsics, look_at_w2c
    rng = np.random.default_rng(seed)
    g = dict(means3D=(rng.standard_normal((P, 3)) * 0.05).astype(np.float32),
             colors=rng.random((P, 3)).astype(np.float32),
             semantic_feature=rng.standard_normal((P, F)).astype(np.float32),
             opacities=(0.1 + 0.3 * rng.random((P, 1))).astype(np.float32),
             scales=(0.4 + 0.3 * rng.random((P, 3))).astype(np.float32),
             rotations=rng.standard_normal((P, 4)).astype(np.float32))
    g["rotations"] /= np.linalg.norm(g["rotations"], axis=1, keepdims=True)
    W, Hh = 40, 32
    cam = setup_camera(W, Hh, intrinsics(W, Hh, 30.0), look_at_w2c([0.3, -0.4, 2.5]))
    return g, cam, W, Hh, F


def _loss_and_grads(g, cam, W, Hh, compat, F, seed=0, swap=False):
    rng = np.random.default_rng(seed)
    wc = rng.standard_normal((3, Hh, W)).astype(np.float32)
    wf = rng.standard_normal((F, Hh, W)).astype(np.float32)
    wd = rng.standard_normal((1, Hh, W)).astype(np.float32) * 0.1
    wa = rng.standard_normal((1, Hh, W)).astype(np.float32)

    def fwd(gg):
        out = O.rasterize_gaussians(np.zeros(3, np.float32), gg["means3D"], gg["colors"],
                                    gg.get("semantic_feature"), gg["opacities"], gg["scales"],
                                    gg["rotations"], 1.0, None, cam.viewmatrix, cam.projmatrix,
                                    cam.c_x, cam.c_y, cam.tanfovx, cam.tanfovy, Hh, W, None, 0,
                                    cam.campos, compat=compat)
        L, color, feat, depth, alpha, radii, st = out
        loss = float(np.sum(color.astype(np.float64) * wc) + np.sum(feat.astype(np.float64) * wf)
                     + np.sum(depth.astype(np.float64) * wd) + np.sum(alpha.astype(np.float64) * wa))
        return loss, out

    loss, out = fwd(g)
    L, color, feat, depth, alpha, radii, st = out
    cam4 = (cam.tanfovx, cam.tanfovy, cam.c_x, cam.c_y) if swap else \
        (cam.c_x, cam.c_y, cam.tanfovx, cam.tanfovy)
    grads = O.rasterize_gaussians_backward(
        np.zeros(3, np.float32), g["means3D"], radii, g["colors"], g.get("semantic_feature"),
        g["scales"], g["rotations"], 1.0, None, cam.viewmatrix, cam.projmatrix, *cam4,
        wc, wf, wd, wa, None, 0, cam.campos, st, L, None, None, alpha, compat=compat)
    return fwd, grads, radii


@pytest.mark.parametrize("key,gi", [("colors", 1), ("semantic_feature", 2), ("opacities", 3),
                                     ("means3D", 4), ("scales", 7), ("rotations", 8)])
def test_fixed_mode_gradients_match_finite_differences(key, gi):
    """In "fixed" mode the analytic gradients are the true derivatives of the
    rendered colour, 32-ch-style features, depth and alpha: central
    differences (float64 loss) agree to < 3e-3 relative L2 for every
    parameter, through the whole EWA / covariance / quaternion chain."""
    g, cam, W, Hh, F = _smooth_scene()
    fwd, grads, radii = _loss_and_grads(g, cam, W, Hh, "fixed", F)
    assert np.all(radii > 0)
    ana = grads[gi].reshape(g[key].shape[0], -1)
    eps = 1e-2 if key in ("colors", "semantic_feature") else 1e-3
    num = np.zeros_like(ana)
    for i in range(ana.shape[0]):
        for c in range(ana.shape[1]):
            gp = {k: v.copy() for k, v in g.items()}
            gm = {k: v.copy() for k, v in g.items()}
            gp[key][i, c] += eps
            gm[key][i, c] -= eps
            num[i, c] = (fwd(gp)[0] - fwd(gm)[0]) / (2 * eps)
    err = np.linalg.norm(num - ana) / np.linalg.norm(num)
    assert err < 3e-3, (key, err)


def test_reference_mode_swapped_camera_args_shrink_scale_grads():
    """Q2: with the Python-order (swapped) camera scalars the reference's
    dL/dscale differs strongly from the one computed with the intended order
    (~7x smaller on its probe scene)."""
    g, cam, W, Hh, F = _smooth_scene()
    _, gs, _ = _loss_and_grads(g, cam, W, Hh, "reference", F, swap=True)
    _, gi_, _ = _loss_and_grads(g, cam, W, Hh, "reference", F, swap=False)
    assert np.linalg.norm(gs[7] - gi_[7]) / np.linalg.norm(gi_[7]) > 0.2


def test_reference_mode_quirks_change_gradients():
    """Q1 (alpha never written -> T_final = 1) makes the reference-mode colour
    gradient differ from the true one; Q5 drops the feature term."""
    g, cam, W, Hh, F = _smooth_scene()
    _, gref, _ = _loss_and_grads(g, cam, W, Hh, "reference", F)
    _, gfix, _ = _loss_and_grads(g, cam, W, Hh, "fixed", F)
    rel = np.linalg.norm(gref[1] - gfix[1]) / np.linalg.norm(gfix[1])
    assert rel > 0.05


def _cov3d_oracle(scales, rotations, mod):
    """The oracle's forward 3D covariance of every Gaussian (means in front of
    a camera so none is culled before computeCov3D, CR/forward.cu:181-204)."""
    P = scales.shape[0]
    cam = setup_camera(64, 64, np.array([[64, 0, 32], [0, 64, 32], [0, 0, 1.0]]), np.eye(4))
    means = np.zeros((P, 3), np.float32)
    means[:, 2] = 3.0
    out = O.rasterize_gaussians(np.zeros(3, np.float32), means, np.ones((P, 3), np.float32), None,
                                np.full((P, 1), 0.5, np.float32), scales.astype(np.float32),
                                rotations.astype(np.float32), mod, None, cam.viewmatrix, cam.projmatrix,
                                cam.c_x, cam.c_y, cam.tanfovx, cam.tanfovy, 64, 64, None, 0, cam.campos)
    return out[6].cov3D


@pytest.mark.parametrize("tag,mod", [("1", 1.0), ("0p7", 0.7)])
def test_cov3d_matches_reference_python(tag, mod):
    """Golden (tests/golden/cov3d.npz): the reference's own Python 3D
    covariance -- utils/general_utils.py build_scaling_rotation /
    strip_symmetric composed as scene/gaussian_model.py:40-44 -- pins the
    oracle's computeCov3D (CR/forward.cu:129-163; the HIP preprocess equals
    the oracle bit for bit, tests/test_gpu_parity.py).  fp32 in both, in
    different operation orders (matmul vs explicit dot products): 99.6 % of
    the entries are bit-identical, every |diff| <= 2e-6 of the covariance's
    largest diagonal entry (measured 6.7e-7).  Q7: the Python builds the rotation from the NORMALISED
    quaternion, the CUDA kernel (and so the oracle) from the raw one -- equal
    for unit quaternions (held here), not for raw ones (shown here)."""
    d = np.load(os.path.join(GOLD, "cov3d.npz"))
    ref = d[f"cov3D_mod{tag}"]
    scale = np.abs(ref[:, [0, 3, 5]]).max(axis=1, keepdims=True)
    got = _cov3d_oracle(d["scales"], d["rotations_unit"], mod)
    assert np.all(np.abs(got - ref) <= 2e-6 * scale), float(np.max(np.abs(got - ref) / scale))
    assert np.mean(got == ref) >= 0.99
    raw = _cov3d_oracle(d["scales"], d["rotations_raw"], mod)
    norms = np.linalg.norm(d["rotations_raw"], axis=1)
    off_unit = np.abs(norms - 1.0) > 0.05
    assert np.all(np.max(np.abs(raw - ref) / scale, axis=1)[off_unit] > 1e-3)


def test_setup_camera_matches_reference_camera_matrices():
    """Golden (tests/golden/cameras.npz): the 3DGS camera of the reference --
    utils/graphics_utils.py getWorld2View2 / getProjectionMatrix composed as
    scene/cameras.py:49-52 -- against camera.setup_camera, the helpers.py:68-95
    form (OpenCV K + w2c) that builds every raster setting here, at a centred
    principal point where both describe the same camera: view matrix, full
    projection and camera centre (fp32, rtol 1e-5)."""
    d = np.load(os.path.join(GOLD, "cameras.npz"))
    for i in range(len(d["W"])):
        W, H = int(d["W"][i]), int(d["H"][i])
        fx = W / (2 * np.tan(d["fovx"][i] / 2))
        fy = H / (2 * np.tan(d["fovy"][i] / 2))
        K = np.array([[fx, 0, W / 2], [0, fy, H / 2], [0, 0, 1.0]])
        w2c = np.eye(4)
        w2c[:3, :3] = d["R"][i].T  # getWorld2View2: Rt[:3, :3] = R^T, Rt[:3, 3] = t
        w2c[:3, 3] = d["T"][i]
        cam = setup_camera(W, H, K, w2c)
        np.testing.assert_allclose(cam.viewmatrix, d["world_view_transform"][i], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(cam.projmatrix, d["full_proj_transform"][i], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(cam.campos, d["camera_center"][i], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(cam.tanfovx, np.tan(d["fovx"][i] / 2), rtol=1e-6)
