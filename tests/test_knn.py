"""Exact k-NN against a brute-force float64 oracle
(oracle/neighbor.py knn: the reference's o3d_knn contract -- k nearest other
points, squared distances in double, here ties to the lower index) and the
params.npz format of helpers.py:149-167."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import neighbor as ON


def _cloud(N, kind, seed=0):
    g = np.random.default_rng(seed)
    if kind == "uniform":
        p = g.random((N, 3))
    elif kind == "clusters":  # dense blobs + sparse outliers, like a capture
        c = g.random((8, 3)) * 4
        p = c[g.integers(0, 8, N)] + g.normal(0, 0.02, (N, 3))
        p[: N // 50] = g.random((N // 50, 3)) * 10 - 3
    elif kind == "plane":  # flat (one extent ~0) and grid-aligned: many ties
        p = np.stack([g.integers(0, 40, N) * 0.05, g.integers(0, 40, N) * 0.05, np.zeros(N)], 1)
    else:
        raise ValueError(kind)
    return p.astype(np.float32)


# ------------------------------------------------------------------- CPU

def test_params_npz_roundtrip(tmp_path):
    from dynamic3dgaussians_amd.params_io import load_params, params2cpu, save_params
    t0 = {k: torch.randn(5, c) for k, c in (("means3D", 3), ("rgb_colors", 3), ("unnorm_rotations", 4),
                                             ("log_scales", 3), ("seg_colors", 3))}
    t1 = {k: v + 1 for k, v in t0.items()}
    outs = [params2cpu(t0, True), params2cpu(t1, False)]
    assert set(outs[1]) == {"means3D", "rgb_colors", "unnorm_rotations"}
    path = save_params(outs, "seq", "exp", root=str(tmp_path))
    z = load_params(path)
    assert z["means3D"].shape == (2, 5, 3) and z["log_scales"].shape == (5, 3)
    np.testing.assert_array_equal(z["means3D"][1], t1["means3D"].numpy())
    np.testing.assert_array_equal(z["seg_colors"], t0["seg_colors"].numpy())


# ------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform", "clusters", "plane"])
@pytest.mark.parametrize("k", [1, 3, 20, 32])
def test_knn_matches_bruteforce(kind, k):
    from dynamic3dgaussians_amd.knn import knn
    p = _cloud(3000, kind, seed=k)
    d, i = knn(torch.from_numpy(p).cuda(), k)
    od, oi = ON.knn(p, k)
    np.testing.assert_array_equal(d.cpu().numpy(), od)  # same double arithmetic, bit-exact
    if kind == "plane":
        # grid ties: the oracle's stable argsort also breaks ties by index
        np.testing.assert_array_equal(i.cpu().numpy(), oi)
    else:
        np.testing.assert_array_equal(i.cpu().numpy(), oi)


@pytest.mark.gpu
def test_knn_large_cloud_sampled_rows():
    """300k points (the bench scale): 256 sampled rows checked against a
    brute-force scan of the whole cloud."""
    from dynamic3dgaussians_amd.knn import knn
    N, k = 300000, 20
    p = _cloud(N, "clusters", seed=7)
    d, i = knn(torch.from_numpy(p).cuda(), k)
    d, i = d.cpu().numpy(), i.cpu().numpy()
    rows = np.random.default_rng(1).choice(N, 256, replace=False)
    P = p.astype(np.float64)
    for r in rows:
        dd = ((P - P[r]) ** 2).sum(-1)
        dd[r] = np.inf
        o = np.argsort(dd, kind="stable")[:k]
        np.testing.assert_array_equal(i[r], o)
        np.testing.assert_array_equal(d[r], dd[o])


@pytest.mark.gpu
def test_knn_edge_cases_and_dropins():
    from dynamic3dgaussians_amd import _lib
    from dynamic3dgaussians_amd.knn import distCUDA2, knn, o3d_knn
    # fewer points than k: tail is (+inf, -1)
    d, i = knn(torch.tensor([[0, 0, 0], [1, 0, 0], [3, 0, 0]], dtype=torch.float32, device="cuda"), 4)
    assert i.cpu().tolist()[0] == [1, 2, -1, -1] and np.isinf(d.cpu().numpy()[0, 2:]).all()
    # duplicates: the point itself is excluded by index, its twin kept at 0
    d, i = knn(torch.tensor([[1, 1, 1], [1, 1, 1], [2, 1, 1]], dtype=torch.float32, device="cuda"), 1)
    assert i.cpu().tolist() == [[1], [0], [0]] and d.cpu().tolist()[0] == [0.0]
    with pytest.raises(_lib.GsplatError):
        knn(torch.zeros(10, 3, device="cuda"), 33)
    # the reference's call shapes
    p = _cloud(2000, "uniform", seed=3)
    sq, idx = o3d_knn(p.astype(np.float64), 3)       # train.py:95
    od, oi = ON.knn(p, 3)
    assert sq.dtype == np.float64 and idx.dtype == np.int64
    np.testing.assert_array_equal(sq, od)
    means, nn = distCUDA2(torch.from_numpy(p).cuda())  # scene/gaussian_model.py:162
    assert means.dtype == torch.float32 and nn.dtype == torch.int32 and nn.shape == (2000, 3)
    np.testing.assert_allclose(means.cpu().numpy(), od.mean(1), rtol=1e-6)
    np.testing.assert_array_equal(nn.cpu().numpy(), oi)
