"""Neighbour losses: HIP kernels vs the reference's
formulas (oracle/neighbor.py: op-for-op PyTorch fp32 restatement of
train.py:253-273, pinned on the CPU by a float64 numpy restatement).

Scene: the reference's setup -- neighbours from the first timestep's
foreground points (train.py:316-326: k = 20, weight exp(-2000 d^2), dist
sqrt(d^2)), previous-timestep state from initialize_per_timestep
(train.py:294-306), then the current points / rotations moved a little."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import neighbor as ON


def make_state(N=2000, K=20, seed=0, spread=0.3, motion=0.01, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    init = (torch.rand(N, 3, generator=g) - 0.5) * spread
    sq, idx = ON.knn(init.numpy(), K)
    prev_pts = init + motion * torch.randn(N, 3, generator=g)
    prev_rot = torch.nn.functional.normalize(torch.randn(N, 4, generator=g), dim=1)
    prev_inv = prev_rot.clone()
    prev_inv[:, 1:] = -prev_inv[:, 1:]                      # train.py:301-302
    nbr = torch.from_numpy(idx)
    variables = {
        "neighbor_indices": nbr.long().contiguous(),
        "neighbor_weight": torch.from_numpy(np.exp(-2000 * sq)).float().contiguous(),
        "neighbor_dist": torch.from_numpy(np.sqrt(sq)).float().contiguous(),
        "prev_inv_rot_fg": prev_inv.contiguous(),
        "prev_offset": (prev_pts[nbr] - prev_pts[:, None]).contiguous(),  # train.py:304
    }
    pts = prev_pts + motion * torch.randn(N, 3, generator=g)
    rot = torch.nn.functional.normalize(prev_rot + 0.05 * torch.randn(N, 4, generator=g), dim=1)
    if device != "cpu":
        variables = {k: v.to(device) for k, v in variables.items()}
        pts, rot = pts.to(device), rot.to(device)
    return pts, rot, variables


# ------------------------------------------------------------------- CPU

def test_torch_restatement_matches_float64():
    pts, rot, v = make_state(N=500, K=8)
    t = ON.torch_reference(pts, rot, v)
    n = ON.numpy_losses(pts.numpy(), rot.numpy(), v["neighbor_indices"].numpy(), v["neighbor_weight"].numpy(),
                        v["neighbor_dist"].numpy(), v["prev_offset"].numpy(), v["prev_inv_rot_fg"].numpy())
    for a, b in zip(t, n):
        assert abs(a.item() - b) <= 1e-5 * abs(b)


def test_reverse_csr_oracle():
    nbr = np.array([[1, 2], [0, 2], [0, 1], [2, 2]])
    ptr, pair = ON.reverse_csr(nbr)
    assert ptr.tolist() == [0, 2, 4, 8, 8]
    assert pair.tolist() == [2, 4, 0, 5, 1, 3, 6, 7]


def test_knn_excludes_self():
    p = np.array([[0, 0, 0], [1, 0, 0], [3, 0, 0], [3.5, 0, 0]], np.float64)
    d, i = ON.knn(p, 2)
    assert i.tolist() == [[1, 2], [0, 2], [3, 1], [2, 1]]
    assert d[0].tolist() == [1.0, 9.0]


# ------------------------------------------------------------------- GPU

gpu = pytest.mark.gpu


def _rel(a, b):
    if b is None:  # the reference term does not reach this input
        return a.abs().max().item()
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@gpu
@pytest.mark.parametrize("N,K", [(3000, 20), (257, 1), (1000, 7)])
def test_neighbor_losses_match_reference(N, K):
    from dynamic3dgaussians_amd.neighbor import neighbor_losses
    pts, rot, v = make_state(N=N, K=K, seed=N + K, device="cuda")
    p1, r1 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
    p2, r2 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
    ours = neighbor_losses(p1, r1, v)
    ref = ON.torch_reference(p2, r2, v)
    for a, b in zip(ours, ref):
        assert abs(a.item() - b.item()) <= 2e-5 * abs(b.item()) + 1e-12
    wts = (0.4, 0.4, 0.2)  # cvpr_dyn.py:332 loss weights
    sum(w * l for w, l in zip(wts, ours)).backward()
    sum(w * l for w, l in zip(wts, ref)).backward()
    # fp32 reassociation only: the reference sums through autograd scatter-adds
    assert _rel(p1.grad, p2.grad) <= 1e-4
    assert _rel(r1.grad, r2.grad) <= 1e-4


@gpu
def test_neighbor_losses_each_term_and_determinism():
    """Each loss alone (the other upstream grads absent), and two backward runs
    bit-identical (no atomics)."""
    from dynamic3dgaussians_amd.neighbor import neighbor_losses
    pts, rot, v = make_state(N=2500, K=20, seed=3, device="cuda")
    for term in range(3):
        p1, r1 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
        p2, r2 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
        neighbor_losses(p1, r1, v)[term].backward()
        ON.torch_reference(p2, r2, v)[term].backward()
        assert _rel(p1.grad, p2.grad) <= 1e-4, term
        assert _rel(r1.grad, r2.grad) <= 1e-4, term
    g = []
    for _ in range(2):
        p1, r1 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
        sum(neighbor_losses(p1, r1, v)).backward()
        g.append((p1.grad, r1.grad))
    assert torch.equal(g[0][0], g[1][0]) and torch.equal(g[0][1], g[1][1])


@gpu
def test_neighbor_losses_through_caller_indexing():
    """The reference calls the block with fg_pts = means3D[is_fg] and
    fg_rot = normalize(unnorm_rotations)[is_fg] (train.py:254-257); gradients
    reach the parameters through the caller's own indexing / normalize."""
    from dynamic3dgaussians_amd.neighbor import neighbor_losses
    P = 4000
    g = torch.Generator().manual_seed(9)
    is_fg = torch.rand(P, generator=g) > 0.4
    N = int(is_fg.sum())
    pts, rot, v = make_state(N=N, K=20, seed=4, device="cuda")
    means = torch.randn(P, 3, generator=g).cuda()
    means[is_fg.cuda()] = pts
    unnorm = torch.randn(P, 4, generator=g).cuda()
    unnorm[is_fg.cuda()] = rot * 1.7
    grads = []
    for fn in (neighbor_losses, ON.torch_reference):
        m, u = means.clone().requires_grad_(True), unnorm.clone().requires_grad_(True)
        fg = is_fg.cuda()
        out = fn(m[fg], torch.nn.functional.normalize(u)[fg], v)
        sum(out).backward()
        grads.append((m.grad, u.grad))
    assert _rel(grads[0][0], grads[1][0]) <= 1e-4
    assert _rel(grads[0][1], grads[1][1]) <= 1e-4
    assert grads[0][0][~is_fg.cuda()].abs().max().item() == 0


@gpu
@pytest.mark.parametrize("N,K", [(1, 1), (64, 3), (5000, 20)])
def test_reverse_csr_bitexact(N, K):
    from dynamic3dgaussians_amd.neighbor import reverse_csr
    g = torch.Generator().manual_seed(N)
    nbr = torch.randint(0, N, (N, K), generator=g)
    nbr[: N // 3, 0] = 0  # a heavy row
    ptr, pair, pos = reverse_csr(nbr.cuda())
    optr, opair = ON.reverse_csr(nbr.numpy())
    np.testing.assert_array_equal(ptr.cpu().numpy(), optr)
    np.testing.assert_array_equal(pair.cpu().numpy(), opair)
    opos = np.empty_like(opair)
    opos[opair] = np.arange(opair.size, dtype=np.int32)
    np.testing.assert_array_equal(pos.cpu().numpy(), opos)


@gpu
def test_neighbor_edge_cases():
    from dynamic3dgaussians_amd import _lib
    from dynamic3dgaussians_amd.neighbor import neighbor_losses, reverse_csr
    # out-of-range neighbour ids are an error, not a fault
    with pytest.raises(_lib.GsplatError):
        reverse_csr(torch.tensor([[1], [2]], device="cuda"))
    # empty: the reference's mean over nothing is NaN
    pts, rot, v = make_state(N=40, K=4, device="cuda")
    e = {k: t[:0] for k, t in v.items()}
    out = neighbor_losses(pts[:0], rot[:0], e)
    assert all(torch.isnan(o).item() for o in out)
    # CPU tensors raise (no CPU path)
    with pytest.raises(_lib.GsplatError):
        neighbor_losses(pts.cpu(), rot.cpu(), {k: t.cpu() for k, t in v.items()})


@gpu
def test_reverse_csr_cache_follows_reassigned_graph():
    """The reference reassigns variables['neighbor_indices'] with a fresh
    tensor (train.py:316-326); a same-shape graph that reuses the freed
    address of the previous one must not pick up the cached reverse CSR."""
    from dynamic3dgaussians_amd.neighbor import neighbor_losses
    N, K = 1000, 7
    pts, rot, v = make_state(N=N, K=K, seed=3, device="cuda")
    p, r = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
    sum(neighbor_losses(p, r, v)).backward()
    # a different graph of the same shape, stored where the old one lived
    perm = torch.randperm(N, generator=torch.Generator().manual_seed(9)).cuda()
    new_nbr = v["neighbor_indices"][perm].clone()
    old_ptr = v["neighbor_indices"].data_ptr()
    v["neighbor_indices"].copy_(new_nbr)  # in place: same address, bumped _version
    assert v["neighbor_indices"].data_ptr() == old_ptr
    for graph in ("in_place", "reassigned"):
        if graph == "reassigned":
            v["neighbor_indices"] = v["neighbor_indices"].clone()  # a new object
        p1, r1 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
        p2, r2 = pts.clone().requires_grad_(True), rot.clone().requires_grad_(True)
        sum(neighbor_losses(p1, r1, v)).backward()
        sum(ON.torch_reference(p2, r2, v)).backward()
        assert _rel(p1.grad, p2.grad) <= 1e-4, graph
        assert _rel(r1.grad, r2.grad) <= 1e-4, graph
