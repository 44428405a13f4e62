"""Oracle for the neighbour losses -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker of
dynamic3dgaussians_amd/neighbor.py (the HIP kernels of csrc/gs_neighbor.hip).

* `torch_reference` restates the reference's loss block op for op in plain
  PyTorch fp32 (train.py:253-273 with helpers.py:117-133 and
  external.py:61-78); autograd gives the reference's gradients.  Run on the
  same device as the kernel it checks.
* `numpy_losses` is the float64 restatement of the same formulas, used on the
  CPU to pin the torch restatement.
* `reverse_csr` is the integer reverse adjacency (numpy stable argsort), the
  bit-exact checker of gs_neighbor_reverse.
* `knn` is brute-force k-nearest neighbours in float64 (the reference uses
  Open3D's KDTreeFlann.search_knn_vector_3d, helpers.py:135-146; Open3D is not
  in this image, so the reference itself cannot be run here -- parity of the
  neighbour losses is pinned to the reference's formulas, not to its outputs).
"""
from __future__ import annotations

import numpy as np
import torch


def _quat_mult(q1, q2):  # helpers.py:124-132
    w1, x1, y1, z1 = q1.T
    w2, x2, y2, z2 = q2.T
    w = w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2
    x = w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2
    y = w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2
    z = w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2
    return torch.stack([w, x, y, z]).T


def _build_rotation(q):  # external.py:61-78
    norm = torch.sqrt(q[:, 0] * q[:, 0] + q[:, 1] * q[:, 1] + q[:, 2] * q[:, 2] + q[:, 3] * q[:, 3])
    q = q / norm[:, None]
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    rows = [1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
            2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
            2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)]
    return torch.stack(rows, 1).reshape(-1, 3, 3)


def _wl2_v1(x, y, w):  # helpers.py:117-118
    return torch.sqrt(((x - y) ** 2) * w + 1e-20).mean()


def _wl2_v2(x, y, w):  # helpers.py:121-122
    return torch.sqrt(((x - y) ** 2).sum(-1) * w + 1e-20).mean()


def torch_reference(fg_pts, fg_rot, variables):
    """train.py:259-273 -> (rigid, rot, iso)."""
    nbr = variables["neighbor_indices"]
    w = variables["neighbor_weight"]
    rel_rot = _quat_mult(fg_rot, variables["prev_inv_rot_fg"])
    rot = _build_rotation(rel_rot)
    neighbor_pts = fg_pts[nbr]
    curr_offset = neighbor_pts - fg_pts[:, None]
    curr_offset_in_prev_coord = (rot.transpose(2, 1)[:, None] @ curr_offset[:, :, :, None]).squeeze(-1)
    rigid = _wl2_v2(curr_offset_in_prev_coord, variables["prev_offset"], w)
    rot_l = _wl2_v2(rel_rot[nbr], rel_rot[:, None], w)
    curr_offset_mag = torch.sqrt((curr_offset ** 2).sum(-1) + 1e-20)
    iso = _wl2_v1(curr_offset_mag, variables["neighbor_dist"], w)
    return rigid, rot_l, iso


def numpy_losses(fg_pts, fg_rot, nbr, w, dist, prev_offset, prev_inv_rot):
    """float64 restatement of the same three means (numpy arrays in)."""
    p = np.asarray(fg_pts, np.float64)
    a = np.asarray(fg_rot, np.float64)
    b = np.asarray(prev_inv_rot, np.float64)
    w = np.asarray(w, np.float64)
    q = np.stack([a[:, 0] * b[:, 0] - a[:, 1] * b[:, 1] - a[:, 2] * b[:, 2] - a[:, 3] * b[:, 3],
                  a[:, 0] * b[:, 1] + a[:, 1] * b[:, 0] + a[:, 2] * b[:, 3] - a[:, 3] * b[:, 2],
                  a[:, 0] * b[:, 2] - a[:, 1] * b[:, 3] + a[:, 2] * b[:, 0] + a[:, 3] * b[:, 1],
                  a[:, 0] * b[:, 3] + a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1] + a[:, 3] * b[:, 0]], 1)
    qn = q / np.linalg.norm(q, axis=1, keepdims=True)
    r, x, y, z = qn.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                  2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                  2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    off = p[nbr] - p[:, None]
    c = np.einsum("iab,ika->ikb", R, off)
    rigid = np.sqrt(((c - prev_offset) ** 2).sum(-1) * w + 1e-20).mean()
    rot = np.sqrt(((q[nbr] - q[:, None]) ** 2).sum(-1) * w + 1e-20).mean()
    mag = np.sqrt((off ** 2).sum(-1) + 1e-20)
    iso = np.sqrt(((mag - dist) ** 2) * w + 1e-20).mean()
    return rigid, rot, iso


def reverse_csr(nbr):
    """(rev_ptr [N+1], rev_pair [N*K]) int32 -- pairs naming each Gaussian,
    ascending pair index."""
    nbr = np.asarray(nbr, np.int64)
    N = nbr.shape[0]
    flat = nbr.reshape(-1)
    order = np.argsort(flat, kind="stable").astype(np.int32)
    counts = np.bincount(flat, minlength=N)
    rev_ptr = np.zeros(N + 1, np.int32)
    rev_ptr[1:] = np.cumsum(counts)
    return rev_ptr, order


def knn(pts, k):
    """Brute-force k nearest neighbours excluding the point itself (the
    reference's o3d_knn drops the first hit, helpers.py:135-146): returns
    (sq_dists [N, k] float64, indices [N, k] int64), ties by index."""
    p = np.asarray(pts, np.float64)
    d2 = ((p[:, None, :] - p[None, :, :]) ** 2).sum(-1)
    np.fill_diagonal(d2, np.inf)
    idx = np.argsort(d2, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(d2, idx, 1), idx.astype(np.int64)
