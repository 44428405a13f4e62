"""Exact k-nearest neighbours on the HIP kernels of csrc/gs_knn.hip
(C ABI include/gs_knn.h).

Drop-ins for the reference's neighbour searches:

* `o3d_knn(pts, num_knn)` -- helpers.py:135-146 (Open3D KDTreeFlann, k + 1
  hits with the point itself dropped): numpy (sq_dists float64 [N, k],
  indices int64 [N, k]); used for the initial scales (train.py:95) and the
  neighbour graph (train.py:316-326).
* `distCUDA2(points)` -- simple_knn._C.distCUDA2
  (submodules_fsgs/simple-knn/spatial.cu:14-27): (mean squared distance of
  the 3 nearest, fp32 [P]; their indices, int32 [P, 3]) on the device.
* `knn(points, k)` -- the device form: (sq_dist float64, index int64).

Exact search (no approximation), distances in double from the fp32
coordinates, ties to the lower index.  Differences from the reference,
documented: coordinates are taken as fp32 (the reference's foreground points
are fp32 tensors; float64 point clouds are rounded once); with exactly
duplicated points Open3D may drop the duplicate instead of the point itself,
this excludes the point itself by index.  No CPU path.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def knn(points: torch.Tensor, k: int):
    """points [N, 3] fp32 device -> (sq_dist [N, k] float64, index [N, k]
    int64); rows with fewer than k other points end in (+inf, -1)."""
    if not isinstance(points, torch.Tensor) or not points.is_cuda:
        raise _lib.GsplatError("knn needs a device tensor (there is no CPU path)")
    if points.dim() != 2 or points.size(1) != 3:
        raise ValueError(f"points must be [N, 3] (got {tuple(points.shape)})")
    pts = points.detach().to(torch.float32).contiguous()
    N = pts.size(0)
    dev = pts.device
    sq = torch.empty(N, k, dtype=torch.float64, device=dev)
    idx = torch.empty(N, k, dtype=torch.int64, device=dev)
    if N == 0:
        return sq, idx
    L = _lib.load()
    ws = torch.empty(L.gs_knn_workspace_bytes(N), dtype=torch.uint8, device=dev)
    _lib.check(L.gs_knn(N, int(k), pts.data_ptr(), sq.data_ptr(), idx.data_ptr(), ws.data_ptr(),
                        torch.cuda.current_stream(dev).cuda_stream), "knn")
    return sq, idx


def o3d_knn(pts, num_knn: int, device="cuda"):
    """helpers.py:135-146 on the GPU: numpy (sq_dists, indices)."""
    t = pts if isinstance(pts, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(pts))
    sq, idx = knn(t.to(device=device, dtype=torch.float32), num_knn)
    return sq.cpu().numpy(), idx.cpu().numpy()


def distCUDA2(points: torch.Tensor):
    """simple_knn._C.distCUDA2: (mean of the 3 nearest squared distances
    [P] fp32, their indices [P, 3] int32)."""
    sq, idx = knn(points, 3)
    d = sq.to(torch.float32)
    means = (d[:, 0] + d[:, 1] + d[:, 2]) / 3.0
    return means, idx.to(torch.int32)
