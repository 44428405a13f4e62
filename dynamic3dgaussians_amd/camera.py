"""Camera construction for the rasterizer boundary.

Restates Dynamic3DGaussians' helpers.setup_camera (helpers.py:68-95): OpenCV
intrinsics K and a world-to-camera matrix become the raster settings the
rasterizer consumes (column-major view / full-projection matrices, tan(fov/2),
principal point).  The reference module imports open3d at module level, so it
is restated rather than imported.  Also provides the synthetic camera rig the
benchmark uses: cameras on a ring/dome looking at the origin.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


@dataclass
class CameraParams:
    """Host-side camera description (numpy, float32)."""
    W: int
    H: int
    viewmatrix: np.ndarray  # [4,4] stored so that .ravel() is column-major w2c
    projmatrix: np.ndarray  # [4,4] stored so that .ravel() is column-major P*w2c
    campos: np.ndarray      # [3]
    c_x: float
    c_y: float
    tanfovx: float
    tanfovy: float


def setup_camera(w, h, k, w2c, near=0.01, far=100.0) -> CameraParams:
    """helpers.py:68-95 restated in numpy (float32 results, same layout)."""
    k = np.asarray(k, dtype=np.float64)
    fx, fy, cx, cy = k[0][0], k[1][1], k[0][2], k[1][2]
    w2c = np.asarray(w2c, dtype=np.float32)
    cam_center = np.linalg.inv(w2c.astype(np.float64))[:3, 3].astype(np.float32)
    view = w2c.T.copy()  # w2c.unsqueeze(0).transpose(1, 2)
    opengl_proj = np.array([[2 * fx / w, 0.0, -(w - 2 * cx) / w, 0.0],
                            [0.0, 2 * fy / h, -(h - 2 * cy) / h, 0.0],
                            [0.0, 0.0, far / (far - near), -(far * near) / (far - near)],
                            [0.0, 0.0, 1.0, 0.0]], dtype=np.float32).T
    full_proj = (view @ opengl_proj).astype(np.float32)  # w2c^T.bmm(proj^T)
    return CameraParams(W=int(w), H=int(h), viewmatrix=view, projmatrix=full_proj,
                        campos=cam_center, c_x=float(cx), c_y=float(cy),
                        tanfovx=float(w / (2 * fx)), tanfovy=float(h / (2 * fy)))


def look_at_w2c(eye, target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)) -> np.ndarray:
    """OpenCV-convention world-to-camera (x right, y down, z forward)."""
    eye = np.asarray(eye, np.float64)
    fwd = np.asarray(target, np.float64) - eye
    fwd /= np.linalg.norm(fwd)
    right = np.cross(fwd, np.asarray(up, np.float64))
    if np.linalg.norm(right) < 1e-8:
        right = np.cross(fwd, np.array([1.0, 0.0, 0.0]))
    right /= np.linalg.norm(right)
    down = np.cross(fwd, right)
    R = np.stack([right, down, fwd])  # rows: camera axes in world coords
    w2c = np.eye(4)
    w2c[:3, :3] = R
    w2c[:3, 3] = -R @ eye
    return w2c.astype(np.float32)


def intrinsics(W, H, fov_deg=60.0, cx=None, cy=None):
    """fx = fy = W / (2 tan(fov/2)); principal point defaults to the centre."""
    f = W / (2.0 * math.tan(math.radians(fov_deg) / 2.0))
    return np.array([[f, 0, W / 2.0 if cx is None else cx],
                     [0, f, H / 2.0 if cy is None else cy],
                     [0, 0, 1]], dtype=np.float64)


def camera_rig(n_cams, W, H, radius=2.5, fov_deg=60.0, seed=0):
    """n_cams cameras on a dome of `radius` looking at the origin (a Panoptic-like
    rig of 27 cameras by default in the bench)."""
    rng = np.random.default_rng(seed)
    cams = []
    golden = math.pi * (3.0 - math.sqrt(5.0))
    for i in range(n_cams):
        # Fibonacci points on the upper part of the sphere (elevation 10..60 deg)
        t = (i + 0.5) / max(n_cams, 1)
        elev = math.radians(10.0 + 50.0 * t)
        azim = golden * i + rng.uniform(-0.05, 0.05)
        eye = radius * np.array([math.cos(elev) * math.cos(azim), -math.sin(elev),
                                 math.cos(elev) * math.sin(azim)])
        cams.append(setup_camera(W, H, intrinsics(W, H, fov_deg), look_at_w2c(eye)))
    return cams
