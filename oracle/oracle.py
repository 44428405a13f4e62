"""CPU oracle for the Gaussian rasterizer -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  It is never used by the product package
(dynamic3dgaussians_amd / diff_gaussian_rasterization).

It wraps oracle/build/libgs_oracle.so (gs_oracle.c, a plain-C restatement of
the reference CUDA rasterizer) and orchestrates the stages exactly like the
reference driver CudaRasterizer::Rasterizer::forward / backward
(DGR/cuda_rasterizer/rasterizer_impl.cu:198-346 and :350-467), exposing the
same positional interface as the reference's pybind module
(DGR/rasterize_points.cu:35-225) but on numpy arrays.

Parity status: "partially pinned" -- see gs_oracle.c header and DESIGN.md.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libgs_oracle.so")

COMPAT = {"reference": 0, "fixed": 1}
TILE = 16

_f = ctypes.POINTER(ctypes.c_float)
_i = ctypes.POINTER(ctypes.c_int)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_u64 = ctypes.POINTER(ctypes.c_uint64)
_u8 = ctypes.POINTER(ctypes.c_uint8)
_I, _F = ctypes.c_int, ctypes.c_float

_lib = None


def build():
    """Compile the oracle with its Makefile (gcc, strict IEEE)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "gs_oracle.c"))
        ):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.or_preprocess.argtypes = [_I, _I, _I, _f, _f, _F, _f, _f, _f, _f, _f, _f, _f, _f,
                                    _I, _I, _F, _F, _F, _F, _I,
                                    _i, _f, _f, _f, _f, _f, _u32, _u8]
        L.or_preprocess.restype = _I
        L.or_binning.argtypes = [_I, _f, _f, _i, _u32, _I, _I, _u32, _u64, _u32]
        L.or_binning.restype = ctypes.c_int64
        L.or_render_fwd.argtypes = [_I, _I, _u32, _u32, _f, _f, _f, _I, _f, _f, _f, _I,
                                    _f, _f, _f, _f, _u32]
        L.or_render_fwd.restype = None
        L.or_render_bwd.argtypes = [_I, _I, _u32, _u32, _f, _f, _f, _f, _f, _I, _f, _f, _u32,
                                    _f, _f, _f, _f, _I, _f, _f, _f, _f, _f, _f]
        L.or_render_bwd.restype = None
        L.or_set_pixel_order.argtypes = [_u32, ctypes.c_int64]
        L.or_set_pixel_order.restype = None
        L.or_preprocess_bwd.argtypes = [_I, _I, _I, _f, _i, _f, _u8, _f, _f, _F, _f, _f, _f,
                                        _I, _I, _F, _F, _F, _F, _f, _f, _f, _f, _f, _I,
                                        _f, _f, _f, _f, _f]
        L.or_preprocess_bwd.restype = None
        L.or_mark_visible.argtypes = [_I, _f, _f, _f, _u8]
        L.or_mark_visible.restype = None
        L.or_higher_msb.argtypes = [ctypes.c_uint32]
        L.or_higher_msb.restype = ctypes.c_uint32
        _lib = L
    return _lib


def _np(x, dtype=np.float32):
    """Tensor/array -> contiguous numpy array, or None for absent inputs."""
    if x is None:
        return None
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    x = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    if x.size == 0:
        return None
    return x


def _p(a, ct=_f):
    return None if a is None else a.ctypes.data_as(ct)


@dataclass
class OracleState:
    """Everything the reference keeps in geomBuffer / binningBuffer / imgBuffer."""
    P: int
    W: int
    H: int
    F: int
    radii: np.ndarray
    means2D: np.ndarray
    depths: np.ndarray
    cov3D: np.ndarray
    rgb: np.ndarray
    conic_opacity: np.ndarray
    tiles_touched: np.ndarray
    clamped: np.ndarray
    num_rendered: int = 0
    point_list: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    keys: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    ranges: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    n_contrib: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    trapped: int = 0


def higher_msb(n: int) -> int:
    return int(lib().or_higher_msb(n))


def mark_visible(means3D, viewmatrix, projmatrix):
    m = _np(means3D)
    P = 0 if m is None else m.shape[0]
    out = np.zeros(P, np.uint8)
    if P:
        lib().or_mark_visible(P, _p(m), _p(_np(viewmatrix)), _p(_np(projmatrix)), _p(out, _u8))
    return out.astype(bool)


def rasterize_gaussians(bg, means3D, colors, semantic_feature, opacity, scales, rotations,
                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, c_x, c_y,
                        tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered=False, debug=False, compat="reference"):
    """Positional mirror of RasterizeGaussiansCUDA (DGR/rasterize_points.cu:35-126).

    Returns (num_rendered, color[3,H,W], feature[F,H,W], depth[1,H,W], alpha[1,H,W],
    radii[P], state) -- `state` stands in for the three opaque byte buffers.
    """
    L_ = lib()
    cm = COMPAT[compat]
    means3D = _np(means3D)
    P = 0 if means3D is None else means3D.shape[0]
    H, W = int(image_height), int(image_width)
    sem = _np(semantic_feature)
    F = 0 if sem is None else int(np.prod(sem.shape[1:]))
    if sem is not None:
        sem = sem.reshape(P, F)
    out_color = np.zeros((3, H, W), np.float32)
    out_feat = np.zeros((F, H, W), np.float32)
    out_depth = np.zeros((1, H, W), np.float32)
    out_alpha = np.zeros((1, H, W), np.float32)
    radii = np.zeros(P, np.int32)
    st = OracleState(P, W, H, F, radii, np.zeros((P, 2), np.float32), np.zeros(P, np.float32),
                     np.zeros((P, 6), np.float32), np.zeros((P, 3), np.float32),
                     np.zeros((P, 4), np.float32), np.zeros(P, np.uint32),
                     np.zeros((P, 3), np.uint8))
    if P == 0:
        return 0, out_color, out_feat, out_depth, out_alpha, radii, st
    sh = _np(sh)
    M = 0 if sh is None else sh.shape[1]
    colors = _np(colors)
    cov_pre = _np(cov3D_precomp)
    view, proj, cam = _np(viewmatrix), _np(projmatrix), _np(campos)
    bgv = _np(bg)
    st.trapped = L_.or_preprocess(
        P, int(degree), M, _p(means3D), _p(_np(scales)), float(scale_modifier), _p(_np(rotations)),
        _p(_np(opacity)), _p(sh), _p(cov_pre), _p(colors), _p(view), _p(proj), _p(cam),
        W, H, float(c_x), float(c_y), float(tan_fovx), float(tan_fovy), int(bool(prefiltered)),
        _p(radii, _i), _p(st.means2D), _p(st.depths), _p(st.cov3D), _p(st.rgb),
        _p(st.conic_opacity), _p(st.tiles_touched, _u32), _p(st.clamped, _u8))
    if st.trapped:
        raise RuntimeError("Point is filtered although prefiltered is set.")
    L = int(st.tiles_touched.astype(np.uint64).sum())
    gx, gy = (W + TILE - 1) // TILE, (H + TILE - 1) // TILE
    st.point_list = np.zeros(max(L, 1), np.uint32)
    st.keys = np.zeros(max(L, 1), np.uint64)
    st.ranges = np.zeros(gx * gy * 2, np.uint32)
    L2 = L_.or_binning(P, _p(st.means2D), _p(st.depths), _p(radii, _i), _p(st.tiles_touched, _u32),
                       W, H, _p(st.point_list, _u32), _p(st.keys, _u64), _p(st.ranges, _u32))
    assert L2 == L
    st.point_list, st.keys = st.point_list[:L], st.keys[:L]
    st.num_rendered = L
    st.n_contrib = np.zeros(H * W, np.uint32)
    feat_colors = colors if colors is not None else st.rgb
    L_.or_render_fwd(W, H, _p(st.ranges, _u32), _p(st.point_list, _u32), _p(st.means2D),
                     _p(feat_colors), _p(sem), F, _p(st.depths), _p(st.conic_opacity), _p(bgv), cm,
                     _p(out_color), _p(out_feat), _p(out_depth), _p(out_alpha),
                     _p(st.n_contrib, _u32))
    return L, out_color, out_feat, out_depth, out_alpha, radii, st


def rasterize_gaussians_backward(bg, means3D, radii, colors, semantic_feature, scales, rotations,
                                 scale_modifier, cov3D_precomp, viewmatrix, projmatrix, c_x, c_y,
                                 tan_fovx, tan_fovy, dL_dout_color, dL_dout_feature,
                                 dL_dout_depth, dL_dout_alpha, sh, degree, campos, state, R,
                                 binning_unused, image_unused, alpha, debug=False,
                                 compat="reference", pixel_order=None):
    """Positional mirror of RasterizeGaussiansBackwardCUDA (DGR/rasterize_points.cu:128-225).

    Camera scalars are taken in C++ positional order (c_x, c_y, tan_fovx, tan_fovy),
    exactly as the reference binding receives them.  Returns
    (dL_dmeans2D, dL_dcolors, dL_dsemantic, dL_dopacity, dL_dmeans3D, dL_dcov3D,
     dL_dsh, dL_dscales, dL_drotations).

    `pixel_order` (optional, a permutation of the H*W pixel indices) changes
    the order in which the blend backward visits pixels, hence the fp32
    summation order of every per-Gaussian gradient sum (the reference sums
    with atomicAdd in arrival order): the spread it causes is the fp32
    envelope the GPU's differences are compared with.
    """
    L_ = lib()
    cm = COMPAT[compat]
    st: OracleState = state
    means3D = _np(means3D)
    P = 0 if means3D is None else means3D.shape[0]
    dLc = _np(dL_dout_color)
    H, W = dLc.shape[1], dLc.shape[2]
    sh = _np(sh)
    M = 0 if sh is None else sh.shape[1]
    F = st.F
    out = dict(
        dmean2D=np.zeros((P, 3), np.float32), dcolors=np.zeros((P, 3), np.float32),
        dsem=np.zeros((P, F), np.float32), dopacity=np.zeros((P, 1), np.float32),
        dmean3D=np.zeros((P, 3), np.float32), dcov3D=np.zeros((P, 6), np.float32),
        dsh=np.zeros((P, M, 3), np.float32), dscales=np.zeros((P, 3), np.float32),
        drot=np.zeros((P, 4), np.float32))
    if P == 0:
        return tuple(out.values())
    dconic = np.zeros((P, 4), np.float32)
    ddepth = np.zeros(P, np.float32)
    colors = _np(colors)
    sem = _np(semantic_feature)
    if sem is not None:
        sem = sem.reshape(P, F)
    dLf = _np(dL_dout_feature)
    if dLf is None:
        dLf = np.zeros((F, H, W), np.float32)
    feat_colors = colors if colors is not None else st.rgb
    radii_np = _np(radii, np.int32)
    order = None
    if pixel_order is not None:
        order = np.ascontiguousarray(pixel_order, np.uint32)
        assert order.size == H * W
        L_.or_set_pixel_order(_p(order, _u32), ctypes.c_int64(order.size))
    L_.or_render_bwd(W, H, _p(st.ranges, _u32), _p(st.point_list, _u32), _p(_np(bg)),
                     _p(st.means2D), _p(st.conic_opacity), _p(feat_colors), _p(sem), F,
                     _p(st.depths), _p(_np(alpha)), _p(st.n_contrib, _u32), _p(dLc), _p(dLf),
                     _p(_np(dL_dout_depth)), _p(_np(dL_dout_alpha)), cm, _p(out["dmean2D"]),
                     _p(dconic), _p(out["dopacity"]), _p(out["dcolors"]), _p(out["dsem"]),
                     _p(ddepth))
    if order is not None:
        L_.or_set_pixel_order(None, ctypes.c_int64(0))
    cov_pre = _np(cov3D_precomp)
    cov = cov_pre if cov_pre is not None else st.cov3D
    L_.or_preprocess_bwd(P, int(degree), M, _p(means3D), _p(radii_np, _i), _p(sh),
                         _p(st.clamped, _u8), _p(_np(scales)), _p(_np(rotations)),
                         float(scale_modifier), _p(cov), _p(_np(viewmatrix)), _p(_np(projmatrix)),
                         W, H, float(c_x), float(c_y), float(tan_fovx), float(tan_fovy),
                         _p(_np(campos)), _p(out["dmean2D"]), _p(dconic), _p(out["dcolors"]),
                         _p(ddepth), cm, _p(out["dmean3D"]), _p(out["dcov3D"]), _p(out["dsh"]),
                         _p(out["dscales"]), _p(out["drot"]))
    state.dconic, state.ddepth = dconic, ddepth
    return tuple(out.values())
