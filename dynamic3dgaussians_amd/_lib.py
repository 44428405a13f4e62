"""ctypes binding of libgsplat_hip.so (C ABI: include/gsplat_hip.h).

This is the only way the package reaches the GPU: there is no CPU or PyTorch
fallback.  If the HIP library is missing or cannot be loaded, every entry point
raises immediately with the reason.
"""
from __future__ import annotations

import ctypes
import os
import threading

from . import build as _build

_lock = threading.Lock()
_lib = None

c_void_p = ctypes.c_void_p
ABI_VERSION = 13  # include/gsplat_hip.h GS_ABI_VERSION
GS_FLAG_ACCUMULATE = 1  # include/gsplat_hip.h
GS_FLAG_ACTIVATE = 2  # include/gsplat_hip.h: raw opacity / scale / rotation parameters
GS_FLAG_SCRATCH_ZEROED = 4  # include/gsplat_hip.h: the backward's scratch was zeroed by the forward
c_int32, c_int64, c_float, c_size_t = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_size_t

GS_COMPAT = {"reference": 0, "fixed": 1}
SUPPORTED_F = (0, 4, 8, 16, 32, 36, 64)


class GsGaussians(ctypes.Structure):
    _fields_ = [("P", c_int32), ("D", c_int32), ("M", c_int32), ("F", c_int32),
                ("means3D", c_void_p), ("shs", c_void_p), ("colors_precomp", c_void_p),
                ("semantic_feature", c_void_p), ("opacities", c_void_p), ("scales", c_void_p),
                ("rotations", c_void_p), ("cov3D_precomp", c_void_p),
                ("scale_modifier", c_float), ("flags", ctypes.c_uint32),
                ("grad_mask", c_void_p), ("densify_accum", c_void_p), ("densify_denom", c_void_p),
                ("max_radius", c_void_p), ("feature_ready", c_void_p), ("walk_order", c_void_p),
                ("zero_fill", c_void_p), ("zero_fill_bytes", c_int64)]


class GsCamera(ctypes.Structure):
    _fields_ = [("viewmatrix", c_void_p), ("projmatrix", c_void_p), ("campos", c_void_p),
                ("background", c_void_p), ("c_x", c_float), ("c_y", c_float),
                ("tan_fovx", c_float), ("tan_fovy", c_float),
                ("image_width", c_int32), ("image_height", c_int32),
                ("tile_x0", c_int32), ("tile_y0", c_int32), ("tile_x1", c_int32), ("tile_y1", c_int32)]


class GsNeighborGraph(ctypes.Structure):
    """include/gs_neighbor.h gs_neighbor_graph."""
    _fields_ = [("N", c_int64), ("K", c_int32), ("_pad", c_int32), ("nbr", c_void_p),
                ("weight", c_void_p), ("dist", c_void_p), ("prev_offset", c_void_p),
                ("prev_inv_rot", c_void_p), ("rev_ptr", c_void_p), ("rev_pos", c_void_p)]


GS_ADAM_MAX_TENSORS = 16  # include/gs_optim.h


class GsAdamTensor(ctypes.Structure):
    """include/gs_optim.h gs_adam_tensor."""
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("numel", c_int64), ("step_size", c_float), ("bc2_sqrt", c_float)]


class GsAdamArgs(ctypes.Structure):
    """include/gs_optim.h gs_adam_args (GS_ADAM_MAX_TENSORS = 16)."""
    _fields_ = [("n_tensors", c_int32), ("_pad", c_int32), ("beta1", ctypes.c_double),
                ("beta2", ctypes.c_double), ("eps", ctypes.c_double), ("t", GsAdamTensor * GS_ADAM_MAX_TENSORS)]


class GsDensifyStats(ctypes.Structure):
    """include/gs_optim.h gs_densify_stats."""
    _fields_ = [("P", c_int64), ("radii", c_void_p), ("means2D_grad", c_void_p), ("max_radius", c_void_p),
                ("grad_accum", c_void_p), ("denom", c_void_p)]


class GsBatchHint(ctypes.Structure):
    """include/gsplat_hip.h gs_batch_hint (ABI 11): the previous plan's sort
    extents, written back by gs_forward_batch."""
    _fields_ = [("valid", c_int32), ("p1", c_int32), ("q1", c_int32), ("p2", c_int32),
                ("max_len", c_int64), ("total", c_int64)]


P_G = ctypes.POINTER(GsGaussians)
P_NG = ctypes.POINTER(GsNeighborGraph)
P_C = ctypes.POINTER(GsCamera)

# name -> (restype, argtypes); must match include/gsplat_hip.h
PROTOTYPES = {
    "gs_version": (ctypes.c_int, []),
    "gs_last_error": (ctypes.c_char_p, []),
    "gs_geom_buffer_bytes": (c_size_t, [c_int64]),
    "gs_binning_buffer_bytes": (c_size_t, [c_int64]),
    "gs_image_buffer_bytes": (c_size_t, [c_int32, c_int32]),
    "gs_backward_scratch_bytes": (c_size_t, [c_int64, c_int32]),
    "gs_forward_plan": (ctypes.c_int, [P_G, P_C, ctypes.c_int, ctypes.c_int, ctypes.c_int, c_void_p,
                                       c_void_p, c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64),
                                       c_void_p]),
    "gs_forward_render": (ctypes.c_int, [P_G, P_C, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                         c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p]),
    "gs_backward": (ctypes.c_int, [P_G, P_C, c_void_p, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                   c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_batch_geom_buffer_bytes": (c_size_t, [c_int64, c_int32]),
    "gs_batch_image_buffer_bytes": (c_size_t, [c_int32, c_int32, c_int32]),
    "gs_batch_binning_buffer_bytes": (c_size_t, [c_int32, ctypes.POINTER(c_int64)]),
    "gs_batch_backward_scratch_bytes": (c_size_t, [c_int64, c_int32, c_int32]),
    "gs_forward_plan_batch": (ctypes.c_int, [P_G, P_C, c_int32, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_int64),
                                             ctypes.POINTER(c_int64), c_void_p]),
    "gs_forward_render_batch": (ctypes.c_int, [P_G, P_C, c_int32, ctypes.c_int, ctypes.c_int, c_void_p,
                                               c_void_p, c_void_p, ctypes.POINTER(c_int64), c_void_p, c_void_p,
                                               c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_forward_batch": (ctypes.c_int, [P_G, P_C, c_int32, ctypes.c_int, ctypes.c_int, c_void_p, c_void_p,
                                        c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(GsBatchHint), c_void_p,
                                        ctypes.POINTER(c_int64), ctypes.POINTER(c_int64), ctypes.POINTER(c_int32),
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_backward_batch": (ctypes.c_int, [P_G, P_C, c_int32, c_void_p, ctypes.c_int, ctypes.c_int, c_void_p,
                                         c_void_p, c_void_p, ctypes.POINTER(c_int64), c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_mark_visible": (ctypes.c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_debug_export": (ctypes.c_int, [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                       c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_sort_scratch_bytes": (c_size_t, [c_int64]),
    "gs_sort_pairs": (ctypes.c_int, [c_int64, c_void_p, c_void_p, ctypes.c_int, c_void_p, c_void_p]),
    "gs_check_plan_header": (ctypes.c_int, [c_void_p, c_int64]),
    "gs_check_ranges": (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int64]),
    "gs_check_point_list": (ctypes.c_int, [c_void_p, c_int64, c_int64]),
    "gs_check_walk_order": (ctypes.c_int, [c_void_p, c_int64]),
    "gs_spatial_order_scratch_bytes": (c_size_t, [c_int64]),
    "gs_spatial_order": (ctypes.c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_test_wave_reduce": (ctypes.c_int, [ctypes.c_int, c_void_p, c_void_p, c_void_p]),
    "gs_timing_enable": (ctypes.c_int, [ctypes.c_int]),
    # include/gs_knn.h
    "gs_knn_workspace_bytes": (c_size_t, [c_int64]),
    "gs_knn": (ctypes.c_int, [c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    # include/gs_optim.h
    "gs_adam_step": (ctypes.c_int, [ctypes.POINTER(GsAdamArgs), ctypes.POINTER(GsDensifyStats), c_void_p]),
    # include/gs_neighbor.h
    "gs_neighbor_workspace_bytes": (c_size_t, [c_int64, c_int32, ctypes.c_int]),
    "gs_neighbor_loss_forward": (ctypes.c_int, [P_NG, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "gs_neighbor_loss_backward": (ctypes.c_int, [P_NG, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                 c_void_p, c_void_p]),
    "gs_neighbor_reverse_workspace_bytes": (c_size_t, [c_int64, c_int32]),
    "gs_neighbor_reverse": (ctypes.c_int, [c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_void_p]),
    "gs_timing_select": (ctypes.c_int, [ctypes.c_uint32]),
    "gs_timing_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int64),
                                      ctypes.c_int]),
}

STAGES = ["preprocess", "scan", "duplicate", "sort", "ranges", "render_fwd", "render_bwd",
          "preprocess_bwd"]


def timing_enable(on: bool = True, stages=None):
    """Enable/disable live stage timing; `stages` (names) restricts it."""
    L = load()
    mask = 0xFFFFFFFF if stages is None else sum(1 << STAGES.index(s) for s in stages)
    L.gs_timing_select(mask)
    L.gs_timing_enable(1 if on else 0)


def timing_read() -> dict:
    """{stage: (total_ms, launches)} since the last timing_enable()."""
    n = len(STAGES)
    ms = (ctypes.c_double * n)()
    cnt = (c_int64 * n)()
    check(load().gs_timing_read(ms, cnt, n), "timing read")
    return {s: (ms[i], cnt[i]) for i, s in enumerate(STAGES)}


class GsplatError(RuntimeError):
    pass


def lib_path() -> str:
    return _build.LIB


def load(auto_build: bool = True):
    """Load libgsplat_hip.so (building it first if stale and hipcc is present)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.LIB
        if auto_build:
            try:
                if _build.is_stale():
                    _build.build()
            except RuntimeError:
                if not os.path.exists(path):
                    raise
        if not os.path.exists(path):
            raise GsplatError(
                f"libgsplat_hip.so not found at {path}; build it with "
                "`python -m dynamic3dgaussians_amd.build` (requires ROCm hipcc). "
                "There is no CPU fallback.")
        L = ctypes.CDLL(path)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.gs_version() != ABI_VERSION:
            raise GsplatError(f"ABI version mismatch: library reports {L.gs_version()}")
        _lib = L
        return L


def check(code: int, what: str):
    if code != 0:
        msg = load().gs_last_error().decode(errors="replace")
        raise GsplatError(f"{what} failed (status {code}): {msg}")
