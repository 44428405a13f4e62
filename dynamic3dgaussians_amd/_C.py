"""Positional mirror of the reference's pybind module `diff_gaussian_rasterization._C`.

Reference: DGR/ext.cpp:15-19 and DGR/rasterize_points.cu:35-246 (DGR =
submodules_fsgs/diff-gaussian-rasterization-confidence).  The three functions
keep the reference's exact positional signatures and return tuples, so the
reference's own autograd wrapper could call them unchanged; they allocate
outputs with torch (caching allocator) and hand raw device pointers to the
HIP C ABI (libgsplat_hip.so).  There is no CPU fallback: non-device inputs or
a missing library raise.

Superset behaviour (documented in DESIGN.md "Boundary"):
  * semantic_feature may be None/empty (F = 0), [P, F] or [P, 1, F]; any F is
    accepted and zero-padded to the next compiled width (0, 4, 8, 16, 32, 36, 64).
  * keyword-only `compat` selects "reference" (as-shipped numerics, default)
    or "fixed" numerics; see DESIGN.md "Quirks".
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import warnings

import torch

from . import _lib
from ._lib import GsCamera, GsGaussians, check

_default_compat = "reference"

# Native fast path (csrc/gs_torch_binding.cpp, lib/_gs_native.so): the same
# argument handling in C++ over the same C ABI, ~0.2 ms less host time per
# camera than the ctypes code below, which stays the documented binding (and
# serves P == 0, CPU-tensor errors, build variants and GS_NATIVE_BINDING=0).
_native = None
_native_tried = False


def _native_mod():
    global _native, _native_tried
    if _native_tried:
        return _native
    _native_tried = True
    if os.environ.get("GS_NATIVE_BINDING", "1") == "0" or _lib._build.VARIANT:
        return None  # variants: the extension is linked against the product library
    path = os.path.join(os.path.dirname(_lib.lib_path()), "_gs_native.so")
    if not os.path.exists(path):
        return None
    _lib.load()
    if _lib._build.native_is_stale():
        # older than its source, a public header or libgsplat_hip.so: its
        # argument handling may not match the library -- serve the calls
        # through the ctypes binding instead (same kernels, more host time)
        warnings.warn("lib/_gs_native.so is stale (rebuild with `python -m dynamic3dgaussians_amd.build`); "
                      "using the ctypes binding", RuntimeWarning)
        return None
    spec = importlib.util.spec_from_file_location("_gs_native", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    if mod.abi_version() != _lib.ABI_VERSION:
        raise _lib.GsplatError(f"_gs_native.so was built for ABI {mod.abi_version()}, the library is "
                               f"{_lib.ABI_VERSION}; rebuild with `python -m dynamic3dgaussians_amd.build`")
    _native = mod
    return _native


def native_loaded() -> bool:
    """Whether the C++ fast path serves the calls (tests / diagnostics)."""
    return _native_mod() is not None


def _opt(t):
    return t if isinstance(t, torch.Tensor) else None


def set_default_compat(mode: str) -> None:
    """Process-wide default numerics mode ("reference" or "fixed")."""
    global _default_compat
    if mode not in _lib.GS_COMPAT:
        raise ValueError(f"compat must be one of {list(_lib.GS_COMPAT)}, got {mode!r}")
    _default_compat = mode


def get_default_compat() -> str:
    return _default_compat


def _present(t) -> bool:
    return t is not None and isinstance(t, torch.Tensor) and t.numel() > 0


def _dev(t: torch.Tensor, device, name: str) -> torch.Tensor:
    if t.device != device:
        raise _lib.GsplatError(f"{name} is on {t.device}, expected {device} (HIP device tensors only)")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _ptr(t) -> int | None:
    return t.data_ptr() if t is not None else None


def _feature_width(F: int) -> int:
    for k in _lib.SUPPORTED_F:
        if k >= F:
            return k
    raise _lib.GsplatError(f"semantic feature width {F} exceeds the largest compiled width "
                           f"{_lib.SUPPORTED_F[-1]}")


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _compat_code(compat) -> int:
    mode = _default_compat if compat is None else compat
    if mode not in _lib.GS_COMPAT:
        raise ValueError(f"compat must be one of {list(_lib.GS_COMPAT)}, got {mode!r}")
    return _lib.GS_COMPAT[mode]


class _Inputs:
    """Device-resident, contiguous views of the per-Gaussian inputs."""

    def __init__(self, means3D, colors, semantic_feature, opacity, scales, rotations,
                 scale_modifier, cov3D_precomp, sh, degree):
        if means3D.ndimension() != 2 or means3D.size(1) != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")  # rasterize_points.cu:60-62
        dev = means3D.device
        if dev.type != "cuda":
            raise _lib.GsplatError("the HIP rasterizer needs device tensors (means3D is on the CPU)")
        self.device = dev
        self.P = P = means3D.size(0)
        self.means3D = _dev(means3D, dev, "means3D")
        self.colors = _dev(colors, dev, "colors_precomp") if _present(colors) else None
        self.opacity = _dev(opacity, dev, "opacities") if _present(opacity) else None
        self.scales = _dev(scales, dev, "scales") if _present(scales) else None
        self.rotations = _dev(rotations, dev, "rotations") if _present(rotations) else None
        self.cov3D = _dev(cov3D_precomp, dev, "cov3D_precomp") if _present(cov3D_precomp) else None
        self.sh = _dev(sh, dev, "sh") if _present(sh) else None
        self.M = self.sh.size(1) if self.sh is not None else 0
        self.D = int(degree)
        self.scale_modifier = float(scale_modifier)
        if _present(semantic_feature):
            sem = _dev(semantic_feature, dev, "semantic_feature").reshape(P, -1)
            self.F_user = sem.size(1)
            self.F = _feature_width(self.F_user)
            if self.F != self.F_user:
                sem = torch.nn.functional.pad(sem, (0, self.F - self.F_user))
            self.sem = sem.contiguous()
        else:
            self.F_user, self.F, self.sem = 0, 0, None

    def struct(self, flags: int = 0) -> GsGaussians:
        return GsGaussians(P=self.P, D=self.D, M=self.M, F=self.F,
                           means3D=_ptr(self.means3D), shs=_ptr(self.sh),
                           colors_precomp=_ptr(self.colors), semantic_feature=_ptr(self.sem),
                           opacities=_ptr(self.opacity), scales=_ptr(self.scales),
                           rotations=_ptr(self.rotations), cov3D_precomp=_ptr(self.cov3D),
                           scale_modifier=self.scale_modifier, flags=flags, grad_mask=None,
                           densify_accum=None, densify_denom=None, max_radius=None)


def _camera(dev, background, viewmatrix, projmatrix, campos, c_x, c_y, tan_fovx, tan_fovy, W, H):
    keep = [_dev(background, dev, "bg").reshape(-1), _dev(viewmatrix, dev, "viewmatrix").reshape(-1),
            _dev(projmatrix, dev, "projmatrix").reshape(-1), _dev(campos, dev, "campos").reshape(-1)]
    cam = GsCamera(viewmatrix=_ptr(keep[1]), projmatrix=_ptr(keep[2]), campos=_ptr(keep[3]),
                   background=_ptr(keep[0]), c_x=float(c_x), c_y=float(c_y),
                   tan_fovx=float(tan_fovx), tan_fovy=float(tan_fovy),
                   image_width=int(W), image_height=int(H))
    return cam, keep


def rasterize_gaussians(background, means3D, colors, semantic_feature, opacity, scales, rotations,
                        scale_modifier, cov3D_precomp, viewmatrix, projmatrix, c_x, c_y, tan_fovx,
                        tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, debug,
                        *, compat=None):
    """RasterizeGaussiansCUDA (DGR/rasterize_points.cu:35-126).

    Returns (num_rendered, color[3,H,W], feature_map[F,H,W], depth[1,H,W],
    alpha[1,H,W], radii[P] int32, geomBuffer, binningBuffer, imgBuffer).
    """
    L_ = _lib.load()
    cm = _compat_code(compat)
    nat = _native_mod()
    if nat is not None and means3D.is_cuda and means3D.dim() == 2 and means3D.size(0) > 0:
        try:
            return nat.forward(background, means3D, _opt(colors), _opt(semantic_feature), _opt(opacity),
                               _opt(scales), _opt(rotations), float(scale_modifier), _opt(cov3D_precomp),
                               viewmatrix, projmatrix, float(c_x), float(c_y), float(tan_fovx),
                               float(tan_fovy), int(image_height), int(image_width), _opt(sh), int(degree),
                               campos, bool(prefiltered), bool(debug), cm,
                               torch.cuda.current_stream(means3D.device).cuda_stream)
        except RuntimeError as ex:
            raise _lib.GsplatError(str(ex)) from None
    inp = _Inputs(means3D, colors, semantic_feature, opacity, scales, rotations, scale_modifier,
                  cov3D_precomp, sh, degree)
    dev, P = inp.device, inp.P
    H, W = int(image_height), int(image_width)
    f32 = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    if P == 0:
        return (0, torch.zeros(3, H, W, **f32), torch.zeros(inp.F_user, H, W, **f32),
                torch.zeros(1, H, W, **f32), torch.zeros(1, H, W, **f32),
                torch.zeros(0, dtype=torch.int32, device=dev), torch.empty(0, **u8),
                torch.empty(0, **u8), torch.empty(0, **u8))
    cam, keep = _camera(dev, background, viewmatrix, projmatrix, campos, c_x, c_y, tan_fovx,
                        tan_fovy, W, H)
    g = inp.struct()
    out_color = torch.empty(3, H, W, **f32)
    out_feature = torch.empty(inp.F, H, W, **f32)
    out_depth = torch.empty(1, H, W, **f32)
    # Q1: the reference never writes out_alpha (it stays 0; the kernel stores
    # those zeros); "fixed" writes 1 - T.
    out_alpha = torch.empty(1, H, W, **f32)
    radii = torch.empty(P, dtype=torch.int32, device=dev)
    geom = torch.empty(L_.gs_geom_buffer_bytes(P), **u8)
    img = torch.empty(L_.gs_image_buffer_bytes(W, H), **u8)
    stream = _stream(dev)
    L = ctypes.c_int64(0)
    NI = ctypes.c_int64(0)
    check(L_.gs_forward_plan(ctypes.byref(g), ctypes.byref(cam), int(bool(prefiltered)),
                             int(bool(debug)), cm, geom.data_ptr(), img.data_ptr(), radii.data_ptr(),
                             ctypes.byref(L), ctypes.byref(NI),
                             stream), "rasterize_gaussians (preprocess)")
    # num_rendered is the reference's count (returned, like the reference);
    # the binned tile lists hold num_instances <= num_rendered entries
    num_rendered = int(L.value)
    num_instances = int(NI.value)
    binning = torch.empty(L_.gs_binning_buffer_bytes(num_instances), **u8)
    check(L_.gs_forward_render(ctypes.byref(g), ctypes.byref(cam), int(bool(debug)), cm,
                               geom.data_ptr(), binning.data_ptr(), img.data_ptr(), num_instances,
                               radii.data_ptr(), out_color.data_ptr(),
                               out_feature.data_ptr() if inp.F else None, out_depth.data_ptr(),
                               out_alpha.data_ptr(), stream), "rasterize_gaussians (render)")
    del keep
    feature_map = out_feature[:inp.F_user] if inp.F_user != inp.F else out_feature
    return (num_rendered, out_color, feature_map, out_depth, out_alpha, radii, geom, binning, img)


_BUFFER_ORDER = ("dmeans2D", "dcolors", "dsem", "dopacity", "dmeans3D", "dcov3D", "dsh", "dscales", "drot")


def spatial_order(means3D: torch.Tensor) -> torch.Tensor:
    """gs_spatial_order: the ids 0..P-1 in 3-D Morton order of the means
    (int32 [P] on the means' device) -- a walk order for the binning passes
    (gs_gaussians.walk_order) that keeps each binning workgroup's slice of
    the Gaussians compact on the screen."""
    if not (means3D.is_cuda and means3D.dtype == torch.float32 and means3D.dim() == 2 and means3D.size(1) == 3):
        raise RuntimeError("spatial_order: means3D must be an fp32 [P, 3] device tensor")
    L_ = _lib.load()
    m = means3D.detach().contiguous()
    P = m.size(0)
    order = torch.empty(P, dtype=torch.int32, device=m.device)
    scratch = torch.empty(max(1, L_.gs_spatial_order_scratch_bytes(P)), dtype=torch.uint8, device=m.device)
    check(L_.gs_spatial_order(P, m.data_ptr(), order.data_ptr(), scratch.data_ptr(), _stream(m.device)),
          "spatial order")
    return order


_NO_DEST = torch.empty(0)  # backward_batch's `out` entry: allocate this gradient


def _buffer_shapes(P, F, M):
    return dict(dmeans2D=(P, 3), dcolors=(P, 3), dsem=(P, F), dopacity=(P, 1), dmeans3D=(P, 3),
                dcov3D=(P, 6), dsh=(P, M, 3), dscales=(P, 3), drot=(P, 4))


def backward_buffers(P, F, M, device, flat=False):
    """Uninitialised gradient outputs of rasterize_gaussians_backward (F = the
    compiled feature width, M = SH coefficients per Gaussian).  With
    `flat=True` they are contiguous views into one buffer (each starting on a
    256-byte boundary) and (views, buffer, offsets) is returned, so that sums
    of whole gradient sets take one elementwise launch."""
    shapes = _buffer_shapes(P, F, M)
    if not flat:
        return {k: torch.empty(*shape, dtype=torch.float32, device=device) for k, shape in shapes.items()}
    offs, o = {}, 0
    for k, shape in shapes.items():
        n = 1
        for d in shape:
            n *= d
        offs[k] = (o, n, shape)
        o += (n + 63) // 64 * 64
    buf = torch.empty(max(o, 1), dtype=torch.float32, device=device)
    return carve_buffers(buf, offs), buf, offs


def carve_buffers(buf, offs) -> dict:
    """The per-gradient views of a flat backward buffer (see backward_buffers)."""
    return {k: buf[o:o + n].view(*shape) for k, (o, n, shape) in offs.items()}


def rasterize_gaussians_backward(background, means3D, radii, colors, semantic_feature, scales,
                                 rotations, scale_modifier, cov3D_precomp, viewmatrix, projmatrix,
                                 c_x, c_y, tan_fovx, tan_fovy, dL_dout_color, dL_dout_feature,
                                 dL_dout_depth, dL_dout_alpha, sh, degree, campos, geomBuffer, R,
                                 binningBuffer, imageBuffer, alphas, debug, *, compat=None,
                                 grad_mask=None, out=None, accumulate=False, densify=None):
    """RasterizeGaussiansBackwardCUDA (DGR/rasterize_points.cu:128-225).

    Camera scalars are consumed in this positional order, exactly as the
    reference binding consumes them.  Returns (dL_dmeans2D[P,3],
    dL_dcolors[P,3], dL_dsemantic[P,F], dL_dopacity[P,1], dL_dmeans3D[P,3],
    dL_dcov3D[P,6], dL_dsh[P,M,3], dL_dscales[P,3], dL_drotations[P,4]).

    `grad_mask` (keyword-only, no reference analogue in the binding): an
    optional per-Gaussian [P] mask fused into the kernel, equal to the
    reference wrapper's `grad * label` (__init__.py:159-173) on every returned
    gradient except dL_dmeans2D and dL_dsemantic.

    `out` / `accumulate` (keyword-only, no reference analogue): caller-owned
    gradient buffers (a dict with the keys of `backward_buffers`) written in
    place, and with `accumulate=True` ADDED to (GS_FLAG_ACCUMULATE) -- the
    multi-camera gradient sink (rasterizer.GradientSink).  Accumulating calls
    into the same buffers must be ordered on one stream.

    `densify` (keyword-only, no reference analogue): optional (accum, denom,
    max_radius) fp32 [P] tensors that receive this view's densification
    statistics (external.py:136-140, train.py:288-290; gsplat_hip.h
    gs_gaussians.densify_accum), written or, with `accumulate`, added.
    """
    L_ = _lib.load()
    cm = _compat_code(compat)
    nat = _native_mod()
    if nat is not None and means3D.is_cuda and means3D.dim() == 2 and means3D.size(0) > 0:
        if accumulate and out is None:
            raise ValueError("accumulate=True needs the caller's gradient buffers (out=...)")
        try:
            return nat.backward(background, means3D, radii, _opt(colors), _opt(semantic_feature),
                                _opt(scales), _opt(rotations), float(scale_modifier), _opt(cov3D_precomp),
                                viewmatrix, projmatrix, float(c_x), float(c_y), float(tan_fovx),
                                float(tan_fovy), _opt(dL_dout_color), _opt(dL_dout_feature),
                                _opt(dL_dout_depth), _opt(dL_dout_alpha), _opt(sh), int(degree), campos,
                                geomBuffer, int(R), _opt(binningBuffer), imageBuffer, alphas, bool(debug), cm,
                                _opt(grad_mask), None if out is None else [out[k] for k in _BUFFER_ORDER],
                                bool(accumulate), None if densify is None else list(densify),
                                torch.cuda.current_stream(means3D.device).cuda_stream)
        except RuntimeError as ex:
            raise _lib.GsplatError(str(ex)) from None
    inp = _Inputs(means3D, colors, semantic_feature, None, scales, rotations, scale_modifier,
                  cov3D_precomp, sh, degree)
    dev, P = inp.device, inp.P
    # rasterize_points.cu:160-161 takes H, W from dL_dout_color; an absent
    # (None / empty) upstream gradient counts as zeros, sized from the alpha image
    img_ref = dL_dout_color if _present(dL_dout_color) else alphas
    H, W = img_ref.size(-2), img_ref.size(-1)
    f32 = dict(dtype=torch.float32, device=dev)
    if P == 0:
        z = lambda *s: torch.zeros(*s, **f32)  # noqa: E731
        return (z(0, 3), z(0, 3), z(0, inp.F_user), z(0, 1), z(0, 3), z(0, 6), z(0, inp.M, 3),
                z(0, 3), z(0, 4))
    cam, keep = _camera(dev, background, viewmatrix, projmatrix, campos, c_x, c_y, tan_fovx,
                        tan_fovy, W, H)
    g = inp.struct()
    if grad_mask is not None:
        gm = grad_mask.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        if gm.numel() != P:
            raise RuntimeError(f"grad_mask must have {P} elements, got {gm.numel()}")
        g.grad_mask = gm.data_ptr()
    dLc = _dev(dL_dout_color, dev, "dL_dout_color") if _present(dL_dout_color) else None
    dLd = _dev(dL_dout_depth, dev, "dL_dout_depth") if _present(dL_dout_depth) else None
    dLa = _dev(dL_dout_alpha, dev, "dL_dout_alpha") if _present(dL_dout_alpha) else None
    alphas_c = _dev(alphas, dev, "alpha")
    dLf = None
    if inp.F and _present(dL_dout_feature):
        dLf = _dev(dL_dout_feature, dev, "dL_dout_feature").reshape(-1, H, W)
        if dLf.size(0) < inp.F:
            dLf = torch.cat([dLf, torch.zeros(inp.F - dLf.size(0), H, W, **f32)]).contiguous()
    radii_c = radii.to(device=dev, dtype=torch.int32).contiguous()
    if out is None:
        if accumulate:
            raise ValueError("accumulate=True needs the caller's gradient buffers (out=...)")
        out = backward_buffers(P, inp.F, inp.M, dev)
    else:
        for k, shape in _buffer_shapes(P, inp.F, inp.M).items():
            t = out[k]
            if (tuple(t.shape) != shape or t.dtype != torch.float32 or t.device != dev
                    or not t.is_contiguous()):
                raise RuntimeError(f"gradient buffer {k} must be a contiguous fp32 {shape} tensor on {dev}")
        if accumulate:
            g.flags = _lib.GS_FLAG_ACCUMULATE
    if densify is not None:
        for t in densify:
            if tuple(t.shape) != (P,) or t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
                raise RuntimeError(f"densify statistics must be contiguous fp32 ({P},) tensors on {dev}")
        g.densify_accum, g.densify_denom, g.max_radius = (t.data_ptr() for t in densify)
    scratch = torch.empty(L_.gs_backward_scratch_bytes(P, inp.F), dtype=torch.uint8, device=dev)
    stream = _stream(dev)
    p = lambda t: t.data_ptr() if (t is not None and t.numel()) else None  # noqa: E731
    check(L_.gs_backward(ctypes.byref(g), ctypes.byref(cam), radii_c.data_ptr(), int(bool(debug)), cm,
                         geomBuffer.data_ptr(), p(binningBuffer), imageBuffer.data_ptr(), int(R),
                         alphas_c.data_ptr(), p(dLc), p(dLf), p(dLd), p(dLa),
                         scratch.data_ptr(), out["dmeans2D"].data_ptr(), out["dcolors"].data_ptr(),
                         p(out["dsem"]), out["dopacity"].data_ptr(), out["dmeans3D"].data_ptr(),
                         out["dcov3D"].data_ptr(), p(out["dsh"]), out["dscales"].data_ptr(),
                         out["drot"].data_ptr(), stream), "rasterize_gaussians_backward")
    del keep
    dsem = out["dsem"][:, :inp.F_user] if inp.F_user != inp.F else out["dsem"]
    return (out["dmeans2D"], out["dcolors"], dsem, out["dopacity"], out["dmeans3D"],
            out["dcov3D"], out["dsh"], out["dscales"], out["drot"])


def binned_instances(imageBuffer, image_height, image_width) -> int:
    """Length of the tile lists a forward binned (num_instances <= the
    returned num_rendered): read from the image buffer's tile ranges.  An
    introspection helper (byte models, tests); synchronises the stream."""
    L_ = _lib.load()
    W, H = int(image_width), int(image_height)
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    rg = torch.empty(max(tiles, 1), 2, dtype=torch.int32, device=imageBuffer.device)
    check(L_.gs_debug_export(0, W, H, None, None, imageBuffer.data_ptr(), 0, None, None, None, None, None,
                             None, rg.data_ptr(), None, _stream(imageBuffer.device)), "binned_instances")
    r = rg[:tiles].cpu().numpy().view("uint32")
    return int(r[:, 1].max()) if tiles else 0


def mark_visible(means3D, viewmatrix, projmatrix):
    """markVisible (DGR/rasterize_points.cu:227-246): bool[P], view-space z > 0."""
    L_ = _lib.load()
    dev = means3D.device
    if dev.type != "cuda":
        raise _lib.GsplatError("mark_visible needs device tensors")
    P = means3D.size(0)
    present = torch.zeros(P, dtype=torch.bool, device=dev)
    if P:
        m = _dev(means3D, dev, "means3D")
        v = _dev(viewmatrix, dev, "viewmatrix").reshape(-1)
        pr = _dev(projmatrix, dev, "projmatrix").reshape(-1)
        check(L_.gs_mark_visible(P, m.data_ptr(), v.data_ptr(), pr.data_ptr(), present.data_ptr(),
                                 _stream(dev)), "mark_visible")
    return present


# ---------------------------------------------------------------------------
# Camera batches (include/gsplat_hip.h gs_*_batch; no reference analogue): the
# C cameras of one multi-camera step rendered with one launch per stage.

def _camera_batch(dev, background, viewmatrices, projmatrices, campos, c_x, c_y, tan_fovx, tan_fovy, W, H,
                  windows=None):
    C = len(c_x)
    if windows is not None and len(windows) != C:
        raise RuntimeError("tile windows: one (x0, y0, x1, y1) per camera")
    if not (1 <= C <= 64):
        raise _lib.GsplatError(f"camera batch size {C} outside 1..64")
    if not (len(c_y) == len(tan_fovx) == len(tan_fovy) == C):
        raise RuntimeError("per-camera scalars must all have C entries")
    view = _dev(viewmatrices, dev, "viewmatrices").reshape(C, 16).contiguous()
    proj = _dev(projmatrices, dev, "projmatrices").reshape(C, 16).contiguous()
    cpos = _dev(campos, dev, "campos").reshape(C, 3).contiguous()
    bg = _dev(background, dev, "bg").reshape(-1)
    cams = (GsCamera * C)()
    for c in range(C):
        cams[c] = GsCamera(viewmatrix=view.data_ptr() + 64 * c, projmatrix=proj.data_ptr() + 64 * c,
                           campos=cpos.data_ptr() + 12 * c, background=bg.data_ptr(), c_x=float(c_x[c]),
                           c_y=float(c_y[c]), tan_fovx=float(tan_fovx[c]), tan_fovy=float(tan_fovy[c]),
                           image_width=int(W), image_height=int(H))
        if windows is not None and windows[c] is not None:
            cams[c].tile_x0, cams[c].tile_y0, cams[c].tile_x1, cams[c].tile_y1 = (int(v) for v in windows[c])
    return cams, C, [view, proj, cpos, bg]


def _event_handle(ev) -> int:
    """The hipEvent_t of a recorded torch.cuda.Event (0 = none)."""
    return 0 if ev is None else int(ev.cuda_event)


def _windows_arg(windows, C):
    """Tile windows as the native binding takes them: C x [x0, y0, x1, y1]
    (all 0 = the whole image), or an empty list for none."""
    if windows is None:
        return []
    return [[0, 0, 0, 0] if w is None else [int(v) for v in w] for w in windows]


class BinningPlan:
    """State of the sync-free batch forward (gs_forward_batch, ABI 11) over
    the calls of one camera set: per camera the binning buffer's capacity
    (the last call's exact list instances x (1 + margin) + slack) and the
    previous plan's sort extents (gs_batch_hint).  The first call has no
    capacity: it runs with capacity 0, which never fits, and takes the retry
    with the exact lengths -- one forward in the two-phase path's cost.
    `calls`, `retries` (attempts that did not fit after the first call) and
    `num_instances` (exact, last call) are for the caller to inspect;
    `force_capacity` (tests) replaces the computed capacities once."""

    def __init__(self, margin: float = 0.125, slack: int = 4096):
        self.margin, self.slack = float(margin), int(slack)
        self.capacity = None
        self.hint = [0, 0, 0, 0, 0, 0]  # gs_batch_hint {valid, p1, q1, p2, max_len, total}
        self.num_instances = None
        self.calls = 0
        self.retries = 0
        self.force_capacity = None

    def next_capacity(self, C):
        if self.force_capacity is not None:
            cap, self.force_capacity = [int(x) for x in self.force_capacity], None
            return cap
        if self.capacity is None or len(self.capacity) != C:
            return [0] * C
        return list(self.capacity)

    def update(self, num_instances, hint, fitted, first):
        self.calls += 1
        if not fitted and not first:
            self.retries += 1
        self.num_instances = [int(x) for x in num_instances]
        self.capacity = [int(n * (1.0 + self.margin)) + self.slack for n in self.num_instances]
        self.hint = [int(x) for x in hint]


def batch_backward_scratch(means3D, semantic_feature, C: int):
    """An uninitialised scratch tensor of the batch backward's size
    (gs_batch_backward_scratch_bytes at the compiled feature width), for a
    caller that has the forward zero it (rasterize_gaussians_batch zero_fill)
    and hands it to the backward."""
    L_ = _lib.load()
    P = means3D.size(0)
    Fu = semantic_feature.numel() // max(P, 1) if _present(semantic_feature) else 0
    n = L_.gs_batch_backward_scratch_bytes(P, _feature_width(Fu), int(C))
    return torch.empty(max(16, n), dtype=torch.uint8, device=means3D.device)


def rasterize_gaussians_batch(background, means3D, colors, semantic_feature, opacity, scales, rotations,
                              scale_modifier, cov3D_precomp, viewmatrices, projmatrices, c_x, c_y, tan_fovx,
                              tan_fovy, image_height, image_width, sh, degree, campos, prefiltered, debug,
                              *, compat=None, activate=False, windows=None, feature_ready=None, plan_state=None,
                              walk_order=None, zero_fill=None):
    """The forward of C cameras at once (gs_forward_plan_batch +
    gs_forward_render_batch): the arguments of rasterize_gaussians with
    per-camera matrices stacked ([C,4,4] or [C,16], campos [C,3]) and the
    camera scalars as length-C sequences.  Returns (num_rendered[C],
    color[C,3,H,W], feature_map[C,F,H,W], depth[C,1,H,W], alpha[C,1,H,W],
    radii[C,P] int32, geomBuffer, binningBuffer, imgBuffer, num_instances[C]);
    camera c's outputs equal rasterize_gaussians' for that camera.
    `activate`: opacity / scales / rotations are the raw parameters
    (logit, log, unnormalised; GS_FLAG_ACTIVATE).  `windows`: per camera a
    tile window (x0, y0, x1, y1) or None (gs_camera tile_*).  `feature_ready`:
    a torch.cuda.Event (recorded) the blend waits for before reading the
    features (gs_gaussians.feature_ready), or None.  `plan_state`: a
    BinningPlan -- the sync-free forward (gs_forward_batch): no host round
    trip between the plan and the render stages, the binning buffer sized
    from the previous call and re-rendered with the exact lengths when it
    does not fit (bit-identical outputs either way).  The returned
    num_instances is then the per-camera length the binning buffer is laid
    out with (what the backward takes); the exact counts are in
    plan_state.num_instances.  `walk_order`: an int32 device tensor of the P
    ids in the order the binning passes walk them (spatial_order), or None
    (gs_gaussians.walk_order; outputs do not depend on it).  `zero_fill`: a
    device tensor the blend zeroes (its whole bytes, rounded down to 16) --
    the backward's scratch, handed to rasterize_gaussians_batch_backward
    with scratch_zeroed=True (gs_gaussians.zero_fill, ABI 13)."""
    L_ = _lib.load()
    sync_free = plan_state is not None and not debug
    cm = _compat_code(compat)
    if feature_ready is not None and _present(semantic_feature):
        sf = semantic_feature
        Fu = sf.numel() // max(means3D.size(0), 1)
        if not (sf.is_cuda and sf.dtype == torch.float32 and sf.is_contiguous() and _feature_width(Fu) == Fu):
            # the binding copies / pads the features on the calling stream
            # before any kernel runs: that copy has to wait too
            torch.cuda.current_stream(means3D.device).wait_event(feature_ready)
            feature_ready = None
    nat = _native_mod()
    if nat is not None and means3D.is_cuda and means3D.dim() == 2 and means3D.size(0) > 0:
        C_ = len(c_x)
        cap = plan_state.next_capacity(C_) if sync_free else []
        try:
            out = nat.forward_batch(background, means3D, _opt(colors), _opt(semantic_feature), _opt(opacity),
                                    _opt(scales), _opt(rotations), float(scale_modifier), _opt(cov3D_precomp),
                                    viewmatrices, projmatrices, [float(x) for x in c_x], [float(x) for x in c_y],
                                    [float(x) for x in tan_fovx], [float(x) for x in tan_fovy], int(image_height),
                                    int(image_width), _opt(sh), int(degree), campos, bool(prefiltered),
                                    bool(debug), cm, bool(activate), _windows_arg(windows, C_),
                                    _event_handle(feature_ready), cap,
                                    plan_state.hint if sync_free else [], _opt(walk_order), _opt(zero_fill),
                                    torch.cuda.current_stream(means3D.device).cuda_stream)
        except RuntimeError as ex:
            raise _lib.GsplatError(str(ex)) from None
        NR, color, fmap, depth, alpha, radii, geom, binning, img, NI, layout, hint, fitted = out
        if sync_free:
            plan_state.update(NI, hint, fitted, first=not any(cap))
            return (NR, color, fmap, depth, alpha, radii, geom, binning, img, layout)
        return (NR, color, fmap, depth, alpha, radii, geom, binning, img, NI)
    inp = _Inputs(means3D, colors, semantic_feature, opacity, scales, rotations, scale_modifier,
                  cov3D_precomp, sh, degree)
    dev, P = inp.device, inp.P
    H, W = int(image_height), int(image_width)
    cams, C, keep = _camera_batch(dev, background, viewmatrices, projmatrices, campos, c_x, c_y, tan_fovx,
                                  tan_fovy, W, H, windows)
    f32 = dict(dtype=torch.float32, device=dev)
    u8 = dict(dtype=torch.uint8, device=dev)
    if P == 0:
        return ([0] * C, torch.zeros(C, 3, H, W, **f32), torch.zeros(C, inp.F_user, H, W, **f32),
                torch.zeros(C, 1, H, W, **f32), torch.zeros(C, 1, H, W, **f32),
                torch.zeros(C, 0, dtype=torch.int32, device=dev), torch.empty(0, **u8), torch.empty(0, **u8),
                torch.empty(0, **u8), [0] * C)
    g = inp.struct(_lib.GS_FLAG_ACTIVATE if activate else 0)
    g.feature_ready = _event_handle(feature_ready) or None
    if walk_order is not None:
        if not (walk_order.is_cuda and walk_order.dtype == torch.int32 and walk_order.is_contiguous()
                and walk_order.numel() == inp.P and walk_order.device == dev):
            raise RuntimeError("walk_order must be a contiguous int32 device tensor of P ids")
        g.walk_order = walk_order.data_ptr()
    if zero_fill is not None:
        if not (zero_fill.is_contiguous() and zero_fill.device == dev):
            raise RuntimeError("zero_fill must be a contiguous device tensor")
        g.zero_fill = zero_fill.data_ptr()
        g.zero_fill_bytes = (zero_fill.numel() * zero_fill.element_size()) & ~15
    out_color = torch.empty(C, 3, H, W, **f32)
    out_feature = torch.empty(C, inp.F, H, W, **f32)
    out_depth = torch.empty(C, 1, H, W, **f32)
    out_alpha = torch.empty(C, 1, H, W, **f32)
    radii = torch.empty(C, P, dtype=torch.int32, device=dev)
    geom = torch.empty(L_.gs_batch_geom_buffer_bytes(P, C), **u8)
    img = torch.empty(L_.gs_batch_image_buffer_bytes(W, H, C), **u8)
    stream = _stream(dev)
    NR = (ctypes.c_int64 * C)()
    NI = (ctypes.c_int64 * C)()
    outs = (out_color.data_ptr(), out_feature.data_ptr() if inp.F else None, out_depth.data_ptr(),
            out_alpha.data_ptr())
    fitted = False
    if sync_free:
        cap_list = plan_state.next_capacity(C)
        cap = (ctypes.c_int64 * C)(*cap_list)
        hint = _lib.GsBatchHint(*plan_state.hint)
        binning = torch.empty(max(1, L_.gs_batch_binning_buffer_bytes(C, cap)), **u8)
        fits = ctypes.c_int32(0)
        check(L_.gs_forward_batch(ctypes.byref(g), cams, C, int(bool(prefiltered)), cm, geom.data_ptr(),
                                  img.data_ptr(), binning.data_ptr(), cap, ctypes.byref(hint), radii.data_ptr(),
                                  NR, NI, ctypes.byref(fits), *outs, stream),
              "rasterize_gaussians_batch (sync-free forward)")
        fitted = bool(fits.value)
    else:
        check(L_.gs_forward_plan_batch(ctypes.byref(g), cams, C, int(bool(prefiltered)), int(bool(debug)), cm,
                                       geom.data_ptr(), img.data_ptr(), radii.data_ptr(), NR, NI, stream),
              "rasterize_gaussians_batch (preprocess)")
    layout = list(NI)
    if fitted:
        layout = cap_list
    else:
        binning = torch.empty(max(1, L_.gs_batch_binning_buffer_bytes(C, NI)), **u8)
        check(L_.gs_forward_render_batch(ctypes.byref(g), cams, C, int(bool(debug)), cm, geom.data_ptr(),
                                         binning.data_ptr(), img.data_ptr(), NI, radii.data_ptr(), *outs, stream),
              "rasterize_gaussians_batch (render)")
    if sync_free:
        plan_state.update(list(NI), [hint.valid, hint.p1, hint.q1, hint.p2, hint.max_len, hint.total], fitted,
                          first=not any(cap_list))
    del keep
    feature_map = out_feature[:, :inp.F_user] if inp.F_user != inp.F else out_feature
    return (list(NR), out_color, feature_map, out_depth, out_alpha, radii, geom, binning, img, layout)


def rasterize_gaussians_batch_backward(background, means3D, radii, colors, semantic_feature, scales,
                                       rotations, scale_modifier, cov3D_precomp, viewmatrices, projmatrices,
                                       c_x, c_y, tan_fovx, tan_fovy, dL_dout_color, dL_dout_feature,
                                       dL_dout_depth, dL_dout_alpha, sh, degree, campos, geomBuffer,
                                       num_instances, binningBuffer, imageBuffer, alphas, debug, *,
                                       compat=None, grad_mask=None, densify=None, opacity=None,
                                       activate=False, windows=None, out=None, scratch=None,
                                       scratch_zeroed=False):
    """The backward of a camera batch (gs_backward_batch): the arguments of
    rasterize_gaussians_backward with stacked per-camera matrices, scalars
    and upstream gradients ([C, ...]), in the binding's positional camera
    semantics.  Returns the rasterize_gaussians_backward tuple with every
    per-Gaussian gradient SUMMED over the cameras.  `densify` as in
    rasterize_gaussians_backward (per-camera statistics, summed).
    `activate` (with the raw `opacity`): the gradients of the raw opacity /
    scale / rotation parameters (GS_FLAG_ACTIVATE).  `out`: optional
    {name: tensor} destinations of backward_buffers' names (e.g. the views of
    a gradient bucket, distributed.ShardedAdam.grad_views): those gradients
    are WRITTEN there (every element, not accumulated) instead of into fresh
    tensors; each must be a contiguous fp32 device tensor of the gradient's
    element count (dsem at the compiled feature width).  `scratch`: the
    backward's scratch (gs_batch_backward_scratch_bytes) kept from the
    forward, `scratch_zeroed`: the forward's blend zeroed it
    (rasterize_gaussians_batch zero_fill; GS_FLAG_SCRATCH_ZEROED)."""
    L_ = _lib.load()
    cm = _compat_code(compat)
    if activate and not _present(opacity):
        raise RuntimeError("activate=True needs the raw opacities")
    if out:
        unknown = set(out) - set(_buffer_shapes(0, 0, 0))
        if unknown:
            raise RuntimeError(f"out: unknown gradient names {sorted(unknown)}")
    nat = _native_mod()
    if nat is not None and means3D.is_cuda and means3D.dim() == 2 and means3D.size(0) > 0:
        try:
            return nat.backward_batch(background, means3D, radii, _opt(colors), _opt(semantic_feature),
                                      _opt(scales), _opt(rotations), float(scale_modifier), _opt(cov3D_precomp),
                                      viewmatrices, projmatrices, [float(x) for x in c_x],
                                      [float(x) for x in c_y], [float(x) for x in tan_fovx],
                                      [float(x) for x in tan_fovy], _opt(dL_dout_color), _opt(dL_dout_feature),
                                      _opt(dL_dout_depth), _opt(dL_dout_alpha), _opt(sh), int(degree), campos,
                                      geomBuffer, [int(x) for x in num_instances], _opt(binningBuffer),
                                      imageBuffer, alphas, bool(debug), cm, _opt(grad_mask),
                                      None if densify is None else list(densify), _opt(opacity), bool(activate),
                                      _windows_arg(windows, len(c_x)),
                                      [out.get(k, _NO_DEST) for k in _buffer_shapes(0, 0, 0)] if out else [],
                                      _opt(scratch), bool(scratch_zeroed),
                                      torch.cuda.current_stream(means3D.device).cuda_stream)
        except RuntimeError as ex:
            raise _lib.GsplatError(str(ex)) from None
    inp = _Inputs(means3D, colors, semantic_feature, opacity if activate else None, scales, rotations,
                  scale_modifier, cov3D_precomp, sh, degree)
    dev, P = inp.device, inp.P
    C = len(c_x)
    img_ref = dL_dout_color if _present(dL_dout_color) else alphas
    H, W = img_ref.size(-2), img_ref.size(-1)
    f32 = dict(dtype=torch.float32, device=dev)
    if P == 0:
        z = lambda *s: torch.zeros(*s, **f32)  # noqa: E731
        return (z(0, 3), z(0, 3), z(0, inp.F_user), z(0, 1), z(0, 3), z(0, 6), z(0, inp.M, 3),
                z(0, 3), z(0, 4))
    cams, C, keep = _camera_batch(dev, background, viewmatrices, projmatrices, campos, c_x, c_y, tan_fovx,
                                  tan_fovy, W, H, windows)
    g = inp.struct(_lib.GS_FLAG_ACTIVATE if activate else 0)
    if grad_mask is not None:
        gm = grad_mask.to(device=dev, dtype=torch.float32).reshape(-1).contiguous()
        if gm.numel() != P:
            raise RuntimeError(f"grad_mask must have {P} elements, got {gm.numel()}")
        g.grad_mask = gm.data_ptr()

    def img(t, ch, name):
        if not _present(t):
            return None
        t = _dev(t, dev, name).reshape(C, -1, H, W)
        if t.size(1) < ch:
            t = torch.cat([t, torch.zeros(C, ch - t.size(1), H, W, **f32)], 1)
        return t.contiguous()
    dLc = img(dL_dout_color, 3, "dL_dout_color")
    dLd = img(dL_dout_depth, 1, "dL_dout_depth")
    dLa = img(dL_dout_alpha, 1, "dL_dout_alpha")
    dLf = img(dL_dout_feature, inp.F, "dL_dout_feature") if inp.F else None
    alphas_c = _dev(alphas, dev, "alpha")
    radii_c = radii.to(device=dev, dtype=torch.int32).contiguous()
    if tuple(radii_c.shape) != (C, P):
        raise RuntimeError(f"radii must be [C={C}, P={P}]")
    dest = out or {}
    out = backward_buffers(P, inp.F, inp.M, dev)
    for k, t in dest.items():
        want = out[k]
        if t.dtype != torch.float32 or t.device != dev or not t.is_contiguous() or t.numel() != want.numel():
            raise RuntimeError(f"out['{k}'] must be a contiguous fp32 tensor of {want.numel()} elements on {dev}")
        out[k] = t.view(want.shape)
    if densify is not None:
        for t in densify:
            if tuple(t.shape) != (P,) or t.dtype != torch.float32 or t.device != dev or not t.is_contiguous():
                raise RuntimeError(f"densify statistics must be contiguous fp32 ({P},) tensors on {dev}")
        g.densify_accum, g.densify_denom, g.max_radius = (t.data_ptr() for t in densify)
    NI = (ctypes.c_int64 * C)(*[int(x) for x in num_instances])
    nscr = L_.gs_batch_backward_scratch_bytes(P, inp.F, C)
    if scratch is None:
        scratch = torch.empty(nscr, dtype=torch.uint8, device=dev)
    else:
        if not (scratch.is_contiguous() and scratch.device == dev and scratch.numel() * scratch.element_size() >= nscr):
            raise RuntimeError(f"scratch must be a contiguous device tensor of {nscr} bytes on {dev}")
        if scratch_zeroed:
            g.flags |= _lib.GS_FLAG_SCRATCH_ZEROED
    stream = _stream(dev)
    p = lambda t: t.data_ptr() if (t is not None and t.numel()) else None  # noqa: E731
    check(L_.gs_backward_batch(ctypes.byref(g), cams, C, radii_c.data_ptr(), int(bool(debug)), cm,
                               geomBuffer.data_ptr(), p(binningBuffer), imageBuffer.data_ptr(), NI,
                               alphas_c.data_ptr(), p(dLc), p(dLf), p(dLd), p(dLa), scratch.data_ptr(),
                               out["dmeans2D"].data_ptr(), out["dcolors"].data_ptr(), p(out["dsem"]),
                               out["dopacity"].data_ptr(), out["dmeans3D"].data_ptr(), out["dcov3D"].data_ptr(),
                               p(out["dsh"]), out["dscales"].data_ptr(), out["drot"].data_ptr(), stream),
          "rasterize_gaussians_batch_backward")
    del keep
    dsem = out["dsem"][:, :inp.F_user] if inp.F_user != inp.F else out["dsem"]
    return (out["dmeans2D"], out["dcolors"], dsem, out["dopacity"], out["dmeans3D"],
            out["dcov3D"], out["dsh"], out["dscales"], out["drot"])
