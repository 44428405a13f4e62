"""Autograd boundary of the MI355X rasterizer -- drop-in for
DGR/diff_gaussian_rasterization/__init__.py (DGR = submodules_fsgs/
diff-gaussian-rasterization-confidence).

Same public names (GaussianRasterizationSettings, GaussianRasterizer,
rasterize_gaussians, _RasterizeGaussians), same argument meaning, same
debug-snapshot and error behaviour, as a SUPERSET of the four caller API
generations found in Dynamic3DGaussians:

  G1 no label, no semantic_feature -> (color, radii, depth)        train.py:142
  G2 label,    no semantic_feature -> (color, radii, depth, alpha)  cvpr_dyn.py:241
  G3 label,    semantic_feature    -> (color, radii, feature_map, depth, alpha)
                                      (the vendored API, __init__.py:108)
  G4 no label, semantic_feature    -> (color, feature_map, radii, depth)
                                      gaussian_renderer/__init__.py:93-102

`rasterize_gaussians` / `_RasterizeGaussians` always return the G3 5-tuple,
like the reference.  Numerics follow settings.compat (default: the module
default, "reference"); see DESIGN.md "Quirks".
"""
from __future__ import annotations

import os

from typing import NamedTuple, Optional, Tuple

import torch
import torch.nn as nn

from . import _C, _lib
from ._C import get_default_compat as _default_compat


def cpu_deep_copy_tuple(input_tuple):
    """__init__.py:17-19: CPU copies of the argument tuple for debug snapshots."""
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item
                 for item in input_tuple)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, semantic_feature, opacities, scales,
                        rotations, cov3Ds_precomp, raster_settings, label=None):
    """__init__.py:21-46."""
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, semantic_feature,
                                     opacities, scales, rotations, cov3Ds_precomp, raster_settings,
                                     label)


def _empty_like_none(t):
    return t if t is not None else torch.Tensor([])


def _compat_of(settings) -> str:
    mode = getattr(settings, "compat", None)
    return _default_compat() if mode is None else mode


def _principal_point(settings):
    cx = settings.c_x if settings.c_x is not None else settings.image_width / 2.0
    cy = settings.c_y if settings.c_y is not None else settings.image_height / 2.0
    return float(cx), float(cy)


_FUSABLE_LABEL_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.bool, torch.uint8,
                         torch.int8, torch.int16, torch.int32, torch.int64)


class _RasterizeGaussians(torch.autograd.Function):
    """__init__.py:48-174."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, semantic_feature, opacities, scales,
                rotations, cov3Ds_precomp, raster_settings, label):
        compat = _compat_of(raster_settings)
        c_x, c_y = _principal_point(raster_settings)
        for name in ("bg", "viewmatrix", "projmatrix", "campos"):
            if getattr(raster_settings, name) is None:
                raise TypeError(f"GaussianRasterizationSettings.{name} is required")
        sh = _empty_like_none(sh)
        colors_precomp = _empty_like_none(colors_precomp)
        scales = _empty_like_none(scales)
        rotations = _empty_like_none(rotations)
        cov3Ds_precomp = _empty_like_none(cov3Ds_precomp)
        # Argument order of the C++ binding (__init__.py:67-90)
        args = (raster_settings.bg, means3D, colors_precomp, semantic_feature, opacities, scales,
                rotations, raster_settings.scale_modifier, cov3Ds_precomp,
                raster_settings.viewmatrix, raster_settings.projmatrix, c_x, c_y,
                raster_settings.tanfovx, raster_settings.tanfovy, raster_settings.image_height,
                raster_settings.image_width, sh, raster_settings.sh_degree, raster_settings.campos,
                raster_settings.prefiltered, raster_settings.debug)
        if raster_settings.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                out = _C.rasterize_gaussians(*args, compat=compat)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
                raise ex
        else:
            out = _C.rasterize_gaussians(*args, compat=compat)
        num_rendered, color, feature_map, depth, alpha, radii, geomBuffer, binningBuffer, imgBuffer = out

        ctx.raster_settings = raster_settings
        ctx.num_rendered = num_rendered
        # outputs without a gradient arrive as None (no zero images are
        # materialized); the binding treats them as zeros
        ctx.set_materialize_grads(False)
        ctx.compat = compat
        ctx.c_xy = (c_x, c_y)
        ctx.sem_shape = None if semantic_feature is None else tuple(semantic_feature.shape)
        ctx.save_for_backward(colors_precomp, semantic_feature, means3D, scales, rotations,
                              cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer, imgBuffer, alpha,
                              label if isinstance(label, torch.Tensor) else None)
        ctx.mark_non_differentiable(radii)
        return color, radii, feature_map, depth, alpha

    @staticmethod
    def backward(ctx, grad_color, grad_radii, grad_out_feature, grad_depth, grad_alpha):
        num_rendered = ctx.num_rendered
        rs = ctx.raster_settings
        (colors_precomp, semantic_feature, means3D, scales, rotations, cov3Ds_precomp, radii, sh,
         geomBuffer, binningBuffer, imgBuffer, alpha, label) = ctx.saved_tensors
        c_x, c_y = ctx.c_xy
        if ctx.compat == "reference":
            # Q2: the reference passes tanfovx, tanfovy, c_x, c_y into the
            # binding's (c_x, c_y, tan_fovx, tan_fovy) slots (__init__.py:130-133
            # vs rasterize_points.cu:141-144); reproduced in "reference" mode.
            cam4 = (rs.tanfovx, rs.tanfovy, c_x, c_y)
        else:
            cam4 = (c_x, c_y, rs.tanfovx, rs.tanfovy)
        args = (rs.bg, means3D, radii, colors_precomp, semantic_feature, scales, rotations,
                rs.scale_modifier, cov3Ds_precomp, rs.viewmatrix, rs.projmatrix, *cam4,
                grad_color, grad_out_feature, grad_depth, grad_alpha, sh, rs.sh_degree, rs.campos,
                geomBuffer, num_rendered, binningBuffer, imgBuffer, alpha, rs.debug)
        # The label mask is fused into the backward kernel when that is
        # bit-identical to the wrapper's `grad * label.unsqueeze(1)` (a [P]
        # label whose dtype does not promote fp32); otherwise it is applied
        # below exactly as the reference does.
        fuse = (label is not None and label.dim() == 1 and label.numel() == means3D.size(0)
                and label.dtype in _FUSABLE_LABEL_DTYPES)
        kw = dict(compat=ctx.compat, grad_mask=label if fuse else None)
        sink = getattr(rs, "grad_sink", None)
        if sink is not None and (label is None or fuse):
            if ctx.needs_input_grad[1] and not sink._warned_means2D:
                # means2D.grad stays None on this path (see GradientSink)
                import warnings
                warnings.warn("GradientSink: means2D.grad is not populated; use sink.densify_stats() / "
                              "sink.update_densify_stats(variables) for the densification statistics "
                              "and sink.gradients()['means2D'] for the summed gradient", RuntimeWarning)
                sink._warned_means2D = True
            # multi-camera step: the kernels add this camera's gradients into
            # the sink's buffers of the current stream; autograd gets None
            P = means3D.size(0)
            F = _C._feature_width(semantic_feature.numel() // max(P, 1)) if (
                semantic_feature is not None and semantic_feature.numel()) else 0
            M = sh.size(1) if sh.numel() else 0
            kw["out"], kw["accumulate"], kw["densify"] = sink._claim(means3D.device, P, F, M, ctx.sem_shape)
            _C.rasterize_gaussians_backward(*args, **kw)
            return (None,) * len(ctx.needs_input_grad)
        if rs.debug:
            cpu_args = cpu_deep_copy_tuple(args)
            try:
                grads = _C.rasterize_gaussians_backward(*args, **kw)
            except Exception as ex:
                torch.save(cpu_args, "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
                raise ex
        else:
            grads = _C.rasterize_gaussians_backward(*args, **kw)
        (grad_means2D, grad_colors_precomp, grad_semantic_feature, grad_opacities, grad_means3D,
         grad_cov3Ds_precomp, grad_sh, grad_scales, grad_rotations) = grads
        if ctx.sem_shape is not None:
            grad_semantic_feature = grad_semantic_feature.reshape(ctx.sem_shape)
        else:
            grad_semantic_feature = None
        if label is not None and not fuse:
            # __init__.py:159-173: every Gaussian-parameter gradient except
            # means2D and the semantic feature is masked by `label` (Q12).
            lab = label.unsqueeze(1)
            grad_means3D = grad_means3D * lab
            grad_sh = grad_sh * lab[..., None]
            grad_colors_precomp = grad_colors_precomp * lab
            grad_opacities = grad_opacities * lab
            grad_scales = grad_scales * lab
            grad_rotations = grad_rotations * lab
            grad_cov3Ds_precomp = grad_cov3Ds_precomp * lab
        grads = (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_semantic_feature,
                 grad_opacities, grad_scales, grad_rotations, grad_cov3Ds_precomp, None, None)
        # inputs that were absent (None) or do not require grad get None
        return tuple(g if need else None for g, need in zip(grads, ctx.needs_input_grad))


class GaussianRasterizationSettings(NamedTuple):
    """__init__.py:176-192, as a superset: c_x / c_y default to the image
    centre (G4 callers omit them), `confidence` is accepted and unused like
    the reference, and `compat` selects reference/fixed numerics."""
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    c_x: Optional[float] = None
    c_y: Optional[float] = None
    bg: Optional[torch.Tensor] = None
    scale_modifier: float = 1.0
    viewmatrix: Optional[torch.Tensor] = None
    projmatrix: Optional[torch.Tensor] = None
    sh_degree: int = 0
    campos: Optional[torch.Tensor] = None
    prefiltered: bool = False
    debug: bool = False
    confidence: Optional[torch.Tensor] = None
    compat: Optional[str] = None
    grad_sink: Optional["GradientSink"] = None  # multi-camera gradient sum (no reference analogue)
    # image sharding (no reference analogue): render only the 16x16 tiles
    # [x0, x1) x [y0, y1) of the camera (gs_camera tile_*); camera batches only
    tile_window: Optional[Tuple[int, int, int, int]] = None


class GradientSink:
    """Sums the per-Gaussian gradients of many rasterizations -- the cameras of
    one multi-camera training step -- inside the backward kernels.

    With `GaussianRasterizationSettings(..., grad_sink=sink)`, the backward of
    every rasterization writes (first camera of the step on a stream) or adds
    (GS_FLAG_ACCUMULATE, the following ones) its gradients into per-stream
    buffers owned by the sink and hands autograd None for the Gaussian
    inputs, instead of returning a fresh gradient set per camera that autograd
    then adds into the leaves (one elementwise add per camera and parameter).
    `gradients()` returns the sums.  The reference has no counterpart: its
    training loop steps once per camera (train.py:422-433); the sum equals
    what autograd accumulates over the same cameras up to fp32 reordering
    (tests/test_gpu_streams.py).  Gradients whose label is not fusable into
    the kernel (see _RasterizeGaussians.backward) bypass the sink.

    Per-stream slots: autograd runs a camera's backward on its forward's
    stream, and the accumulation is a non-atomic read-modify-write, so each
    stream sums into its own buffers.

    Densification statistics.  The sink hands autograd None, so means2D.grad
    is not populated; the reference's per-camera bookkeeping
    (accumulate_mean2d_gradient, external.py:136-140: the NORM of each
    camera's own means2D gradient, and the max screen radius,
    train.py:288-290) is kept by the backward kernel instead, per camera
    (gs_gaussians.densify_accum): `densify_stats()` returns this step's
    increments and `update_densify_stats(variables)` adds them to the
    reference's `variables` dict.  (The norm of the summed means2D gradient,
    sink.gradients()['means2D'], would be a different criterion.)  Equal to
    the reference's per-camera updates up to fp32 reordering of the sum.
    """
    # backward buffer -> GaussianRasterizer argument name
    NAMES = {"dmeans3D": "means3D", "dmeans2D": "means2D", "dsh": "shs", "dcolors": "colors_precomp",
             "dsem": "semantic_feature", "dopacity": "opacities", "dscales": "scales",
             "drot": "rotations", "dcov3D": "cov3D_precomp"}

    def __init__(self):
        self._slots = {}
        self._sem_shape = None
        self._warned_means2D = False

    def reset(self) -> None:
        """Start a new sum (the next backward on each stream overwrites)."""
        for slot in self._slots.values():
            slot["fresh"] = True

    def _claim(self, device, P, F, M, sem_shape):
        key = (device, torch.cuda.current_stream(device).cuda_stream)
        slot = self._slots.get(key)
        if slot is None or slot["shape"] != (P, F, M):
            bufs, flat, offs = _C.backward_buffers(P, F, M, device, flat=True)
            stats = torch.empty(3, P, dtype=torch.float32, device=device)  # accum, denom, max radius
            slot = {"bufs": bufs, "flat": flat, "offs": offs, "shape": (P, F, M), "fresh": True,
                    "stats": stats}
            self._slots[key] = slot
        accumulate = not slot["fresh"]
        slot["fresh"] = False
        self._sem_shape = sem_shape
        return slot["bufs"], accumulate, tuple(slot["stats"].unbind(0))

    def densify_stats(self) -> dict:
        """This step's densification statistics, summed over its cameras:
        {'means2D_gradient_accum': sum of the per-camera |dL/dmeans2D[:, :2]|
        of the cameras that saw each Gaussian, 'denom': how many saw it,
        'max_2D_radius': the largest screen radius} -- [P] fp32 each, zero
        for Gaussians no camera saw.  Call like gradients()."""
        live = [s for s in self._slots.values() if not s["fresh"]]
        if not live:
            return {}
        st = live[0]["stats"].clone()
        for slot in live[1:]:
            st[:2] += slot["stats"][:2]
            torch.maximum(st[2], slot["stats"][2], out=st[2])
        return {"means2D_gradient_accum": st[0], "denom": st[1], "max_2D_radius": st[2]}

    def update_densify_stats(self, variables: dict) -> None:
        """The reference's per-camera statistics updates for every camera of
        the step (external.py:136-140, train.py:288-290) on its `variables`
        dict: accum += sum of norms, denom += count, max_2D_radius =
        max(max_2D_radius, radius) -- unseen Gaussians are unchanged."""
        st = self.densify_stats()
        if not st:
            return
        variables["means2D_gradient_accum"] += st["means2D_gradient_accum"]
        variables["denom"] += st["denom"]
        torch.maximum(variables["max_2D_radius"], st["max_2D_radius"], out=variables["max_2D_radius"])

    def gradients(self) -> dict:
        """Summed gradients by GaussianRasterizer argument name (means3D,
        means2D, shs, colors_precomp, semantic_feature, opacities, scales,
        rotations, cov3D_precomp); absent inputs are left out.  Call on a
        stream ordered after every accumulating stream.  With one stream the
        tensors alias the sink's buffers: valid until the next reset()."""
        live = [s for s in self._slots.values() if not s["fresh"]]
        if not live:
            return {}
        if any(s["shape"] != live[0]["shape"] for s in live[1:]):
            raise _lib.GsplatError("GradientSink: the streams' gradient sets have different shapes")
        # one elementwise add per extra stream over the whole gradient set
        if len(live) == 1:
            bufs = live[0]["bufs"]
        else:
            flat = live[0]["flat"] + live[1]["flat"]
            for slot in live[2:]:
                flat.add_(slot["flat"])
            bufs = _C.carve_buffers(flat, live[0]["offs"])
        out = {name: bufs[k] for k, name in self.NAMES.items()}
        P, F, M = live[0]["shape"]
        if M == 0:
            del out["shs"]
        if self._sem_shape is None or F == 0:
            del out["semantic_feature"]
        else:
            n = 1
            for d in self._sem_shape[1:]:
                n *= d
            out["semantic_feature"] = out["semantic_feature"][:, :n].reshape(self._sem_shape)
        return out


_UNSET = object()


class GaussianRasterizer(nn.Module):
    """__init__.py:194-245 with the caller-generation arity dispatch."""

    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities=None, shs=None, semantic_feature=None,
                colors_precomp=None, scales=None, rotations=None, cov3D_precomp=None, label=_UNSET):
        rs = self.raster_settings
        if getattr(rs, "tile_window", None) is not None:
            raise NotImplementedError("tile_window (image sharding) is a camera-batch feature: use "
                                      "GaussianRasterizerBatch")
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or '
                            'precomputed 3D covariance!')
        # __init__.py:218-230: absent inputs become empty tensors
        shs = torch.Tensor([]) if shs is None else shs
        colors_precomp = torch.Tensor([]) if colors_precomp is None else colors_precomp
        scales = torch.Tensor([]) if scales is None else scales
        rotations = torch.Tensor([]) if rotations is None else rotations
        cov3D_precomp = torch.Tensor([]) if cov3D_precomp is None else cov3D_precomp
        has_label = label is not _UNSET
        lab = label if (has_label and isinstance(label, torch.Tensor)) else None
        color, radii, feature_map, depth, alpha = rasterize_gaussians(
            means3D, means2D, shs, colors_precomp, semantic_feature, opacities, scales, rotations,
            cov3D_precomp, rs, lab)
        has_sem = semantic_feature is not None
        if has_label and has_sem:      # G3 (vendored API)
            return color, radii, feature_map, depth, alpha
        if has_label:                  # G2
            return color, radii, depth, alpha
        if has_sem:                    # G4 (feature-3DGS style)
            return color, feature_map, radii, depth
        return color, radii, depth     # G1 (upstream "w-depth" API)


# ---------------------------------------------------------------------------
# Camera batches (no reference analogue): the C cameras of one multi-camera
# training step rasterized together -- one launch per stage
# over all cameras (include/gsplat_hip.h gs_*_batch).  Camera c's outputs are
# those of GaussianRasterizer with settings[c]; the backward returns the
# gradients summed over the cameras, i.e. what autograd accumulates when the
# same inputs feed C per-camera rasterizations.

def _batch_settings(settings_list, check_values=True):
    """Validate a camera batch: one image size, scale modifier, SH degree,
    numerics and background.  The background comparison reads device values
    (a host synchronisation per camera), so GaussianRasterizerBatch does it
    once at construction (check_values=False afterwards)."""
    rs0 = settings_list[0]
    for rs in settings_list[1:]:
        for name in ("image_height", "image_width", "scale_modifier", "sh_degree", "prefiltered", "debug"):
            if getattr(rs, name) != getattr(rs0, name):
                raise ValueError(f"the cameras of a batch share {name}")
        if _compat_of(rs) != _compat_of(rs0):
            raise ValueError("the cameras of a batch share compat")
        if check_values and rs.bg is not rs0.bg and not torch.equal(rs.bg, rs0.bg):
            raise ValueError("the cameras of a batch share one background")
    for name in ("bg", "viewmatrix", "projmatrix", "campos"):
        if any(getattr(rs, name) is None for rs in settings_list):
            raise TypeError(f"GaussianRasterizationSettings.{name} is required")
    return rs0


class _BatchCameras:
    """The stacked per-camera device tensors and scalars of a validated
    camera batch (built once per GaussianRasterizerBatch)."""

    def __init__(self, settings_list, check_values=True):
        self.rs0 = _batch_settings(settings_list, check_values)
        self.C = len(settings_list)
        self.pp = [_principal_point(rs) for rs in settings_list]
        self.views = torch.stack([rs.viewmatrix.reshape(16) for rs in settings_list]).float().contiguous()
        self.projs = torch.stack([rs.projmatrix.reshape(16) for rs in settings_list]).float().contiguous()
        self.cpos = torch.stack([rs.campos.reshape(3) for rs in settings_list]).float().contiguous()
        self.tx = [rs.tanfovx for rs in settings_list]
        self.ty = [rs.tanfovy for rs in settings_list]
        wins = [getattr(rs, "tile_window", None) for rs in settings_list]
        self.windows = wins if any(w is not None for w in wins) else None


class _RasterizeGaussiansBatch(torch.autograd.Function):
    """_RasterizeGaussians over a list of camera settings (one launch per
    stage for all of them); outputs stacked [C, ...]."""

    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, semantic_feature, opacities, scales, rotations,
                cov3Ds_precomp, cams, label, densify_out, raw_params=False, feature_ready=None, plan_state=None,
                grad_into=None, walk_order=None):
        if not isinstance(cams, _BatchCameras):
            cams = _BatchCameras(cams)
        rs0 = cams.rs0
        compat = _compat_of(rs0)
        C = cams.C
        pp, views, projs, cpos = cams.pp, cams.views, cams.projs, cams.cpos
        sh = _empty_like_none(sh)
        colors_precomp = _empty_like_none(colors_precomp)
        scales = _empty_like_none(scales)
        rotations = _empty_like_none(rotations)
        cov3Ds_precomp = _empty_like_none(cov3Ds_precomp)
        tx, ty = cams.tx, cams.ty
        # the backward's scratch, zeroed by the forward's blend (whose HBM is
        # mostly idle) instead of a fill launch before the backward blend
        # (gs_gaussians.zero_fill, ABI 13): only when a backward can follow
        scratch = None
        if (any(ctx.needs_input_grad) and means3D.is_cuda and means3D.size(0) > 0
                and os.environ.get("GS_FORWARD_ZERO_SCRATCH", "1") != "0"):
            scratch = _C.batch_backward_scratch(means3D, semantic_feature, C)
        out = _C.rasterize_gaussians_batch(
            rs0.bg, means3D, colors_precomp, semantic_feature, opacities, scales, rotations, rs0.scale_modifier,
            cov3Ds_precomp, views, projs, [p[0] for p in pp], [p[1] for p in pp], tx, ty, rs0.image_height,
            rs0.image_width, sh, rs0.sh_degree, cpos, rs0.prefiltered, rs0.debug, compat=compat,
            activate=raw_params, windows=cams.windows, feature_ready=feature_ready, plan_state=plan_state,
            walk_order=walk_order, zero_fill=scratch)
        ctx.scratch, ctx.scratch_zeroed = scratch, scratch is not None
        num_rendered, color, feature_map, depth, alpha, radii, geom, binning, img, num_instances = out
        ctx.rs0 = rs0
        ctx.cams = (views, projs, cpos, pp, tx, ty, cams.windows)
        ctx.num_rendered = num_rendered
        ctx.num_instances = num_instances
        ctx.compat = compat
        ctx.C = C
        ctx.densify_out = densify_out
        ctx.raw_params = raw_params
        ctx.grad_into = _grad_destinations(grad_into, semantic_feature)
        if ctx.grad_into and isinstance(label, torch.Tensor) and not (
                label.dim() == 1 and label.numel() == means3D.size(0) and label.dtype in _FUSABLE_LABEL_DTYPES):
            raise ValueError("grad_into needs a per-Gaussian float label (applied in-kernel) or none")
        ctx.set_materialize_grads(False)
        ctx.sem_shape = None if semantic_feature is None else tuple(semantic_feature.shape)
        ctx.save_for_backward(colors_precomp, semantic_feature, means3D, scales, rotations, cov3Ds_precomp,
                              radii, sh, geom, binning, img, alpha,
                              label if isinstance(label, torch.Tensor) else None,
                              opacities if raw_params else None)
        ctx.mark_non_differentiable(radii)
        return color, radii, feature_map, depth, alpha

    @staticmethod
    def backward(ctx, grad_color, grad_radii, grad_out_feature, grad_depth, grad_alpha):
        rs0 = ctx.rs0
        views, projs, cpos, pp, tx, ty, windows = ctx.cams
        (colors_precomp, semantic_feature, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geom,
         binning, img, alpha, label, raw_opacities) = ctx.saved_tensors
        cx, cy = [p[0] for p in pp], [p[1] for p in pp]
        # Q2 in reference mode, per camera (see _RasterizeGaussians.backward)
        cam4 = (tx, ty, cx, cy) if ctx.compat == "reference" else (cx, cy, tx, ty)
        fuse = (label is not None and label.dim() == 1 and label.numel() == means3D.size(0)
                and label.dtype in _FUSABLE_LABEL_DTYPES)
        grads = _C.rasterize_gaussians_batch_backward(
            rs0.bg, means3D, radii, colors_precomp, semantic_feature, scales, rotations, rs0.scale_modifier,
            cov3Ds_precomp, views, projs, *cam4, grad_color, grad_out_feature, grad_depth, grad_alpha, sh,
            rs0.sh_degree, cpos, geom, ctx.num_instances, binning, img, alpha, rs0.debug, compat=ctx.compat,
            grad_mask=label if fuse else None, densify=ctx.densify_out, opacity=raw_opacities,
            activate=ctx.raw_params, windows=windows, out=ctx.grad_into, scratch=ctx.scratch,
            scratch_zeroed=ctx.scratch_zeroed)
        ctx.scratch_zeroed = False  # a second backward (retain_graph) finds it written
        (grad_means2D, grad_colors_precomp, grad_semantic_feature, grad_opacities, grad_means3D,
         grad_cov3Ds_precomp, grad_sh, grad_scales, grad_rotations) = grads
        if ctx.sem_shape is not None:
            grad_semantic_feature = grad_semantic_feature.reshape(ctx.sem_shape)
        else:
            grad_semantic_feature = None
        if label is not None and not fuse:
            if ctx.raw_params:
                raise RuntimeError("raw_params=True needs a per-Gaussian fp32 label (or none): the mask is "
                                   "applied in-kernel before the activations' backward")
            lab = label.unsqueeze(1)
            grad_means3D = grad_means3D * lab
            grad_sh = grad_sh * lab[..., None]
            grad_colors_precomp = grad_colors_precomp * lab
            grad_opacities = grad_opacities * lab
            grad_scales = grad_scales * lab
            grad_rotations = grad_rotations * lab
            grad_cov3Ds_precomp = grad_cov3Ds_precomp * lab
        grads = (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_semantic_feature,
                 grad_opacities, grad_scales, grad_rotations, grad_cov3Ds_precomp, None, None, None, None, None,
                 None, None, None)
        # gradients written into caller-owned destinations: autograd gets None
        taken = [False] * len(grads)
        for k in (ctx.grad_into or {}):
            taken[_GRAD_SLOT[k]] = True
        return tuple(g if (need and not t) else None for g, need, t in zip(grads, ctx.needs_input_grad, taken))


# backward_buffers' gradient name -> _RasterizeGaussiansBatch.forward argument slot
_GRAD_SLOT = dict(dmeans3D=0, dmeans2D=1, dsh=2, dcolors=3, dsem=4, dopacity=5, dscales=6, drot=7, dcov3D=8)
# GaussianRasterizer argument name -> backward_buffers' gradient name
_GRAD_NAME = dict(means3D="dmeans3D", means2D="dmeans2D", shs="dsh", colors_precomp="dcolors",
                  semantic_feature="dsem", opacities="dopacity", scales="dscales", rotations="drot",
                  cov3D_precomp="dcov3D")


def _grad_destinations(grad_into, semantic_feature):
    """{argument name: tensor} -> backward_batch's {gradient name: tensor}."""
    if not grad_into:
        return None
    out = {}
    for k, t in grad_into.items():
        if k not in _GRAD_NAME:
            raise ValueError(f"grad_into: unknown argument '{k}' (one of {sorted(_GRAD_NAME)})")
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"grad_into['{k}'] must be a tensor")
        out[_GRAD_NAME[k]] = t
    return out


def rasterize_gaussians_batch(means3D, means2D, sh, colors_precomp, semantic_feature, opacities, scales,
                              rotations, cov3Ds_precomp, settings_list, label=None, densify_out=None,
                              raw_params=False, feature_ready=None, plan_state=None, grad_into=None, walk_order=None):
    """rasterize_gaussians over a list of camera settings; outputs [C, ...]
    (color, radii, feature_map, depth, alpha).  `densify_out`: optional
    (accum, denom, max_radius) fp32 [P] tensors the backward fills with the
    cameras' densification statistics (GradientSink.densify_stats).
    `raw_params`: opacities / scales / rotations are the raw parameters of
    helpers.py:98-107 (logit_opacities, log_scales, unnorm_rotations); the
    kernels apply sigmoid / exp / normalize and return their gradients.
    `feature_ready`: a recorded torch.cuda.Event the blend waits for before it
    reads semantic_feature (an overlapped optimizer update of the features on
    another stream; gs_gaussians.feature_ready).  `plan_state`: a
    _C.BinningPlan for the sync-free forward (gs_forward_batch).
    `grad_into`: {argument name: tensor} -- the backward WRITES those
    arguments' camera-summed gradients into the given tensors (e.g. a
    gradient bucket's views, distributed.ShardedAdam.grad_views) and hands
    autograd None for them, so no gradient tensor is allocated, accumulated
    or copied into a bucket; gradients reaching those tensors through other
    autograd paths are not added.  `walk_order`: the binning passes' walk
    order (_C.spatial_order; outputs do not depend on it)."""
    cams = settings_list if isinstance(settings_list, _BatchCameras) else _BatchCameras(list(settings_list))
    return _RasterizeGaussiansBatch.apply(means3D, means2D, sh, colors_precomp, semantic_feature, opacities,
                                          scales, rotations, cov3Ds_precomp, cams, label, densify_out,
                                          bool(raw_params), feature_ready, plan_state, grad_into, walk_order)


class GaussianRasterizerBatch(nn.Module):
    """GaussianRasterizer for a batch of cameras of one image size (the
    cameras of one multi-camera training step): the same keyword call and
    caller-generation arity dispatch, outputs stacked [C, ...], gradients
    summed over the cameras.  `track_densify=True` keeps the cameras'
    densification statistics of the last backward in `densify_stats`
    (the reference's accumulate_mean2d_gradient / max_2D_radius inputs,
    external.py:136-140, train.py:288-290; see GradientSink).  The cameras'
    matrices are stacked once at construction: build a new rasterizer when
    they change (as the reference builds its settings per camera).

    `raw_params=True` takes the Dynamic3DGaussians raw parameters as
    opacities / scales / rotations (logit_opacities, log_scales,
    unnorm_rotations: helpers.py:98-107 params2rendervar) and applies the
    activations -- sigmoid, exp, F.normalize -- inside the preprocess kernels,
    forward and backward (GS_FLAG_ACTIVATE): the same step without the ~20
    elementwise launches of the activations and their autograd backward.

    `sync_free=True` (the default): the forward does not wait for the host
    between the plan and the render stages (gs_forward_batch, ABI 11): the
    binning buffer is sized from the previous call's list lengths (a
    _C.BinningPlan kept in `self.plan`) and the headers are read after every
    stage is enqueued; a call whose lists outgrow it is rendered again with
    the exact lengths.  Outputs and gradients are bit-identical to
    sync_free=False (the reference's two-phase order).

    `spatial_order`: True -- the binning passes walk the Gaussians in 3-D
    Morton order of their means (gs_gaussians.walk_order, ABI 12), so each
    binning workgroup's slice is compact on every camera's screen and its
    per-tile key runs are long; "auto" (the default) -- only when the
    previous call's lists outgrow the bucket pass's LDS staging (large
    scenes, e.g. BASELINE configs[4]); False -- id order.  Outputs are
    bit-identical either way (every tile list is sorted by its unique
    (depth bits, id) keys)."""

    def __init__(self, settings_list, track_densify=False, raw_params=False, sync_free=True, spatial_order="auto",
                 order_refresh=256):
        super().__init__()
        self.settings_list = list(settings_list)
        self.plan = _C.BinningPlan() if sync_free else None
        if spatial_order not in (True, False, "auto"):
            raise ValueError("spatial_order: True, False or 'auto'")
        self.spatial_order = spatial_order
        self.order_refresh = max(1, int(order_refresh))
        self._walk, self._walk_calls = None, 0
        self._cams = _BatchCameras(self.settings_list)
        if track_densify and self._cams.windows is not None:
            raise ValueError("densification statistics need whole-image cameras: a tile window counts a "
                             "Gaussian seen by its camera once per window (gs_camera tile_*)")
        self.track_densify = track_densify
        self.raw_params = bool(raw_params)
        self.densify_stats = None

    # The bucket pass's blocks (gs_common.h TB_BLOCKS per camera) stage their
    # keys in LDS when they fit: cap = (159 KiB - 8 B x tiles) / 10 B per key
    # (launch_tile_bucket, gs_tiles.hip); past it every key is stored where its
    # slot lands, and only then does a spatially coherent walk pay (adjacent
    # lanes' keys in consecutive slots: configs[4] bucket 0.75 -> 0.48 ms; at
    # the bench scene, staged, the walk's rect gathers cost more than it saves).
    _TB_BLOCKS, _TB_BINS = 128, 16384

    def _walk_wanted(self):
        if self.spatial_order != "auto":
            return bool(self.spatial_order)
        ni = self.plan.num_instances if self.plan is not None else None
        if not ni:
            return False
        rs = self._cams.rs0
        tiles = ((rs.image_width + 15) // 16) * ((rs.image_height + 15) // 16)
        cap = (159 * 1024 - 8 * min(self._TB_BINS, tiles)) // 10
        return max(ni) / self._TB_BLOCKS > cap

    def _walk_order(self, means3D):
        """The binning passes' walk: with spatial_order=True (or "auto" once
        the previous call's lists outgrow the bucket pass's LDS staging) the
        Gaussians in 3-D Morton order of their means (_C.spatial_order),
        recomputed when P changes and every `order_refresh` calls (the means
        move while they train; a stale order is only less coherent, never
        wrong); else None (id order)."""
        if not self._walk_wanted() or not means3D.is_cuda or means3D.size(0) == 0:
            return None
        if (self._walk is None or self._walk.numel() != means3D.size(0)
                or self._walk_calls % self.order_refresh == 0):
            self._walk = _C.spatial_order(means3D)
        self._walk_calls += 1
        return self._walk

    def forward(self, means3D, means2D, opacities=None, shs=None, semantic_feature=None, colors_precomp=None,
                scales=None, rotations=None, cov3D_precomp=None, label=_UNSET, feature_ready=None,
                grad_into=None):
        """The GaussianRasterizer call; `feature_ready` (keyword, optional): a
        recorded torch.cuda.Event the blend waits for before reading
        semantic_feature (gs_gaussians.feature_ready).  `grad_into` (keyword,
        optional): {argument name: tensor} destinations the backward writes
        those gradients into (rasterize_gaussians_batch)."""
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or '
                            'precomputed 3D covariance!')
        shs = torch.Tensor([]) if shs is None else shs
        colors_precomp = torch.Tensor([]) if colors_precomp is None else colors_precomp
        scales = torch.Tensor([]) if scales is None else scales
        rotations = torch.Tensor([]) if rotations is None else rotations
        cov3D_precomp = torch.Tensor([]) if cov3D_precomp is None else cov3D_precomp
        has_label = label is not _UNSET
        lab = label if (has_label and isinstance(label, torch.Tensor)) else None
        dens = None
        if self.track_densify:
            P = means3D.size(0)
            dens = tuple(torch.zeros(P, dtype=torch.float32, device=means3D.device) for _ in range(3))
            self.densify_stats = {"means2D_gradient_accum": dens[0], "denom": dens[1], "max_2D_radius": dens[2]}
        color, radii, feature_map, depth, alpha = rasterize_gaussians_batch(
            means3D, means2D, shs, colors_precomp, semantic_feature, opacities, scales, rotations,
            cov3D_precomp, self._cams, lab, dens, self.raw_params, feature_ready, self.plan, grad_into,
            self._walk_order(means3D))
        has_sem = semantic_feature is not None
        if has_label and has_sem:      # G3
            return color, radii, feature_map, depth, alpha
        if has_label:                  # G2
            return color, radii, depth, alpha
        if has_sem:                    # G4
            return color, feature_map, radii, depth
        return color, radii, depth     # G1
