"""Fused colour + segmentation rendering.

The reference training step rasterizes every camera twice: once for colour
(`train.py:145`, `dyn_train.py:244`) and once more with
`colors_precomp = params['seg_colors']` for the segmentation image
(`train.py:246-249`).  Both passes share the geometry, so here the seg
colours ride along as 3 extra feature channels of the colour pass -- one
projection, one binning, one blend -- and come back as the seg image.

Channel layout.  Without caller features the seg colours are the feature
channels themselves (F = 3, padded to the 4-wide kernel): in reference
numerics features 0..2 receive the background exactly like colour
(`CR/forward.cu:398-404`, Q4: bg[ch] for ch < 3) and the blend adds
w * feature with the same fp32 fma chain as colour, so the fused seg image is
bit-identical to the reference's second render
(`tests/test_gpu_fused.py::test_fused_colour_seg_matches_two_passes`).  With
the caller's F semantic channels the layout is [features (F), seg (3), ones
(1)]: the caller's channels keep their indices, hence the Q4 background of
channels 0..2 exactly as the plain colour render's feature map has it, and at
F = 32 the pass is the F = 36 instantiation (32 matrix-core channels + a
4-channel VALU tail: seg and ones) instead of a padded 64.  The ones channel
renders sum(w) = 1 - T, which gives the seg channels their background term
T * bg in reference numerics (where the alpha output is never written, Q1).
In this layout the seg image is NOT bit-identical to the reference's second
render when the background is nonzero: the second render adds T_final * bg
with T_final the blend's running product, the fused pass (1 - sum w) * bg,
equal in exact arithmetic and within fp32 rounding of each other -- the
1e-5 bar of tests/test_gpu_fused.py::test_fused_colour_seg_f32_against_oracle
(bit-identity holds only at bg = 0 and in the F = 3 layout above).

Gradients.  dL/dseg_colors is the same per-Gaussian sum of w * dL/dseg as
the second pass's dL/dcolors_precomp.  Geometry: in reference numerics the
feature term of dL/dalpha is dead (Q5, `CR/backward.cu:596-612`), so the fused
pass's geometry and means2D gradients are exactly the colour render's -- what
the reference wants for densification ("Gradient only accum from colour
render", `train.py:245`) -- while two passes would add the seg image's
geometry term (the reference's seg loss is disabled, `train.py:250`, so its
training sees no difference).  In compat="fixed" features feed dL/dalpha, so
the fused pass gives the full two-pass gradient, with means2D carrying the sum
of both renders' screen-space gradients; the background is added to seg as
(1 - alpha) * bg there, since fixed-mode features get no background.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from ._C import get_default_compat as _default_compat
from .rasterizer import GaussianRasterizer


def render_colour_and_seg(raster_settings, means3D: torch.Tensor, means2D: torch.Tensor,
                          opacities: torch.Tensor, seg_colors: torch.Tensor,
                          colors_precomp: Optional[torch.Tensor] = None,
                          shs: Optional[torch.Tensor] = None, scales=None, rotations=None,
                          cov3D_precomp=None, semantic_feature: Optional[torch.Tensor] = None,
                          label=None) -> Tuple[torch.Tensor, ...]:
    """One rasterization for the colour image AND the seg image.

    Returns (colour[3,H,W], radii[P], depth[1,H,W], seg[3,H,W]) -- plus the
    caller's own semantic feature map [F,H,W] as a fifth element when
    `semantic_feature` is given (the seg channels are appended after it).
    """
    if seg_colors.dim() != 2 or seg_colors.size(1) != 3:
        raise ValueError("seg_colors must be [P, 3]")
    P = means3D.size(0)
    F_user = 0 if semantic_feature is None else semantic_feature.reshape(P, -1).size(1)
    if F_user:
        # [caller's features, seg, ones]: the caller's channels keep their
        # indices (and Q4 background); the ones channel renders 1 - T
        ones = torch.ones(P, 1, device=seg_colors.device, dtype=seg_colors.dtype)
        feats = torch.cat([semantic_feature.reshape(P, -1), seg_colors, ones], dim=1)
    else:
        feats = seg_colors  # channels 0..2: the reference's background (Q4)
    ras = GaussianRasterizer(raster_settings)
    lab = label if label is not None else torch.ones(means3D.size(0), device=means3D.device)
    color, radii, feature_map, depth, alpha = ras(
        means3D=means3D, means2D=means2D, opacities=opacities, shs=shs, colors_precomp=colors_precomp,
        semantic_feature=feats, scales=scales, rotations=rotations, cov3D_precomp=cov3D_precomp, label=lab)
    compat = getattr(raster_settings, "compat", None) or _default_compat()
    bg = raster_settings.bg.reshape(3, 1, 1)
    if F_user:
        seg = feature_map[F_user:F_user + 3]
        # T * bg: T = 1 - alpha (fixed numerics write alpha) or 1 - sum(w)
        cover = alpha if compat != "reference" else feature_map[F_user + 3:F_user + 4]
        seg = seg + (1.0 - cover) * bg
        return color, radii, depth, seg, feature_map[:F_user]
    seg = feature_map[:3]
    if compat != "reference":
        seg = seg + (1.0 - alpha) * bg
    return color, radii, depth, seg
