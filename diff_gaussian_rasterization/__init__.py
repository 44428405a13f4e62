"""Drop-in import name: `from diff_gaussian_rasterization import
GaussianRasterizationSettings, GaussianRasterizer` resolves to the MI355X-native
implementation in dynamic3dgaussians_amd (the reference module is
submodules_fsgs/diff-gaussian-rasterization-confidence/diff_gaussian_rasterization)."""
import sys as _sys

from dynamic3dgaussians_amd import _C  # noqa: F401
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings,  # noqa: F401
                                               GaussianRasterizer, GradientSink, _RasterizeGaussians,
                                               cpu_deep_copy_tuple, rasterize_gaussians)
from dynamic3dgaussians_amd._C import get_default_compat, set_default_compat  # noqa: F401

_sys.modules[__name__ + "._C"] = _C
