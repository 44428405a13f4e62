"""dynamic3dgaussians_amd -- MI355X-native (gfx950, HIP) differentiable 3D-Gaussian
rasterizer, a drop-in for Dynamic3DGaussians' `diff_gaussian_rasterization`.

Layout:
  csrc/           hand-written HIP kernels + the C ABI (include/gsplat_hip.h)
  build.py        hipcc build of lib/libgsplat_hip.so (in-tree)
  _lib.py         ctypes binding of the C ABI (fails loudly; no CPU fallback)
  _C.py           positional mirror of the reference pybind module `_C`
  rasterizer.py   autograd boundary (GaussianRasterizer & friends)
  camera.py       helpers.setup_camera restatement + synthetic camera rig
  scene.py        synthetic scenes for tests and the benchmark
  distributed.py  camera-sharded data parallelism with one RCCL all-reduce
"""
from .rasterizer import (GaussianRasterizationSettings, GaussianRasterizer, GradientSink,  # noqa: F401
                         _RasterizeGaussians, rasterize_gaussians)
from ._C import set_default_compat, get_default_compat  # noqa: F401

__version__ = "0.1.0"
