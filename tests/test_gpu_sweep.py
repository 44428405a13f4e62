"""Seeded sweep of small random configurations: the HIP forward and backward
against the CPU oracle at the tolerances of test_gpu_parity.py (SURVEY.md
8(c)).  Each case draws image size (odd sizes, not multiples of the 16-pixel
tile), scene size and Gaussian extent, scene seed, camera of the 27-camera
rig or an off-centre principal point, feature width (every instantiation:
plain VALU widths, the padded ones, the matrix-core 32/64 and the fused 36),
SH degree or precomputed colours, scale modifier, background and compat mode
from one fixed generator, so the case list is the same on every run.

The reference's own entry points are the same for every case
(CR/rasterizer_impl.cu:195-357 forward, :359-433 backward); the sweep only
varies the inputs the reference's tests and callers vary (train.py:246-249,
external.py calc_psnr inputs, dyn_train.py F = 32)."""
import numpy as np
import pytest

from tests import _harness as H
from tests.test_gpu_parity import GRAD_NAMES, _cmp_forward

pytestmark = pytest.mark.gpu

_FWIDTHS = [0, 3, 5, 8, 16, 20, 32, 35, 36, 64]


def _cases(n=40, seed=2026):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        W = int(rng.integers(17, 200))
        Hh = int(rng.integers(15, 160))
        kw = dict(W=W, H=Hh, P=int(rng.integers(200, 5000)), seed=int(rng.integers(0, 1000)),
                  F=int(rng.choice(_FWIDTHS)), scale_mult=float(rng.uniform(1.0, 6.0)),
                  bg=tuple(float(x) for x in rng.uniform(0.0, 1.0, 3).round(3)))
        if rng.uniform() < 0.3:
            kw.update(cx=float(rng.uniform(0.2, 0.8) * W), cy=float(rng.uniform(0.2, 0.8) * Hh))
        else:
            kw["cam_index"] = int(rng.integers(0, 27))
        if rng.uniform() < 0.35:
            kw.update(use_sh=True, sh_degree=int(rng.integers(0, 4)))
        mod = float(rng.choice([1.0, 1.0, 0.6, 1.4]))
        compat = "fixed" if rng.uniform() < 0.4 else "reference"
        out.append(pytest.param(kw, mod, compat, id=f"case{i}"))
    return out


@pytest.mark.parametrize("kw,mod,compat", _cases())
def test_random_config_forward_backward(kw, mod, compat):
    inp = H.scene(**kw)
    inp["scale_modifier"] = mod
    F = kw["F"]
    g, o = _cmp_forward(inp, compat, F)
    grads = H.upstream_grads(inp["image_height"], inp["image_width"], F, seed=kw["seed"] + 1)
    gb = H.gpu_backward(inp, g, grads, compat)
    ob = H.oracle_backward(inp, o, grads, compat)
    for name, a, b in zip(GRAD_NAMES, gb, ob):
        assert a.shape == b.shape, name
        if b.size == 0 or not np.any(b):
            assert not np.any(a) or np.abs(a).max() < 1e-6, name
            continue
        assert H.rel_l2(a, b) <= 1e-4, (name, H.rel_l2(a, b))
