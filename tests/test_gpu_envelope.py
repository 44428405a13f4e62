"""The GPU backward against the reference algorithm's own fp32 noise.

The reference sums every per-Gaussian gradient with float atomicAdd in
arrival order (CR/backward.cu:586-649), so two runs of it differ by fp32
summation order alone.  The oracle restates that: with a permuted pixel
visiting order (oracle.rasterize_gaussians_backward(pixel_order=...)) its
per-Gaussian sums are added in a different order, and the relative L2 spread
between the two oracle runs is the envelope.  The HIP backward -- whose
feature, colour and geometry sums are matrix-core contractions of 3-piece
bf16 splits (gs_render.hip) -- must stay within 10x that envelope (measured
<= 6.5x; the round-2 two-piece split measured 10-20x, profiles/
r03_parity_errors_split2.jsonl) and within SURVEY 8(c)'s 1e-4."""
import numpy as np
import pytest

from tests import _harness as H
from tests.test_gpu_parity import GRAD_NAMES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [dict(F=32), dict(F=32, bg=(0.3, 0.1, 0.7)), dict(F=8, use_sh=True, sh_degree=3),
                                dict(P=20000, F=32, W=256, H=192)])
def test_backward_within_fp32_summation_envelope(kw):
    inp = H.scene(**kw)
    g = H.gpu_forward(inp)
    o = H.oracle_forward(inp)
    grads = H.upstream_grads(inp["image_height"], inp["image_width"], kw.get("F", 0))
    gb = H.gpu_backward(inp, g, grads)
    ob = H.oracle_backward(inp, o, grads)
    perm = np.random.default_rng(5).permutation(inp["image_width"] * inp["image_height"]).astype(np.uint32)
    pb = H.oracle_backward(inp, o, grads, pixel_order=perm)
    report = {}
    for name, a, b, c in zip(GRAD_NAMES, gb, ob, pb):
        if not (b.size and np.any(b)):
            continue
        err, env = H.rel_l2(a, b), H.rel_l2(c, b)
        report[name] = (err, env)
        assert env > 0, name  # the permutation did reorder the sums
        assert err <= max(10.0 * env, 2e-6), (name, err, env)
        assert err <= 1e-4, (name, err)
    print({k: f"{e:.1e}/{v:.1e}" for k, (e, v) in report.items()})
