#!/usr/bin/env python3
"""Measured parity errors of the HIP rasterizer against the CPU oracle (GPU).

For each configuration: the forward images' max |diff|, the fraction of
pixels within 1e-5 (colour, depth, features), PSNR, and per gradient tensor
the relative L2 difference GPU vs oracle next to the oracle's own fp32
summation-order envelope (oracle vs oracle with a permuted pixel order).
One JSON line per (config, compat).  The numbers behind the tolerances in
tests/test_gpu_parity.py and DESIGN.md section 5.

    python tools/parity_errors.py [--full]   # --full adds the 800x800 configs
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests import _harness as H  # noqa: E402
from tests.test_gpu_parity import GRAD_NAMES  # noqa: E402

CONFIGS = [dict(), dict(F=32), dict(F=8, use_sh=True, sh_degree=3), dict(F=16, use_cov=True),
           dict(F=64, W=80, H=48), dict(F=32, bg=(0.3, 0.1, 0.7)), dict(F=32, cx=30.0, cy=60.0),
           dict(P=20000, F=32, W=256, H=192)]
FULL = [dict(P=100_000, F=0, W=800, H=800), dict(P=300_000, F=32, W=800, H=800, scale_mult=1.0)]


def measure(kw, compat):
    inp = H.scene(**kw)
    F = kw.get("F", 0)
    g = H.gpu_forward(inp, compat)
    o = H.oracle_forward(inp, compat)
    out = dict(cfg=kw, compat=compat, L=int(o[0]), L_equal=bool(g[0] == o[0]))
    for name, a, b in (("color", g[1], o[1]), ("depth", g[3], o[3]), ("feature", g[2], o[2])):
        a = a.cpu().numpy()
        if b is None or np.size(b) == 0:
            continue
        d = np.abs(a - b)
        out[name] = dict(max=float(d.max()), within_1e5=float(np.mean(d <= 1e-5)), psnr=H.psnr(a, b))
    grads = H.upstream_grads(inp["image_height"], inp["image_width"], F)
    gb = H.gpu_backward(inp, g, grads, compat)
    ob = H.oracle_backward(inp, o, grads, compat)
    W, Hh = inp["image_width"], inp["image_height"]
    perm = np.random.default_rng(5).permutation(W * Hh).astype(np.uint32)
    pb = H.oracle_backward(inp, o, grads, compat, pixel_order=perm)
    rel = {}
    for name, a, b, c in zip(GRAD_NAMES, gb, ob, pb):
        if b.size and np.any(b):
            rel[name] = dict(gpu=H.rel_l2(a, b), envelope=H.rel_l2(c, b))
    out["grad_rel_l2"] = rel
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    args = ap.parse_args()
    cfgs = CONFIGS + (FULL if args.full else [])
    for kw in cfgs:
        for compat in ("reference", "fixed"):
            print(json.dumps(measure(kw, compat)), flush=True)


if __name__ == "__main__":
    main()
