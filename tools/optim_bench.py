#!/usr/bin/env python3
"""Optimizer step at the bench scale: torch.optim.Adam (foreach, the
reference's default), torch.optim.Adam(fused=True) and FusedAdam (one HIP
launch; optionally with the densification statistics fused in), on the
reference's parameter groups for P Gaussians (+ F semantic channels).
JSON lines with ms per step and the HBM rate of the 28 B/element update.

    python tools/optim_bench.py --gaussians 300000 --features 32 --reps 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd.optim import FusedAdam, densify_stats  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300000)
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    P, dev = a.gaussians, "cuda"
    shapes = {"means3D": 3, "rgb_colors": 3, "seg_colors": 3, "unnorm_rotations": 4, "logit_opacities": 1,
              "log_scales": 3}
    if a.features:
        shapes["semantic_feature"] = a.features
    lrs = {"means3D": 5e-6, "rgb_colors": 2.5e-5, "seg_colors": 0.0, "unnorm_rotations": 0.0,
           "logit_opacities": 0.05, "log_scales": 0.001, "semantic_feature": 1e-3}
    numel = P * sum(shapes.values())
    g = torch.Generator(device=dev).manual_seed(0)
    radius = torch.randint(0, 30, (P,), device=dev, generator=g).int()

    def make(kind):
        params = {k: torch.nn.Parameter(torch.randn(P, c, device=dev, generator=g)) for k, c in shapes.items()}
        for p in params.values():
            p.grad = torch.randn_like(p)
        groups = [{"params": [v], "name": k, "lr": lrs[k]} for k, v in params.items()]
        if kind == "fused_hip":
            return FusedAdam(groups, lr=0.0, eps=1e-15), params
        return torch.optim.Adam(groups, lr=0.0, eps=1e-15, fused=(kind == "torch_fused")), params

    m2 = torch.zeros(P, 3, device=dev, requires_grad=True)
    m2.grad = torch.randn(P, 3, device=dev, generator=g)
    variables = {"max_2D_radius": torch.zeros(P, device=dev), "means2D_gradient_accum": torch.zeros(P, device=dev),
                 "denom": torch.zeros(P, device=dev), "means2D": m2}

    def ref_stats():  # train.py:288-290 + external.py:136-140
        seen = radius > 0
        variables["max_2D_radius"][seen] = torch.max(radius[seen], variables["max_2D_radius"][seen])
        variables["means2D_gradient_accum"][seen] += torch.norm(m2.grad[seen, :2], dim=-1)
        variables["denom"][seen] += 1

    cases = [("torch_foreach", False), ("torch_fused", False), ("fused_hip", False),
             ("torch_foreach+stats", True), ("fused_hip+stats", True), ("stats_only_hip", True)]
    for name, with_stats in cases:
        kind = name.split("+")[0]
        opt, params = make("fused_hip" if kind == "stats_only_hip" else kind)

        def step():
            if name == "stats_only_hip":
                densify_stats(variables, radius)
            elif name == "fused_hip+stats":
                opt.step(stats=(variables, radius))
            else:
                if with_stats:
                    ref_stats()
                opt.step()

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.reps):
            step()
        s1.record()
        torch.cuda.synchronize()
        ms = s0.elapsed_time(s1) / a.reps
        rec = {"impl": name, "ms_per_step": round(ms, 4), "P": P, "elements": numel}
        if name != "stats_only_hip":
            rec["adam_GBs_at_28B_per_elem"] = round(28.0 * numel / ms / 1e6, 1)
        print(json.dumps(rec), flush=True)
        del opt, params


if __name__ == "__main__":
    main()
