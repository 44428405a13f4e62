#!/usr/bin/env python3
"""Neighbour losses, forward + backward per training step: the HIP kernels
(dynamic3dgaussians_amd.neighbor) against the reference's PyTorch block
(oracle/neighbor.py torch_reference, the op-for-op restatement of
train.py:253-273) on the same device.  Synthetic graph of the reference's
shape (N foreground Gaussians, K = 20 neighbours drawn from a local window of
a shuffled-free ordering, so gathers have realistic locality).  JSON lines.

    python tools/neighbor_bench.py --n 150000 --k 20 --reps 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import neighbor as NB  # noqa: E402
from oracle import neighbor as ON  # noqa: E402


def state(N, K, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    pts = torch.rand(N, 3, device=dev, generator=g)
    off = torch.randint(1, 64, (N, K), device=dev, generator=g)
    nbr = (torch.arange(N, device=dev)[:, None] + off) % N
    prev_rot = torch.nn.functional.normalize(torch.randn(N, 4, device=dev, generator=g), dim=1)
    inv = prev_rot.clone()
    inv[:, 1:] = -inv[:, 1:]
    v = {"neighbor_indices": nbr.long().contiguous(),
         "neighbor_weight": torch.rand(N, K, device=dev, generator=g),
         "neighbor_dist": torch.rand(N, K, device=dev, generator=g) * 0.05,
         "prev_inv_rot_fg": inv.contiguous(),
         "prev_offset": (pts[nbr] - pts[:, None]).contiguous()}
    rot = torch.nn.functional.normalize(prev_rot + 0.05 * torch.randn(N, 4, device=dev, generator=g), dim=1)
    return pts + 0.01, rot, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=150000)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--hip-only", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    pts, rot, v = state(a.n, a.k, dev)
    p = pts.clone().requires_grad_(True)
    r = rot.clone().requires_grad_(True)

    def step(fn):
        out = fn(p, r, v)
        (0.4 * out[0] + 0.4 * out[1] + 0.2 * out[2]).backward()

    impls = [("hip", NB.neighbor_losses), ("torch_reference", ON.torch_reference)]
    for name, fn in impls[:1] if a.hip_only else impls:
        step(fn)
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(a.reps):
            step(fn)
        s1.record()
        torch.cuda.synchronize()
        ms = s0.elapsed_time(s1) / a.reps
        print(json.dumps({"impl": name, "ms_fwd_bwd": round(ms, 4), "N": a.n, "K": a.k, "reps": a.reps}),
              flush=True)


if __name__ == "__main__":
    main()
