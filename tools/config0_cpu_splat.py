#!/usr/bin/env python3
"""BASELINE.json configs[0]: 10k Gaussians, SH degree 0, one 256x256 camera.
Times the naive pure-PyTorch CPU splat (oracle/torch_splat.py: dense
float64 forward + autograd backward) and the single-threaded C oracle on the
host cores, and the HIP rasterizer (fwd + bwd through the drop-in
GaussianRasterizer) on the GPU when one is present; reports the images'
PSNR between the three.  One JSON line.

    python tools/config0_cpu_splat.py [--threads N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import torch_splat as TS  # noqa: E402
from tests import _harness as H  # noqa: E402


def psnr(a, b):
    mse = float(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2))
    return float("inf") if mse == 0 else 10 * np.log10(1.0 / mse)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
    ap.add_argument("--gaussians", type=int, default=10000)
    ap.add_argument("--size", type=int, default=256)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    inp = H.scene(P=a.gaussians, F=0, W=a.size, H=a.size, seed=0, use_sh=True, sh_degree=0)
    grads = H.upstream_grads(a.size, a.size, 0, alpha_grad=False)
    out = {"config": f"{a.gaussians // 1000}k Gaussians, SH degree 0, 1 camera {a.size}x{a.size}",
           "torch_threads": a.threads}
    # naive PyTorch CPU splat, forward + autograd backward
    d64 = lambda t: t.double().clone().requires_grad_(True)  # noqa: E731
    t0 = time.perf_counter()
    m3, op, sc, rot, sh = (d64(inp[k]) for k in ("means3D", "opacity", "scales", "rotations", "sh"))
    col = TS.sh_colors(m3, sh, 0, inp["campos"])
    color, depth, _, _ = TS.render(m3, col, op, sc, rot, inp["viewmatrix"].double(), inp["projmatrix"].double(),
                                   inp["tan_fovx"], inp["tan_fovy"], inp["c_x"], inp["c_y"], a.size, a.size,
                                   inp["bg"].double())
    t1 = time.perf_counter()
    ((color * grads[0].double()).sum() + (depth * grads[2].double()).sum()).backward()
    t2 = time.perf_counter()
    out["torch_cpu_splat_s"] = {"fwd": round(t1 - t0, 3), "bwd": round(t2 - t1, 3)}
    out["torch_cpu_splat_mpix_s"] = round(a.size * a.size / 1e6 / (t2 - t0), 4)
    # C oracle (single thread), fixed numerics like the splat
    t0 = time.perf_counter()
    o = H.oracle_forward(inp, "fixed")
    t1 = time.perf_counter()
    H.oracle_backward(inp, o, grads, "fixed")
    t2 = time.perf_counter()
    out["c_oracle_s"] = {"fwd": round(t1 - t0, 3), "bwd": round(t2 - t1, 3)}
    out["c_oracle_mpix_s"] = round(a.size * a.size / 1e6 / (t2 - t0), 4)
    out["psnr_splat_vs_oracle_db"] = round(psnr(color.detach().numpy(), o[1]), 2)
    if torch.cuda.is_available():
        g = H.gpu_forward(inp, "fixed")
        for _ in range(3):
            H.gpu_backward(inp, H.gpu_forward(inp, "fixed"), grads, "fixed")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        reps = 20
        for _ in range(reps):
            H.gpu_backward(inp, H.gpu_forward(inp, "fixed"), grads, "fixed")
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        out["hip_ms_fwd_bwd_incl_host_copies"] = round(dt * 1e3, 3)
        out["psnr_hip_vs_oracle_db"] = round(psnr(g[1].cpu().numpy(), o[1]), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
