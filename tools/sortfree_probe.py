#!/usr/bin/env python3
"""Feasibility probe of sort-free binning: the
per-camera depth sort it needs before an order-stable bucket pass, timed on
the bench scene.

Sort-free binning = sort every camera's visible Gaussians once by (depth
bits, index), walk them in that order in the plan and bucket passes with an
order-stable slot claim, and drop the per-tile sort.  Its cost floor is the
depth sort plus today's bucket walk.  This probe times, on the GPU, the
library's stable LSD radix sort (gs_sort_pairs: 8-bit digits, 3 kernels per
pass) over the 27 cameras' (camera << 32 | depth bits, id) pairs -- 27 x P
keys, the culled ones keyed past every depth -- against the product's
bucket + tile-sort stages of the same scene (bench.py's stage times).

    python tools/sortfree_probe.py [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dynamic3dgaussians_amd import _C, _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    args = argparse.Namespace(gaussians=300_000, features=32, seed=0, compat="reference")
    dev = torch.device("cuda", 0)
    params, label = bench.make_params(args, dev)
    rig = camera_rig(27, 800, 800)
    sets = bench.make_settings(rig, dev, "reference")
    L = _lib.load()
    P = args.gaussians
    keys = []
    with torch.no_grad():
        rv = bench.params2rendervar(params, label)
        for c, s in enumerate(sets):
            o = _C.rasterize_gaussians_batch(
                s.bg, rv["means3D"], rv["colors_precomp"], None, rv["opacities"], rv["scales"], rv["rotations"],
                1.0, torch.Tensor([]), s.viewmatrix.reshape(1, 16), s.projmatrix.reshape(1, 16), [s.c_x], [s.c_y],
                [s.tanfovx], [s.tanfovy], 800, 800, torch.Tensor([]), 0, s.campos.reshape(1, 3), False, False,
                compat="reference")
            radii = o[5][0]
            depth = torch.zeros(P, device=dev)
            _lib.check(L.gs_debug_export(P, 800, 800, o[6].data_ptr(), None, o[8].data_ptr(), 0, None,
                                         depth.data_ptr(), None, None, None, None, None, None,
                                         torch.cuda.current_stream(dev).cuda_stream), "export")
            bits = depth.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            bits = torch.where(radii > 0, bits, torch.full_like(bits, 0xFFFFFFFF))
            keys.append((c << 32) | bits)
    k0 = torch.cat(keys).contiguous()
    n = k0.numel()
    v0 = torch.arange(P, device=dev, dtype=torch.int32).repeat(27).contiguous()
    scratch = torch.empty(L.gs_sort_scratch_bytes(n), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    times = []
    for r in range(a.reps + 3):
        kk, vv = k0.clone(), v0.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _lib.check(L.gs_sort_pairs(n, kk.data_ptr(), vv.data_ptr(), 37, scratch.data_ptr(), st), "sort")
        e1.record()
        e1.synchronize()
        if r >= 3:
            times.append(e0.elapsed_time(e1))
    ok = bool(torch.all(kk[1:] >= kk[:-1]).item())
    visible = int((k0 & 0xFFFFFFFF != 0xFFFFFFFF).sum().item())
    times.sort()
    print(json.dumps({"keys": n, "visible_keys": visible, "end_bit": 37, "passes": 5,
                      "depth_sort_ms_median": round(times[len(times) // 2], 4),
                      "depth_sort_ms_min": round(times[0], 4), "sorted": ok}))


if __name__ == "__main__":
    main()
