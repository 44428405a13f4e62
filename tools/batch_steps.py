#!/usr/bin/env python3
"""Batch forward + backward of the bench scene (300k Gaussians, 27 cameras
800x800, F = 32) through GaussianRasterizerBatch, a few times -- the program
rocprofv3 --pmc runs to count the bench's kernels per launch (one launch = all
27 cameras).

    rocprofv3 --pmc FETCH_SIZE -- python3 tools/batch_steps.py --reps 2

Every rep is one launch per stage of the same work: the forward is the
two-phase plan -> render (sync_free=False; the sync-free forward's first call
renders every camera empty and retries, which would add a launch of no work
to the counts -- tools/pmc_*.py refuse such files).  --sync-free runs the
sync-free forward after one warm call, for timing and stamps only (the warm
call's launches would be counted too).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import (GaussianRasterizationSettings,  # noqa: E402
                                               GaussianRasterizerBatch)
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300_000)
    ap.add_argument("--cams", type=int, default=27)
    ap.add_argument("--features", type=int, default=32)
    ap.add_argument("--size", type=int, default=800)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--sync-free", action="store_true", help="the sync-free forward (one warm call first)")
    ap.add_argument("--stamps", action="store_true", help="read the stamps build's wave-lifetime shares")
    ap.add_argument("--dump-stamps", default="", help="with --stamps: save the raw per-wave stamps (npz)")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    W = H = a.size
    g = make_gaussians(a.gaussians, F=a.features, seed=0, device=dev)
    bg = torch.zeros(3, device=dev)
    sets = [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y, bg=bg,
        viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference") for c in camera_rig(a.cams, W, H)]
    ras = GaussianRasterizerBatch(sets, sync_free=a.sync_free)
    gen = torch.Generator(device=dev).manual_seed(1)
    C = a.cams
    up = [torch.randn(C, 3, H, W, device=dev, generator=gen), torch.randn(C, 1, H, W, device=dev, generator=gen)]
    if a.features:
        up.append(torch.randn(C, a.features, H, W, device=dev, generator=gen))
    leaves = {k: g[k].clone().requires_grad_(True) for k in ("means3D", "colors", "opacities", "scales", "rotations")}
    label = torch.ones(a.gaussians, device=dev)
    stamps = None
    if a.stamps:  # one 4 x u64 record per blend wave of the last launch (gs_stamps_set)
        import ctypes
        L = _lib.load(auto_build=False)
        T = ((W + 15) // 16) * ((H + 15) // 16)
        nf = T * 4 * C
        buf = torch.zeros(2 * nf * 8, dtype=torch.int64, device=dev)
        L.gs_stamps_set.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
        assert L.gs_stamps_set(ctypes.c_void_p(buf.data_ptr()), nf) == 0
        stamps = (buf, nf)
    for rep in range(a.reps + (1 if a.sync_free else 0)):
        kw = dict(means3D=leaves["means3D"], means2D=torch.zeros(a.gaussians, 3, device=dev),
                  opacities=leaves["opacities"], colors_precomp=leaves["colors"], scales=leaves["scales"],
                  rotations=leaves["rotations"], label=label)
        if a.features:
            im, radius, feat, depth, _ = ras(semantic_feature=g["semantic_feature"], **kw)
            torch.autograd.backward([im, depth, feat], up)
        else:
            im, radius, depth, _ = ras(**kw)
            torch.autograd.backward([im, depth], up)
    torch.cuda.synchronize()
    if ras.plan is not None:
        # the counted reps after the warm call rendered every camera once
        print(f"sync-free retries: {ras.plan.retries} over {ras.plan.calls} calls", flush=True)
        print("num_instances", list(ras.plan.num_instances), flush=True)
        assert ras.plan.retries == 0, "a counted rep was rendered twice (binning capacity retry)"
    if a.stamps:
        import json
        st = stamps[0].cpu().numpy().reshape(-1, 8).astype(np.float64)
        nf = stamps[1]
        if a.dump_stamps:  # rows = waves in block order (forward first, then backward), 8 fields each
            np.savez_compressed(a.dump_stamps, stamps=stamps[0].cpu().numpy().reshape(-1, 8), n_fwd=nf, cams=C)
        out = {}
        for name, v in (("render_fwd", st[:nf]), ("render_bwd", st[nf:])):
            v = v[v[:, 3] > 0]
            tot = v[:, 3].sum()
            out[name] = {"start": round(v[:, 0].sum() / tot, 4), "loop": round((v[:, 1] - v[:, 0]).sum() / tot, 4),
                         "tail_issue": round((v[:, 2] - v[:, 1]).sum() / tot, 4),
                         "drain": round((v[:, 3] - v[:, 2]).sum() / tot, 4), "waves": int(len(v)),
                         "ticks_per_wave": round(float(tot / max(len(v), 1)))}
            if (v[:, 6] > 0).all():  # absolute real-time clock (100 MHz): the launch's waves in flight
                t0, t1 = v[:, 6], v[:, 7]
                span = t1.max() - t0.min()
                ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
                ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
                live = np.cumsum(ev[:, 1])
                dt = np.diff(ev[:, 0], append=ev[-1, 0])
                peak = live.max()
                low = live < 0.5 * peak
                # the launch's tail: from the last time the chip was at >= half its peak to the end
                last_full = ev[np.nonzero(~low)[0].max(), 0]
                out[name]["timeline"] = {
                    "span_us": round(span / 100.0, 1), "peak_waves": int(peak),
                    "mean_waves_in_flight": round(float((live * dt).sum() / span), 1),
                    "below_half_peak_us": round(float(dt[low].sum()) / 100.0, 1),
                    "tail_us": round(float(t1.max() - last_full) / 100.0, 1),
                    "ramp_us": round(float(ev[np.nonzero(~low)[0].min(), 0] - t0.min()) / 100.0, 1),
                    "longest_wave_us": round(float((t1 - t0).max()) / 100.0, 1),
                    "mean_wave_us": round(float((t1 - t0).mean()) / 100.0, 1)}
            if (v[:, 4:6] > 0).any():  # GS_STAMPS_FINE: backward prologue stages after full waits
                d = np.diff(np.concatenate([np.zeros((len(v), 1)), v[:, 4:8]], axis=1), axis=1)
                out[name]["prologue"] = {k: round(float(d[:, i].sum() / tot), 4) for i, k in
                                         enumerate(["to_record", "pixel_loads", "operands", "first_chunk"])}
        print(json.dumps(out), flush=True)
    print("batch steps done", flush=True)


if __name__ == "__main__":
    main()
