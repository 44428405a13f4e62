#!/usr/bin/env python3
"""BASELINE.json configs[3] shape: a sequence of timesteps of the 27-camera
rig, cameras sharded over the ranks (camera c on rank c mod N), through
dynamic3dgaussians_amd.timesteps.TimestepDriver -- the per-timestep
constant-velocity initialisation, a new gradient bucket per timestep, one
SUM + one MAX all-reduce and FusedAdam per iteration, L1 loss against
synthetic targets (the rig's renders of the scene with jittered colours).

    python tools/timesteps_run.py --timesteps 4 --iters 5
    torchrun --nproc-per-node N --master-addr 127.0.0.1 tools/timesteps_run.py ...

Rank 0 prints one JSON line: rendered Mpix/s over the whole run (all
timesteps, iterations and cameras; max elapsed over ranks), ms per
iteration, the per-timestep initialisation time and the loss trajectory.
GS_BENCH_BACKEND=gloo GS_BENCH_SHARE_GPU=1 rehearse N ranks on one GPU.

BASELINE configs[3] at its stated length (150 timesteps):

    python tools/timesteps_run.py --timesteps 150 --iters 2 --features 32 --neighbors --per-timestep

--features F: the semantic channels in the parameters, rendered through the
G3 call and fitted with an L1 term (the overlapped feature exchange of the
sharded step applies); --neighbors: after timestep 0 the foreground k-NN
graph (initialize_post_first_timestep, train.py:316-341, HIP k-NN) and from
timestep 1 on the rigidity / rotation / isometry losses (HIP kernels) with
dyn_train.py's weights 0.4 / 0.4 / 0.2 (dyn_train.py:313); --sharded: the
driver's ShardedStep even at one rank; --per-timestep: every timestep timed
on its own (device-synchronised) with its peak device memory.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.distributed import shard_cameras  # noqa: E402
from dynamic3dgaussians_amd.optim import FusedAdam  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings  # noqa: E402
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402
from dynamic3dgaussians_amd.timesteps import TimestepDriver, batch_renderer, params2rendervar  # noqa: E402

LRS = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
       "log_scales": 1e-3}  # train.py:119-135


def _or_zero(x, params):
    """An extra loss that does not apply yet (timestep 0) as a zero that
    still reaches the graph (so the sum with the image loss is a tensor)."""
    return x if x is not None else params["means3D"].sum() * 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=300_000)
    ap.add_argument("--cams-total", type=int, default=27)
    ap.add_argument("--size", type=int, default=800)
    ap.add_argument("--timesteps", type=int, default=4)
    ap.add_argument("--iters", type=int, default=5, help="iterations per timestep")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--features", type=int, default=0)
    ap.add_argument("--neighbors", action="store_true")
    ap.add_argument("--sharded", action="store_true")
    ap.add_argument("--per-timestep", action="store_true")
    ap.add_argument("--out", default="", help="also write the JSON to this file")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("GS_BENCH_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("GS_BENCH_SHARE_GPU") == "1" else local
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    _lib.load()
    W = H = a.size
    rig = camera_rig(a.cams_total, W, H, seed=a.seed)
    settings = [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.zeros(3, device=dev), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(dev), compat="reference") for c in rig]
    g = make_gaussians(a.gaussians, F=a.features, seed=a.seed, device=dev)
    base = {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
            "logit_opacities": torch.logit(g["opacities"]), "log_scales": torch.log(g["scales"])}
    lrs = dict(LRS)
    if a.features:
        base["semantic_feature"] = g["semantic_feature"]
        lrs["semantic_feature"] = 1e-3
    render = batch_renderer(settings)
    mine = shard_cameras(a.cams_total, rank, world)
    with torch.no_grad():
        tg, _ = render(params2rendervar(base), mine)  # this rank's targets [C_rank, 3, H, W] (+ features)
        tg = tuple(x.detach().clone() for x in tg) if isinstance(tg, tuple) else tg.detach().clone()
    params = {k: torch.nn.Parameter(v.clone()) for k, v in base.items()}
    gen = torch.Generator(device=dev).manual_seed(a.seed + 5)
    with torch.no_grad():
        params["rgb_colors"].add_(0.2 * torch.randn(params["rgb_colors"].shape, device=dev, generator=gen))
        if a.features:
            params["semantic_feature"].add_(0.2 * torch.randn(params["semantic_feature"].shape, device=dev,
                                                              generator=gen))
    opt = FusedAdam([{"params": [params[k]], "name": k, "lr": lr} for k, lr in lrs.items()], lr=0.0, eps=1e-15)
    extra, post_first = None, None
    if a.neighbors:
        from dynamic3dgaussians_amd.neighbor import neighbor_losses
        from dynamic3dgaussians_amd.timesteps import initialize_post_first_timestep

        def extra(pr, variables, rv, t):  # dyn_train.py:313 weights (train.py:253-273 terms)
            if t == 0 or "neighbor_indices" not in variables:
                return None
            rot = torch.nn.functional.normalize(pr["unnorm_rotations"])
            rigid, rot_l, iso = neighbor_losses(pr["means3D"], rot, variables)
            return 0.4 * rigid + 0.4 * rot_l + 0.2 * iso

        def post_first(pr, variables, optimizer):
            return initialize_post_first_timestep(pr, variables, optimizer, num_knn=20)
    drv = TimestepDriver(params, {}, opt, a.cams_total, render, rank=rank, world=world,
                         targets_sharded=True,  # tg holds this rank's cameras only
                         extra_loss=(lambda pr, v, rv, t: _or_zero(extra(pr, v, rv, t), pr)) if extra else None,
                         sharded=True if a.sharded else None)
    # warm-up: one step of timestep 0 (kernel load, allocator), not timed
    drv.step(tg)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per_ts = []
    if a.per_timestep:  # drv.run's loop, each timestep synchronised and measured on its own
        losses = []
        for t in range(a.timesteps):
            torch.cuda.reset_peak_memory_stats(dev)
            ta = time.perf_counter()
            losses.append(drv.timestep(t, a.iters, tg))
            if t == 0:
                if post_first is not None:
                    drv.variables = post_first(drv.params, drv.variables, drv.optimizer)
                elif "prev_pts" not in drv.variables:
                    drv.variables["prev_pts"] = drv.params["means3D"].detach()
                    drv.variables["prev_rot"] = torch.nn.functional.normalize(
                        drv.params["unnorm_rotations"]).detach()
            torch.cuda.synchronize()
            per_ts.append({"t": t, "ms": round((time.perf_counter() - ta) * 1e3, 3),
                           "loss": round(sum(losses[-1]) / a.iters, 6),
                           "peak_mib": round(torch.cuda.max_memory_allocated(dev) / 2 ** 20, 1),
                           "alloc_mib": round(torch.cuda.memory_allocated(dev) / 2 ** 20, 1)})
        drv.sync_optimizer()
    else:
        losses = drv.run(a.timesteps, lambda t: a.iters, lambda t: tg, post_first=post_first)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ls = torch.tensor([sum(x) for x in losses], device=dev, dtype=torch.float64)
        dist.all_reduce(ls)
        loss_per_t = [float(x) / a.iters for x in ls.tolist()]
    else:
        loss_per_t = [sum(x) / a.iters for x in losses]
    n_iter = a.timesteps * a.iters
    if rank == 0:
        line = {
            "metric": "rendered Mpix/s fwd+bwd over a timestep sequence (configs[3] shape)",
            "value": round(n_iter * a.cams_total * W * H / elapsed / 1e6, 3), "unit": "Mpix/s",
            "n_ranks": world, "backend": backend if world > 1 else None,
            "ms_per_iteration": round(elapsed / n_iter * 1e3, 3), "timesteps": a.timesteps, "iters": a.iters,
            "cams_total": a.cams_total, "cams_per_rank": [len(shard_cameras(a.cams_total, r, world))
                                                          for r in range(world)],
            "gaussians": a.gaussians, "size": [W, H], "mean_loss_per_timestep": [round(x, 6) for x in loss_per_t],
            "features": a.features, "neighbors": a.neighbors,
            "optimizer_step": ("distributed.ShardedStep" + (" (features overlapped)" if drv.zs.overlap else "")
                               if drv.zs is not None else "GradBucket all-reduce + FusedAdam"),
            "data": "synthetic (targets: the rig's renders of the scene before a colour jitter)"}
        if per_ts:
            ms = [x["ms"] for x in per_ts[2:]] or [0.0]
            pk = [x["peak_mib"] for x in per_ts[2:]] or [0.0]
            line["per_timestep"] = per_ts
            line["after_t1"] = {"ms_min": min(ms), "ms_median": sorted(ms)[len(ms) // 2], "ms_max": max(ms),
                                "ms_first10_mean": round(sum(ms[:10]) / max(len(ms[:10]), 1), 3),
                                "ms_last10_mean": round(sum(ms[-10:]) / max(len(ms[-10:]), 1), 3),
                                "peak_mib_min": min(pk), "peak_mib_max": max(pk)}
        print(json.dumps(line), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(line, f, indent=1)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
