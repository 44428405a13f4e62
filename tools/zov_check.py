#!/usr/bin/env python3
"""Step-level check of the overlapped ZeRO-1 exchange (distributed.ShardedStep
with overlap: geometry in line, features reduce-scattered / updated /
all-gathered on a side stream behind the next step, double-buffered) over N
ranks -- the gloo rehearsal of the "zov" mode that once landed far above the
noise floor after several Adam steps (profiles/r05c/overlap_first).  Instead of
comparing parameters after training (where Adam turns float-atomic order noise
into +-lr moves), every step is checked on its own:

  1. each rank's gradients of step k equal a replay's autograd gradients from
     the parameters step k READ (relative L2 <= 1e-6 per tensor: the
     backward's float-atomic reorder noise), and its forward outputs equal
     the replay's bit for bit;
  2. the parameters step k read equal an in-line Adam replay (no exchange, no
     side stream) over the ranks' summed captured gradients, bit for bit --
     the exchange summed exactly what the ranks computed, the update used
     the right buffer, and the blend read the features after the update;
  3. every rank ends with the same parameters.

The side stream's update is delayed by a spin kernel each step, so a missing
wait shows up as a stale read or a clobbered buffer.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29561 tools/zov_check.py          # gloo, both ranks on GPU 0

Rank 0 prints one JSON line ({"ok": ...}); the exit status is 0 iff every
check holds on every rank.  GS_ZOV_BACKEND=nccl runs it over RCCL (one GPU
per rank).
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dynamic3dgaussians_amd import _lib  # noqa: E402
from dynamic3dgaussians_amd.camera import camera_rig  # noqa: E402
from dynamic3dgaussians_amd.distributed import ShardedAdam, ShardedStep  # noqa: E402
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizerBatch  # noqa: E402
from dynamic3dgaussians_amd.scene import make_gaussians  # noqa: E402

LRS = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
       "log_scales": 1e-3, "semantic_feature": 1e-3}  # train.py:119-135 (+ the features)
ARG = {"means3D": "means3D", "rgb_colors": "colors_precomp", "unnorm_rotations": "rotations",
       "logit_opacities": "opacities", "log_scales": "scales", "semantic_feature": "semantic_feature"}
GEO = [k for k in LRS if k != "semantic_feature"]


def main():
    # the JSON line is the only output on stdout (gloo / RCCL print banners
    # there): fd 1 goes to stderr for the run, the line to the saved fd
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend = os.environ.get("GS_ZOV_BACKEND", "gloo")
    dev = torch.device("cuda", 0 if backend == "gloo" else int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    _lib.load()
    P, F, C, W, H, steps = int(os.environ.get("GS_ZOV_P", "12000")), 32, 3, 192, 160, 3
    rig = camera_rig(C * world, W, H, seed=3)
    sets = [GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
        bg=torch.zeros(3, device=dev), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(dev),
        projmatrix=torch.from_numpy(c.projmatrix.copy()).to(dev), sh_degree=0,
        campos=torch.from_numpy(c.campos.copy()).to(dev)) for c in rig[rank::world]]
    gen = torch.Generator(device=dev).manual_seed(11 + rank)
    ups = [torch.randn(C, 3, H, W, device=dev, generator=gen), torch.randn(C, 1, H, W, device=dev, generator=gen),
           torch.randn(C, F, H, W, device=dev, generator=gen)]
    label = torch.ones(P, device=dev)
    g = make_gaussians(P, F=F, seed=4, device=dev)
    init = {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
            "logit_opacities": torch.logit(g["opacities"]), "log_scales": torch.log(g["scales"]),
            "semantic_feature": g["semantic_feature"]}
    init = {k: v.detach().clone().contiguous() for k, v in init.items()}
    params = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
    zs = ShardedStep(params, LRS, eps=1e-15, overlap=True)  # the process group's rank / world, collectives on
    upd = zs.feat.update

    def slow_update(*a, **k):  # the side stream's update starts ~2 ms late
        torch.cuda._sleep(int(4.8e6))
        return upd(*a, **k)
    zs.feat.update = slow_update

    ras = GaussianRasterizerBatch(sets, raw_params=True)
    cap = []
    for _ in range(steps):
        zs.begin()
        geo = {k: params[k].detach().clone() for k in GEO}
        im, _, feat, depth, _ = ras(means2D=torch.zeros_like(params["means3D"]), label=label,
                                    feature_ready=zs.feature_ready, grad_into=zs.grad_into(ARG),
                                    **{ARG[k]: p for k, p in params.items()})
        fread = params["semantic_feature"].detach().clone()  # behind the (gated) blend on the main stream
        outs = (im.detach().clone(), feat.detach().clone(), depth.detach().clone())
        torch.autograd.backward([im, depth, feat], ups)
        grads = {k: v.clone() for k, v in zs.grad_into().items()}
        cap.append((dict(geo, semantic_feature=fread), outs, grads))
        zs.finish()
    zs.drain()
    torch.cuda.synchronize()
    final = {k: v.detach().clone() for k, v in params.items()}

    report = {"rank": rank, "world": world, "backend": backend, "grad_rel": [], "fwd_equal": [], "read_equal": []}
    ok = True
    # 1) this rank's gradients vs a replay from what the step read
    for read, outs, grads in cap:
        leaves = {k: v.clone().requires_grad_(True) for k, v in read.items()}
        rr = GaussianRasterizerBatch(sets, raw_params=True, sync_free=False)
        im, _, feat, depth, _ = rr(means2D=torch.zeros_like(leaves["means3D"]), label=label,
                                   **{ARG[k]: p for k, p in leaves.items()})
        same = all(bool(torch.equal(a, b.detach())) for a, b in zip(outs, (im, feat, depth)))
        torch.autograd.backward([im, depth, feat], ups)
        rel = {}
        for k in LRS:
            a, b = grads[k].double(), leaves[k].grad.double()
            rel[k] = float((a - b).norm() / b.norm().clamp_min(1e-30))
        report["grad_rel"].append(rel)
        report["fwd_equal"].append(same)
        ok &= same and max(rel.values()) <= 1e-6
    # 2) in-line replay of Adam over the ranks' summed gradients
    rp = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
    ropt = ShardedAdam(rp, LRS, rank=0, world=1, eps=1e-15, collectives=False)
    for read, _, grads in cap:
        eq = {k: bool(torch.equal(rp[k].detach(), read[k])) for k in LRS}
        report["read_equal"].append(eq)
        ok &= all(eq.values())
        for k, v in ropt.grad_views(0).items():
            s = grads[k].clone()
            dist.all_reduce(s)  # the sum the exchange should have formed (2 ranks: order-free)
            v.copy_(s)
        ropt.step(0)
    report["final_equal_replay"] = {k: bool(torch.equal(rp[k].detach(), final[k])) for k in LRS}
    ok &= all(report["final_equal_replay"].values())
    # 3) the ranks agree
    flat = torch.cat([final[k].reshape(-1) for k in LRS])
    mx, mn = flat.clone(), flat.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    report["ranks_agree"] = bool(torch.equal(mx, mn))
    ok &= report["ranks_agree"]
    flag = torch.tensor([0.0 if ok else 1.0], device=dev)
    dist.all_reduce(flag)
    all_ok = float(flag.item()) == 0.0
    reports = [None] * world
    dist.all_gather_object(reports, report)
    if rank == 0:
        with os.fdopen(line_fd, "w") as out:
            out.write(json.dumps({"ok": all_ok, "steps": steps, "gaussians": P, "cams_per_rank": C,
                                  "ranks": reports}) + "\n")
    dist.destroy_process_group()
    sys.exit(0 if all_ok else 1)


if __name__ == "__main__":
    main()
