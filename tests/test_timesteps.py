"""The per-timestep driver (dynamic3dgaussians_amd/timesteps.py) on the CPU:
the reference's timestep initialisation and optimizer-state surgery
(train.py:294-314, external.py:143-155) restated independently here, and
the camera-sharded loop over two gloo ranks against one process rendering
the whole rig.  The renders come from the dense PyTorch splat
(oracle/torch_splat.py, test infrastructure) standing in for the HIP batch
renderer, which needs a GPU (tests/test_gpu_timesteps.py runs that one)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.distributed import ShardedAdam, ShardedStep
from dynamic3dgaussians_amd.scene import camera_tensors, make_gaussians
from dynamic3dgaussians_amd.timesteps import (TimestepDriver, initialize_post_first_timestep,
                                              initialize_per_timestep, update_params_and_optimizer)
from oracle import torch_splat as TS

N_CAMS, W, H, P = 4, 32, 32, 80
LRS = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
       "log_scales": 1e-3}


def _params(seed=0):
    g = make_gaussians(P, seed=seed, extent=0.6)
    seg = torch.zeros(P, 3)
    seg[: P // 2, 0] = 1.0  # first half foreground
    return {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
            "logit_opacities": torch.logit(g["opacities"].clamp(0.05, 0.9)), "log_scales": torch.log(g["scales"] * 6),
            "seg_colors": seg}


def _optimizer(params, cls=torch.optim.Adam):
    return cls([{"params": [params[k]], "name": k, "lr": lr} for k, lr in LRS.items()], lr=0.0, eps=1e-15)


def _leaf(params):
    return {k: torch.nn.Parameter(v.clone()) if k != "seg_colors" else v.clone() for k, v in params.items()}


# ------------------------------------------------------------ initialisation

def test_update_params_and_optimizer_resets_moments_keeps_step():
    params = _leaf(_params())
    opt = _optimizer(params)
    for p in (params[k] for k in LRS):
        p.grad = torch.randn_like(p)
    opt.step()
    old = params["means3D"]
    step_before = opt.state[old]["step"].clone()
    new = torch.randn_like(old)
    update_params_and_optimizer({"means3D": new}, params, opt)
    p = params["means3D"]
    assert p is not old and isinstance(p, torch.nn.Parameter) and p.requires_grad
    group = [g for g in opt.param_groups if g["name"] == "means3D"][0]
    assert group["params"][0] is p
    assert old not in opt.state
    st = opt.state[p]
    assert torch.equal(st["exp_avg"], torch.zeros_like(new)) and torch.equal(st["exp_avg_sq"], torch.zeros_like(new))
    assert torch.equal(st["step"], step_before)
    assert torch.equal(p.data, new)
    # the untouched groups keep their state
    assert opt.state[params["rgb_colors"]]["exp_avg"].abs().sum() > 0


def test_initialize_per_timestep_constant_velocity():
    params = _leaf(_params())
    opt = _optimizer(params)
    for p in (params[k] for k in LRS):
        p.grad = torch.randn_like(p)
    opt.step()
    prev_pts = params["means3D"].detach().clone() - 0.01
    prev_rot = torch.nn.functional.normalize(params["unnorm_rotations"].detach().clone() + 0.05)
    variables = {"prev_pts": prev_pts, "prev_rot": prev_rot,
                 "neighbor_indices": torch.randint(0, P // 2, (P // 2, 5))}
    pts0 = params["means3D"].detach().clone()
    rot0 = torch.nn.functional.normalize(params["unnorm_rotations"].detach().clone())
    col0 = params["rgb_colors"].detach().clone()
    params, variables = initialize_per_timestep(params, variables, opt)
    # train.py:297-298
    np.testing.assert_allclose(params["means3D"].detach(), pts0 + (pts0 - prev_pts), rtol=0, atol=1e-7)
    want_rot = torch.nn.functional.normalize(rot0 + (rot0 - prev_rot))
    np.testing.assert_allclose(params["unnorm_rotations"].detach(), want_rot, rtol=0, atol=1e-7)
    # train.py:300-309
    fg = params["seg_colors"][:, 0] > 0.5
    inv = rot0[fg].clone()
    inv[:, 1:] *= -1
    assert torch.equal(variables["prev_inv_rot_fg"], inv)
    fg_pts = pts0[fg]
    assert torch.equal(variables["prev_offset"], fg_pts[variables["neighbor_indices"]] - fg_pts[:, None])
    assert torch.equal(variables["prev_pts"], pts0) and torch.equal(variables["prev_rot"], rot0)
    assert torch.equal(variables["prev_col"], col0)
    # the two replaced groups start from zero moments
    assert opt.state[params["means3D"]]["exp_avg"].abs().sum() == 0


def test_initialize_post_first_timestep_graph():
    params = _leaf(_params())
    opt = _optimizer(params)

    def brute_knn(pts, k):  # squared distances, excluding the point itself (o3d_knn semantics)
        d = ((pts[:, None] - pts[None]) ** 2).sum(-1)
        d.fill_diagonal_(float("inf"))
        sq, idx = torch.topk(d, k, largest=False)
        return sq, idx

    v = initialize_post_first_timestep(params, {}, opt, num_knn=4, knn_fn=brute_knn)
    fg = params["seg_colors"][:, 0] > 0.5
    sq, idx = brute_knn(params["means3D"][fg].detach(), 4)
    assert torch.equal(v["neighbor_indices"], idx)
    np.testing.assert_allclose(v["neighbor_weight"], torch.exp(-2000 * sq), rtol=1e-6)
    np.testing.assert_allclose(v["neighbor_dist"], torch.sqrt(sq), rtol=1e-6)
    assert torch.equal(v["init_bg_pts"], params["means3D"][~fg].detach())
    for g in opt.param_groups:
        assert (g["lr"] == 0.0) == (g["name"] in ("logit_opacities", "log_scales"))


# ------------------------------------------------------------ sharded loop

def _rig():
    return [camera_tensors(c) for c in camera_rig(N_CAMS, W, H, radius=2.0)]


def _splat_render(rig):
    """render(rendervar, cams) through the dense PyTorch splat (float32)."""
    def render(rv, cams):
        ims = []
        for c in cams:
            ct = rig[c]
            col, _, _, _ = TS.render(rv["means3D"], rv["colors_precomp"], rv["opacities"], rv["scales"],
                                     rv["rotations"], ct["viewmatrix"], ct["projmatrix"], ct["tanfovx"],
                                     ct["tanfovy"], ct["c_x"], ct["c_y"], W, H, ct["bg"])
            ims.append(col)
        return torch.stack(ims), None
    return render


def _targets(t):
    return torch.rand(N_CAMS, 3, H, W, generator=torch.Generator().manual_seed(100 + t))


class _RecordingAdam(torch.optim.Adam):
    """torch.optim.Adam that records the gradients it is handed."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.seen = []

    def step(self, closure=None):
        self.seen.append({g["name"]: g["params"][0].grad.detach().clone() for g in self.param_groups
                          if g["params"][0].grad is not None})
        return super().step(closure)


def _toy_densify(params, variables, optimizer, i):
    """At iteration 1: remove Gaussian 3 and clone Gaussian 0, with the
    reference's optimizer-state surgery (external.py:157-205 restated:
    rows dropped from / zero rows appended to the Adam moments, new
    Parameters, the statistics tensors rebound)."""
    if i != 1:
        return params, variables
    trainable = [g["name"] for g in optimizer.param_groups]
    keep = torch.ones(params["means3D"].shape[0], dtype=torch.bool)
    keep[3] = False
    for k in list(params):
        if k in trainable:
            g = [x for x in optimizer.param_groups if x["name"] == k][0]
            st = optimizer.state.pop(g["params"][0], None)
            p = torch.nn.Parameter(g["params"][0][keep].detach().requires_grad_(True))
            if st is not None:
                st["exp_avg"], st["exp_avg_sq"] = st["exp_avg"][keep], st["exp_avg_sq"][keep]
                optimizer.state[p] = st
            g["params"][0] = p
            params[k] = p
        else:
            params[k] = params[k][keep]
    for k in ("means2D_gradient_accum", "denom", "max_2D_radius"):
        variables[k] = variables[k][keep]
    for k in list(params):
        v = params[k][:1].detach()
        if k in trainable:
            g = [x for x in optimizer.param_groups if x["name"] == k][0]
            st = optimizer.state.pop(g["params"][0], None)
            p = torch.nn.Parameter(torch.cat((g["params"][0].detach(), v), 0).requires_grad_(True))
            if st is not None:
                st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(v)), 0)
                st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(v)), 0)
                optimizer.state[p] = st
            g["params"][0] = p
            params[k] = p
        else:
            params[k] = torch.cat((params[k], v), 0)
    for k in ("means2D_gradient_accum", "denom", "max_2D_radius"):
        variables[k] = torch.cat((variables[k], torch.zeros(1)), 0)
    return params, variables


def _run(rank, world, densify=None):
    torch.manual_seed(0)
    params = _leaf(_params())
    opt = _optimizer(params, _RecordingAdam)
    drv = TimestepDriver(params, {}, opt, N_CAMS, _splat_render(_rig()), rank=rank, world=world, densify=densify)
    losses = drv.run(2, lambda t: 2 if densify is None else 3, _targets)
    return ({k: v.detach().clone() for k, v in drv.params.items()}, opt.seen, losses)


def _worker(rank, world, port, q, densify=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params, grads, losses = _run(rank, world, _toy_densify if densify else None)
        # numpy through the queue (tensors would be shared by file descriptor,
        # which dies with the process)
        q.put((rank, ({k: v.numpy() for k, v in params.items()},
                      [{k: v.numpy() for k, v in g.items()} for g in grads], losses)))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("densify", [False, True])
def test_driver_two_ranks_match_whole_rig(densify):
    """densify=True: a densification at timestep 0 replaces every tensor;
    the driver builds a new bucket at the next step, the replaced
    Parameters skip that iteration's optimizer step (no .grad), as in the
    reference, and the ranks stay identical."""
    single_params, single_grads, single_losses = _run(0, 1, _toy_densify if densify else None)
    if densify:
        assert single_params["means3D"].shape[0] == P  # one removed, one cloned
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, densify)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (p0, g0, l0), (p1, g1, l1) = res[0], res[1]
    # the ranks hold identical parameters after every all-reduced step
    for k in p0:
        assert np.array_equal(p0[k], p1[k]), k
    # 2 timesteps x 2 (3) iterations, each step's all-reduced gradient = the
    # whole rig's gradient in one process (fp32 summation order)
    assert len(g0) == len(single_grads) == (6 if densify else 4)
    for gs, gd in zip(single_grads, g0):
        for k in gs:
            a, b = gs[k].numpy(), gd[k]
            rel = float(np.linalg.norm(a - b) / max(float(np.linalg.norm(a)), 1e-30))
            assert rel < 1e-5, (k, rel)
    # the ranks' loss shares add up to the rig's loss
    for ls, a, b in zip(single_losses, l0, l1):
        np.testing.assert_allclose(np.add(a, b), ls, rtol=1e-5)
    # timestep 1 started from the constant-velocity initialisation
    for k in single_params:
        np.testing.assert_allclose(p0[k], single_params[k], rtol=0, atol=5e-4)


def test_driver_loss_decreases_on_fit():
    """Fitting the rig's renders of a perturbed scene: the timestep-0 loss
    falls over the iterations (the loop trains)."""
    torch.manual_seed(0)
    rig = _rig()
    render = _splat_render(rig)
    target_params = _params(seed=0)
    with torch.no_grad():
        from dynamic3dgaussians_amd.timesteps import params2rendervar
        tg, _ = render(params2rendervar(target_params), list(range(N_CAMS)))
    params = _leaf(_params(seed=0))
    with torch.no_grad():
        params["rgb_colors"].add_(0.2 * torch.randn_like(params["rgb_colors"])).clamp_(0, 1)
    opt = _optimizer(params)
    for g in opt.param_groups:
        g["lr"] = g["lr"] * 4
    drv = TimestepDriver(params, {}, opt, N_CAMS, render)
    losses = drv.timestep(0, 8, tg)
    assert losses[-1] < 0.8 * losses[0], losses


# ------------------------------------------------------------ sharded optimizer step

class _TorchAdamSlices(ShardedAdam):
    """ShardedAdam with its update restated as torch.optim.Adam's own
    single-tensor arithmetic (the CPU path of torch/optim/adam.py: lerp_,
    mul_/addcmul_, (sqrt / bc2_sqrt) + eps, addcdiv_), so a sharded driver
    on the CPU is held bit-for-bit to the plain driver's torch.optim.Adam.
    (On the GPU the update is the HIP kernel, held to FusedAdam bit-for-bit
    by tests/test_gpu_sharded_adam.py.)"""

    def _apply(self, k, entries):
        for p, g, m, v, step_size, bc2s in entries:
            m.lerp_(g, 1 - self.beta1)
            v.mul_(self.beta2).addcmul_(g, g, value=1 - self.beta2)
            p.addcdiv_(m, (v.sqrt() / bc2s).add_(self.eps), value=step_size)


def _sharded_factory(params, lr, rank, world, group):
    return ShardedStep(params, lr, rank=rank, world=world, group=group, eps=1e-15, overlap=False,
                       adam_cls=_TorchAdamSlices)


def _run_driver(rank, world, sharded, densify=None, steps=(2, 2)):
    """A 2-timestep run; a parameter reached by no loss ('idle', skipped by
    Adam on both paths) and one reached only by rank 0's extra loss
    ('rank0_only': updated on every rank from the union of the ranks' reach);
    lr = 0 for log_scales after timestep 0 (initialize_post_first_timestep's
    params_to_fix) -- the learning rates come from the optimizer each step."""
    torch.manual_seed(0)
    params = _leaf(_params())
    lrs = dict(LRS)
    if densify is None:  # (the toy densification handles per-Gaussian tensors only)
        params["idle"] = torch.nn.Parameter(torch.ones(5, 2))
        params["rank0_only"] = torch.nn.Parameter(torch.full((3,), 0.5))
        lrs.update(idle=1e-2, rank0_only=1e-2)
    opt = torch.optim.Adam([{"params": [params[k]], "name": k, "lr": lr} for k, lr in lrs.items()], lr=0.0,
                           eps=1e-15)

    def extra(pr, variables, rv, t):
        out = 0.01 * (pr["means3D"] ** 2).mean()
        if rank == 0 and "rank0_only" in pr:
            out = out + (pr["rank0_only"] ** 2).sum()
        return out

    def post_first(pr, variables, optimizer):
        for g in optimizer.param_groups:
            if g["name"] == "log_scales":
                g["lr"] = 0.0
        variables["prev_pts"] = pr["means3D"].detach()
        variables["prev_rot"] = torch.nn.functional.normalize(pr["unnorm_rotations"]).detach()
        return variables

    drv = TimestepDriver(params, {}, opt, N_CAMS, _splat_render(_rig()), rank=rank, world=world, densify=densify,
                         extra_loss=extra, sharded=sharded)
    losses = drv.run(steps[0], lambda t: steps[1], _targets, post_first=post_first)
    state = {k: {n: v.detach().clone() for n, v in opt.state[p].items() if torch.is_tensor(v)}
             for k, p in drv.params.items() if isinstance(p, torch.nn.Parameter) and opt.state.get(p)}
    return ({k: v.detach().clone() for k, v in drv.params.items()},
            {k: drv.variables[k].clone() for k in ("means2D_gradient_accum", "denom", "max_2D_radius")},
            state, losses, drv.zs is not None)


def _sharded_worker(rank, world, port, q, densify):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for sharded in (False, _sharded_factory):
            pr, var, st, losses, used = _run_driver(rank, world, sharded, _toy_densify if densify else None)
            out.append(({k: v.numpy() for k, v in pr.items()}, {k: v.numpy() for k, v in var.items()},
                        {k: {n: v.numpy() for n, v in d.items()} for k, d in st.items()}, losses, used))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _check_same(a, b, exact, what):
    if exact:
        np.testing.assert_array_equal(a, b, err_msg=what)
    else:  # three ranks' sums: the collectives may add in different orders
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7, err_msg=what)


def test_sharded_driver_one_rank_equals_plain_driver():
    plain = _run_driver(0, 1, False)
    shard = _run_driver(0, 1, _sharded_factory)
    assert not plain[4] and shard[4]
    for k in plain[0]:
        _check_same(shard[0][k].numpy(), plain[0][k].numpy(), True, k)
    for k in plain[1]:
        _check_same(shard[1][k].numpy(), plain[1][k].numpy(), True, k)
    # the optimizer holds the sharded step's state at the end of run()
    assert set(shard[2]) == set(plain[2]) and "idle" not in plain[2]
    for k in plain[2]:
        for n in ("step", "exp_avg", "exp_avg_sq"):
            _check_same(shard[2][k][n].numpy(), plain[2][k][n].numpy(), True, f"{k}.{n}")


@pytest.mark.parametrize("world,densify", [(2, False), (3, False), (2, True)])
def test_sharded_driver_equals_plain_bucket_driver(world, densify):
    """The driver with distributed.ShardedStep (reduce-scatter, Adam on the
    rank's slice, all-gather; statistics + reach flags in one small
    all-reduce) against the plain GradBucket + torch.optim.Adam driver, both
    over `world` gloo ranks for 2 timesteps x 2 iterations: the per-timestep
    re-initialisation (replace with zeroed moments), the lr change after
    timestep 0, an unreached and a rank-0-only parameter, and (densify=True)
    the plain path through timestep 0's densification before the sharded
    step takes over from the optimizer's state."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, densify)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    exact = world == 2
    for r in range(world):
        (pp, vp, sp, lp, up), (ps, vs, ss, ls, us) = res[r]
        assert not up and us
        for k in pp:
            _check_same(ps[k], pp[k], exact, f"rank {r} {k}")
            np.testing.assert_array_equal(ps[k], res[0][1][0][k])  # every rank holds the same parameters
        if not densify:
            assert not np.array_equal(pp["rank0_only"], np.full(3, 0.5, np.float32))  # updated on every rank
            np.testing.assert_array_equal(pp["idle"], np.ones((5, 2), np.float32))     # never updated
        for k in vp:
            _check_same(vs[k], vp[k], exact, f"rank {r} {k}")
        assert set(ss) == set(sp)
        for k in sp:
            for n in sp[k]:
                _check_same(ss[k][n], sp[k][n], exact, f"rank {r} {k}.{n}")
        np.testing.assert_allclose(np.asarray(ls), np.asarray(lp), rtol=1e-5)
