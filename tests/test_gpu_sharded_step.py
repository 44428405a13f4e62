"""distributed.ShardedStep on the GPU: the overlapped ZeRO-1 step -- geometry
reduce-scatter + Adam on the rank's slice + all-gather in line, the features'
exchange and update on a side stream behind the next step, double-buffered
gradients, the next blend gated by `feature_ready` -- checked so that a
stream race cannot hide behind float-atomic noise (VERDICT r05 "next" 1,
ADVICE r05):

* fixed gradients, no rasterizer: the overlapped sequence must equal
  ShardedAdam.step() in line BIT FOR BIT -- every step's feature read (gated
  like the blend) and the final parameters -- with the side stream's work
  delayed by a spin kernel, so a missing wait shows as a stale read or a
  clobbered gradient buffer.  With and without a world-1 RCCL process group
  (the reduce-scatter / all-gather run through RCCL);
* the rasterizer: for 3 steps of the camera batch through the overlapped
  step (side stream delayed), each step's forward outputs equal a replay
  forward from the parameters that step read (bit for bit: no atomics in the
  forward), each step's gradients equal the replay's autograd gradients to
  the float-atomic reorder noise (relative L2 <= 1e-6 per tensor), and the
  parameters each step read equal an in-line Adam replay of the captured
  gradients bit for bit -- so a step that read stale features, or whose
  exchange mixed buffers, fails here whatever Adam does with order noise;
* the training driver (timesteps.TimestepDriver) with sharded=True at a
  world of one takes the overlapped path (features in the parameters, the
  G3 call) and trains like the plain driver.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist

from dynamic3dgaussians_amd.camera import camera_rig
from dynamic3dgaussians_amd.distributed import ShardedAdam, ShardedStep
from dynamic3dgaussians_amd.optim import FusedAdam
from dynamic3dgaussians_amd.rasterizer import GaussianRasterizationSettings, GaussianRasterizerBatch
from dynamic3dgaussians_amd.scene import make_gaussians

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
LRS = {"means3D": 1.6e-4, "rgb_colors": 2.5e-3, "unnorm_rotations": 1e-3, "logit_opacities": 0.05,
       "log_scales": 1e-3, "semantic_feature": 1e-3}
ARG = {"means3D": "means3D", "rgb_colors": "colors_precomp", "unnorm_rotations": "rotations",
       "logit_opacities": "opacities", "log_scales": "scales", "semantic_feature": "semantic_feature"}
GEO = [k for k in LRS if k != "semantic_feature"]


def _raw_params(P, F, seed=0):
    g = make_gaussians(P, F=F, seed=seed, device=DEV)
    p = {"means3D": g["means3D"], "rgb_colors": g["colors"], "unnorm_rotations": g["rotations"],
         "logit_opacities": torch.logit(g["opacities"]), "log_scales": torch.log(g["scales"]),
         "semantic_feature": g["semantic_feature"]}
    return {k: torch.nn.Parameter(v.detach().clone().contiguous()) for k, v in p.items()}


_BURN = {}


def _delay(ms=2.0):
    """Occupy the current stream for about `ms` (the work queued behind it
    starts late: a consumer that does not wait for it reads old data):
    torch's spin kernel, or matrix products where it is missing."""
    try:
        torch.cuda._sleep(int(ms * 2.4e6))
        return
    except (AttributeError, RuntimeError):
        pass
    a = _BURN.get("a")
    if a is None:
        a = _BURN["a"] = torch.randn(2048, 2048, device=DEV)
    for _ in range(max(1, int(ms * 2))):
        a = a @ a * 1e-3


def _slow_side(zs, ms=2.0):
    """Delay the side stream's feature update of every step."""
    upd = zs.feat.update

    def slow(*a, **k):
        _delay(ms)
        return upd(*a, **k)
    zs.feat.update = slow


@pytest.fixture
def rccl_world1():
    """A world-1 RCCL process group (the collectives run through RCCL)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=DEV)
    try:
        yield True
    finally:
        dist.destroy_process_group()


def _grad_seq(params, steps, seed=7):
    gen = torch.Generator(device=DEV).manual_seed(seed)
    return [{k: torch.randn(p.shape, device=DEV, generator=gen) for k, p in params.items()} for _ in range(steps)]


def _overlapped_equals_inline(collectives):
    P, F, steps = 40_000, 32, 6
    grads = _grad_seq(_raw_params(P, F), steps)
    ref = _raw_params(P, F)
    ropt = ShardedAdam(ref, LRS, rank=0, world=1, eps=1e-15, collectives=False)
    want_reads = []
    for g in grads:
        want_reads.append(ref["semantic_feature"].detach().clone())
        for k, v in ropt.grad_views(0).items():
            v.copy_(g[k])
        ropt.step(0)
    params = _raw_params(P, F)
    zs = ShardedStep(params, LRS, rank=0, world=1, eps=1e-15, overlap=True, collectives=collectives)
    assert zs.overlap and zs.feat is not None
    _slow_side(zs)
    main = torch.cuda.current_stream(DEV)
    reads = []
    for g in grads:
        zs.begin()
        ev = zs.feature_ready
        if ev is not None:  # the blend's gate (gs_gaussians.feature_ready)
            main.wait_event(ev)
        reads.append(params["semantic_feature"].detach().clone())
        _delay(0.5)  # the "backward" writes its buffers late
        for k, v in zs.grad_into().items():
            v.copy_(g[k])
        zs.finish()
    zs.drain()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(reads, want_reads)):
        assert torch.equal(a, b), f"step {i}: the features read differ from the in-line run"
    for k in params:
        assert torch.equal(params[k].detach(), ref[k].detach()), k


def test_overlapped_sequence_equals_inline_steps_bit_for_bit():
    _overlapped_equals_inline(collectives=False)


def test_overlapped_sequence_over_rccl_equals_inline_steps(rccl_world1):
    _overlapped_equals_inline(collectives=True)


def _cams(n, W, H):
    out = []
    for c in camera_rig(n, W, H, seed=3):
        out.append(GaussianRasterizationSettings(
            image_height=H, image_width=W, tanfovx=c.tanfovx, tanfovy=c.tanfovy, c_x=c.c_x, c_y=c.c_y,
            bg=torch.zeros(3, device=DEV), viewmatrix=torch.from_numpy(c.viewmatrix.copy()).to(DEV),
            projmatrix=torch.from_numpy(c.projmatrix.copy()).to(DEV), sh_degree=0,
            campos=torch.from_numpy(c.campos.copy()).to(DEV)))
    return out


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _rasterizer_step_chain(collectives):
    P, F, C, W, H, steps = 12_000, 32, 4, 192, 160, 3
    sets = _cams(C, W, H)
    gen = torch.Generator(device=DEV).manual_seed(5)
    ups = [torch.randn(C, 3, H, W, device=DEV, generator=gen), torch.randn(C, 1, H, W, device=DEV, generator=gen),
           torch.randn(C, F, H, W, device=DEV, generator=gen)]
    label = torch.ones(P, device=DEV)
    params = _raw_params(P, F, seed=4)
    init = {k: v.detach().clone() for k, v in params.items()}
    zs = ShardedStep(params, LRS, rank=0, world=1, eps=1e-15, overlap=True, collectives=collectives)
    _slow_side(zs)
    ras = GaussianRasterizerBatch(sets, raw_params=True)
    cap = []
    for _ in range(steps):
        zs.begin()
        geo = {k: params[k].detach().clone() for k in GEO}  # in line: final for this step
        kw = {ARG[k]: p for k, p in params.items()}
        im, _, feat, depth, _ = ras(means2D=torch.zeros_like(params["means3D"]), label=label,
                                    feature_ready=zs.feature_ready, grad_into=zs.grad_into(ARG), **kw)
        # behind the blend on the main stream: the features the blend read
        fread = params["semantic_feature"].detach().clone()
        outs = (im.detach().clone(), feat.detach().clone(), depth.detach().clone())
        torch.autograd.backward([im, depth, feat], ups)
        grads = {k: v.clone() for k, v in zs.grad_into().items()}
        cap.append((dict(geo, semantic_feature=fread), outs, grads))
        zs.finish()
    zs.drain()
    torch.cuda.synchronize()
    final = {k: v.detach().clone() for k, v in params.items()}

    # 1) each step: a replay from the parameters it read (plain autograd,
    # the two-phase forward, no exchange, no side stream)
    for i, (read, outs, grads) in enumerate(cap):
        leaves = {k: v.clone().requires_grad_(True) for k, v in read.items()}
        rr = GaussianRasterizerBatch(sets, raw_params=True, sync_free=False)
        im, _, feat, depth, _ = rr(means2D=torch.zeros_like(leaves["means3D"]), label=label,
                                   **{ARG[k]: p for k, p in leaves.items()})
        for name, a, b in zip(("color", "feature", "depth"), outs, (im, feat, depth)):
            assert torch.equal(a, b.detach()), f"step {i}: forward {name} differs from the replay"
        torch.autograd.backward([im, depth, feat], ups)
        for k in LRS:
            r = _rel(grads[k], leaves[k].grad)
            assert r <= 1e-6, (i, k, r)
    # 2) the parameters each step read = in-line Adam over the captured
    # gradients (deterministic given the gradients: bit for bit)
    rp = {k: torch.nn.Parameter(v.clone()) for k, v in init.items()}
    ropt = ShardedAdam(rp, LRS, rank=0, world=1, eps=1e-15, collectives=False)
    for i, (read, _, grads) in enumerate(cap):
        for k in LRS:
            assert torch.equal(rp[k].detach(), read[k]), f"step {i}: '{k}' read differs from the in-line replay"
        for k, v in ropt.grad_views(0).items():
            v.copy_(grads[k])
        ropt.step(0)
    for k in LRS:
        assert torch.equal(rp[k].detach(), final[k]), k


def test_overlapped_rasterizer_steps_gradients_and_feature_reads():
    _rasterizer_step_chain(collectives=False)


def test_overlapped_rasterizer_steps_over_rccl(rccl_world1):
    _rasterizer_step_chain(collectives=True)


def test_driver_takes_the_overlapped_sharded_step():
    """TimestepDriver(sharded=True) at a world of one with feature channels:
    the overlapped ShardedStep (features behind the next step) against the
    plain driver with FusedAdam, 2 timesteps x 2 iterations.  Both runs carry
    the backward's float-atomic order noise, which Adam's first steps turn
    into +-lr moves of elements whose gradient is ~0, so the bound is on the
    99.9th percentile of |delta| (1e-3 lr) plus Adam's step size for every
    element; the step-level race checks are the tests above."""
    from dynamic3dgaussians_amd.timesteps import TimestepDriver, batch_renderer, params2rendervar
    P, F, C, W, H = 20_000, 32, 4, 160, 128
    sets = _cams(C, W, H)
    base = _raw_params(P, F, seed=6)
    render = batch_renderer(sets)
    with torch.no_grad():
        (tim, tft), _ = render(params2rendervar(base), list(range(C)))
        targets = (tim.detach().clone(), (tft + 0.1).detach().clone())
    runs = {}
    for sharded in (False, True):
        params = {k: torch.nn.Parameter(v.detach().clone()) for k, v in base.items()}
        with torch.no_grad():
            params["rgb_colors"].add_(0.05)
        opt = FusedAdam([{"params": [params[k]], "name": k, "lr": lr} for k, lr in LRS.items()], lr=0.0,
                        eps=1e-15)
        drv = TimestepDriver(params, {}, opt, C, batch_renderer(sets), sharded=sharded)
        losses = drv.run(2, lambda t: 2, lambda t: targets)
        if sharded:
            assert drv.zs is not None and drv.zs.overlap and drv.zs.k == 4  # one ShardedStep for the run
        torch.cuda.synchronize()
        runs[sharded] = ({k: v.detach().clone() for k, v in drv.params.items()}, losses,
                         {k: opt.state[p]["exp_avg"].clone() for k, p in drv.params.items()})
    (pp, lp, mp_), (ps, ls, ms) = runs[False], runs[True]
    for a, b in zip(lp, ls):
        for x, y in zip(a, b):
            assert abs(x - y) <= 1e-5 * abs(x) + 1e-7, (lp, ls)
    for k in LRS:
        d = (ps[k] - pp[k]).abs().reshape(-1)
        assert float(d.max()) <= 4 * 2 * LRS[k] + 1e-6, (k, float(d.max()))
        q = float(torch.quantile(d[:1_000_000].double(), 0.999))
        assert q <= 1e-3 * LRS[k], (k, q)
        assert ms[k].shape == mp_[k].shape  # the optimizer got the sharded state back (run -> sync_optimizer)


def test_two_rank_gloo_rehearsal_of_the_overlapped_exchange():
    """tools/zov_check.py over two gloo ranks sharing the GPU (the exchange
    emulated by all-reduces, gloo's CUDA path): per step, each rank's
    gradients vs a replay from what it read (<= 1e-6), the parameters read
    vs an in-line Adam over the ranks' summed gradients (bit for bit), and
    the ranks' final parameters equal."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(repo, "tools", "zov_check.py")]
    r = subprocess.run(cmd, cwd=repo, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-4000:], r.stderr[-4000:])
    assert '"ok": true' in r.stdout
