"""Fused Adam + densification statistics against
torch.optim.Adam and the reference's statistics code, on the reference's
parameter groups (train.py:119-135: per-group lr, two of them 0, eps=1e-15).

Adam: the kernel evaluates torch's multi-tensor Adam op sequence in fp32
(lerp, mul, addcmul, sqrt, div, add, addcdiv; scalars rounded once from
double like torch's scalar arguments; the multiply-adds torch's ROCm build
contracts as explicit fmas), so parameters and moments are BIT-IDENTICAL to
torch.optim.Adam's (tools/adam_probe.py reports the per-word agreement)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu

LRS = {"means3D": 0.0000016 * 3.2, "rgb_colors": 0.000025, "seg_colors": 0.0, "unnorm_rotations": 0.0,
       "logit_opacities": 0.05, "log_scales": 0.001, "cam_m": 1e-5, "cam_c": 1e-5}
SHAPES = {"means3D": 3, "rgb_colors": 3, "seg_colors": 3, "unnorm_rotations": 4, "logit_opacities": 1,
          "log_scales": 3}


def make_params(P=10007, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    params = {k: torch.randn(P, c, device="cuda", generator=g) for k, c in SHAPES.items()}
    params["cam_m"] = torch.randn(27, 3, device="cuda", generator=g)
    params["cam_c"] = torch.randn(27, 3, device="cuda", generator=g)
    return {k: torch.nn.Parameter(v.contiguous()) for k, v in params.items()}


def make_opt(cls, params, **kw):
    groups = [{"params": [v], "name": k, "lr": LRS[k]} for k, v in params.items()]
    return cls(groups, lr=0.0, eps=1e-15, **kw)


def set_grads(params, step, skip=()):
    g = torch.Generator(device="cuda").manual_seed(100 + step)
    for k, p in params.items():
        p.grad = None if k in skip else torch.randn(p.shape, device="cuda", generator=g) * 10 ** (step % 3 - 1)


def assert_params_equal(a, b):
    for k in a:
        x, y = a[k].detach(), b[k].detach()
        assert torch.equal(x, y), (k, (x - y).abs().max().item(), (x != y).float().mean().item())


def _clone(params):
    return {k: torch.nn.Parameter(v.detach().clone()) for k, v in params.items()}


def test_fused_adam_matches_torch_adam():
    from dynamic3dgaussians_amd.optim import FusedAdam
    ref = make_params()
    ours = _clone(ref)
    o_ref = make_opt(torch.optim.Adam, ref)
    o_ours = make_opt(FusedAdam, ours)
    for step in range(6):
        skip = ("cam_m",) if step == 2 else ()
        set_grads(ref, step, skip)
        set_grads(ours, step, skip)
        o_ref.step()
        o_ours.step()
        assert_params_equal(ours, ref)
    for k in ref:
        sr, so = o_ref.state[ref[k]], o_ours.state[ours[k]]
        assert sr["step"].item() == so["step"].item(), k
        assert so["step"].device.type == "cpu" and so["step"].dtype == torch.float32
        for key in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(so[key], sr[key]), (k, key)
    # lr 0 groups never move, but their moments do (like torch)
    assert torch.equal(ours["seg_colors"].detach(), ref["seg_colors"].detach())


def _cat_params(new_params, params, optimizer):
    """The reference's cat_params_to_optimizer (external.py:158-182), restated."""
    for k, v in new_params.items():
        group = [g for g in optimizer.param_groups if g["name"] == k][0]
        st = optimizer.state.get(group["params"][0], None)
        st["exp_avg"] = torch.cat((st["exp_avg"], torch.zeros_like(v)), dim=0)
        st["exp_avg_sq"] = torch.cat((st["exp_avg_sq"], torch.zeros_like(v)), dim=0)
        del optimizer.state[group["params"][0]]
        group["params"][0] = torch.nn.Parameter(torch.cat((group["params"][0], v), dim=0).requires_grad_(True))
        optimizer.state[group["params"][0]] = st
        params[k] = group["params"][0]
    return params


def _remove(to_keep, params, optimizer):
    """The reference's remove_points (external.py:185-207), restated."""
    for k in list(params):
        if k in ("cam_m", "cam_c"):
            continue
        group = [g for g in optimizer.param_groups if g["name"] == k][0]
        st = optimizer.state.get(group["params"][0], None)
        st["exp_avg"] = st["exp_avg"][to_keep]
        st["exp_avg_sq"] = st["exp_avg_sq"][to_keep]
        del optimizer.state[group["params"][0]]
        group["params"][0] = torch.nn.Parameter(group["params"][0][to_keep].requires_grad_(True))
        optimizer.state[group["params"][0]] = st
        params[k] = group["params"][0]
    return params


def test_fused_adam_survives_reference_state_surgery():
    from dynamic3dgaussians_amd.optim import FusedAdam
    ref = make_params(P=5000, seed=1)
    ours = _clone(ref)
    o_ref, o_ours = make_opt(torch.optim.Adam, ref), make_opt(FusedAdam, ours)
    for step in range(2):
        set_grads(ref, step)
        set_grads(ours, step)
        o_ref.step()
        o_ours.step()
    sel = torch.arange(0, 5000, 7, device="cuda")
    for params, opt in ((ref, o_ref), (ours, o_ours)):
        new = {k: v.detach()[sel] for k, v in params.items() if k not in ("cam_m", "cam_c")}
        _cat_params(new, params, opt)
        keep = torch.ones(params["means3D"].shape[0], dtype=torch.bool, device="cuda")
        keep[::5] = False
        _remove(keep, params, opt)
    for step in range(2, 5):
        set_grads(ref, step)
        set_grads(ours, step)
        o_ref.step()
        o_ours.step()
    assert_params_equal(ours, ref)


def _ref_stats(variables, radius):
    """train.py:288-290 + external.py:136-140."""
    seen = radius > 0
    variables["max_2D_radius"][seen] = torch.max(radius[seen], variables["max_2D_radius"][seen])
    variables["means2D_gradient_accum"][seen] += torch.norm(variables["means2D"].grad[seen, :2], dim=-1)
    variables["denom"][seen] += 1
    variables["seen"] = seen


def _stats_vars(P, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    m2 = torch.zeros(P, 3, device="cuda", requires_grad=True)
    m2.grad = torch.randn(P, 3, device="cuda", generator=g) * 1e-3
    return {"max_2D_radius": torch.rand(P, device="cuda", generator=g) * 20,
            "means2D_gradient_accum": torch.rand(P, device="cuda", generator=g),
            "denom": torch.randint(0, 9, (P,), device="cuda", generator=g).float(),
            "means2D": m2}


def test_densify_stats_match_reference():
    from dynamic3dgaussians_amd.optim import densify_stats
    P = 30001
    g = torch.Generator(device="cuda").manual_seed(4)
    radius = (torch.randint(-3, 40, (P,), device="cuda", generator=g)).clamp_min(0).int()
    a, b = _stats_vars(P, 5), _stats_vars(P, 5)
    _ref_stats(a, radius)
    densify_stats(b, radius)
    assert torch.equal(b["max_2D_radius"], a["max_2D_radius"])
    assert torch.equal(b["denom"], a["denom"])
    assert torch.equal(b["means2D_gradient_accum"], a["means2D_gradient_accum"])
    assert torch.equal(b["seen"], a["seen"])
    # max radius only (the non-densifying timesteps)
    c = _stats_vars(P, 5)
    acc0 = c["means2D_gradient_accum"].clone()
    densify_stats(c, radius, accumulate=False)
    assert torch.equal(c["max_2D_radius"], a["max_2D_radius"])
    assert torch.equal(c["means2D_gradient_accum"], acc0)


def test_step_with_fused_stats_equals_separate():
    from dynamic3dgaussians_amd.optim import FusedAdam, densify_stats
    P = 10007
    base = make_params(P=P, seed=2)
    p1, p2 = _clone(base), _clone(base)
    o1, o2 = make_opt(FusedAdam, p1), make_opt(FusedAdam, p2)
    g = torch.Generator(device="cuda").manual_seed(8)
    radius = torch.randint(0, 30, (P,), device="cuda", generator=g).int()
    v1, v2 = _stats_vars(P, 9), _stats_vars(P, 9)
    set_grads(p1, 0)
    set_grads(p2, 0)
    densify_stats(v1, radius)
    o1.step()
    o2.step(stats=(v2, radius))
    for k in p1:
        assert torch.equal(p1[k].detach(), p2[k].detach()), k
    for k in ("max_2D_radius", "means2D_gradient_accum", "denom", "seen"):
        assert torch.equal(v1[k], v2[k]), k


def test_fused_adam_step_counts_follow_external_changes():
    """FusedAdam caches each parameter's step count against its state tensor;
    a step tensor replaced (load_state_dict, state surgery) or changed in place
    from outside must be re-read, exactly as torch.optim.Adam reads it."""
    from dynamic3dgaussians_amd.optim import FusedAdam
    ref = make_params(P=4099, seed=3)
    ours = _clone(ref)
    o_ref = make_opt(torch.optim.Adam, ref)
    o_ours = make_opt(FusedAdam, ours)

    def both_step(step):
        set_grads(ref, step)
        set_grads(ours, step)
        o_ref.step()
        o_ours.step()

    for step in range(3):
        both_step(step)
    for o, ps in ((o_ref, ref), (o_ours, ours)):
        o.state[ps["means3D"]]["step"] = torch.tensor(40.0)   # replaced tensor
        o.state[ps["log_scales"]]["step"].fill_(7.0)           # changed in place
    both_step(3)
    for o, ps in ((o_ref, ref), (o_ours, ours)):
        assert float(o.state[ps["means3D"]]["step"]) == 41.0
        assert float(o.state[ps["log_scales"]]["step"]) == 8.0
    # a state_dict round trip (new step tensors) mid-training
    o_ours.load_state_dict(o_ours.state_dict())
    for step in range(4, 6):
        both_step(step)
    assert_params_equal(ref, ours)
    for k in ref:
        assert float(o_ours.state[ours[k]]["step"]) == float(o_ref.state[ref[k]]["step"])
