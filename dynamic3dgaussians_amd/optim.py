"""Fused Adam + densification statistics on one HIP launch (SURVEY.md 8(f)
rank 3; csrc/gs_optim.hip, C ABI include/gs_optim.h).

`FusedAdam` is a drop-in for the reference's optimizer
(`torch.optim.Adam(param_groups, lr=0.0, eps=1e-15)`, train.py:119-135):
same constructor, same `param_groups` (with the reference's 'name' keys) and
the same per-parameter state ('step' as a CPU fp32 tensor, 'exp_avg',
'exp_avg_sq'), so the reference's in-place optimizer-state surgery
(cat_params_to_optimizer / remove_points / update_params_and_optimizer,
external.py:143-213) works on it unchanged.  `step()` updates every
parameter of every group in ONE kernel launch instead of torch's chain of
multi-tensor kernels.

`densify_stats(variables, radius, accumulate=True)` is the statistics half
on its own (train.py:288-290 and external.py:136-140); `step(stats=...)`
fuses it into the same launch:

    loss.backward()
    optimizer.step(stats=(variables, radius))   # max_2D_radius, grad accum, denom, Adam
    optimizer.zero_grad(set_to_none=True)

(call `densify_stats` + `densify` + `step()` separately on the iterations
where densify() clones / splits / prunes, as the reference orders them).
No CPU path: parameters must be contiguous fp32 device tensors.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

MAX_TENSORS = 16


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _stats_struct(variables: dict, radius: torch.Tensor, accumulate: bool):
    P = radius.numel()
    if not radius.is_cuda or radius.dtype != torch.int32:
        raise _lib.GsplatError("radius must be the rasterizer's int32 device tensor")
    mr = variables["max_2D_radius"]
    for name, t in (("max_2D_radius", mr),):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == P):
            raise _lib.GsplatError(f"variables['{name}'] must be a contiguous fp32 device tensor of length {P}")
    st = _lib.GsDensifyStats(P=P, radii=radius.contiguous().data_ptr(), max_radius=mr.data_ptr())
    keep = [radius]
    if accumulate:
        acc, den = variables["means2D_gradient_accum"], variables["denom"]
        g = variables["means2D"].grad
        if g is None:
            raise _lib.GsplatError("variables['means2D'].grad is None (call after backward)")
        for name, t in (("means2D_gradient_accum", acc), ("denom", den)):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == P):
                raise _lib.GsplatError(f"variables['{name}'] must be a contiguous fp32 device tensor of length {P}")
        g = g.contiguous()
        if g.shape != (P, 3) or g.dtype != torch.float32:
            raise _lib.GsplatError(f"means2D.grad must be fp32 [P, 3] (got {tuple(g.shape)} {g.dtype})")
        st.means2D_grad, st.grad_accum, st.denom = g.data_ptr(), acc.data_ptr(), den.data_ptr()
        keep.append(g)
    return st, keep


def densify_stats(variables: dict, radius: torch.Tensor, accumulate: bool = True):
    """seen = radius > 0; max_2D_radius[seen] = max(radius, max_2D_radius)
    (train.py:288-290) and, with `accumulate`, accumulate_mean2d_gradient
    (external.py:136-140) -- one launch.  Also sets variables['seen']."""
    st, keep = _stats_struct(variables, radius, accumulate)
    args = _lib.GsAdamArgs(n_tensors=0, beta1=0.9, beta2=0.999, eps=1e-8)
    _lib.check(_lib.load().gs_adam_step(ctypes.byref(args), ctypes.byref(st), _stream(radius.device)),
               "densify stats")
    variables["seen"] = radius > 0
    del keep
    return variables


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False, **unused):
        if weight_decay != 0 or amsgrad or maximize:
            raise ValueError("FusedAdam implements the reference's Adam (no weight decay / amsgrad / maximize)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)

    def _next_step(self, p, state) -> float:
        """Advance the parameter's step count (the CPU tensor state['step'],
        as torch.optim.Adam keeps it) and return it as a float.  The float is
        cached against the tensor's identity and version, so the usual step
        costs one in-place fill instead of an add plus a device-less .item();
        a step tensor replaced or modified from outside is re-read."""
        st = state["step"]
        c = self._step_cache.get(id(p))
        t = (c[2] if (c is not None and c[0] is st and c[1] == st._version) else float(st.item())) + 1.0
        st.fill_(t)
        self._step_cache[id(p)] = (st, st._version, t)
        return t

    @torch.no_grad()
    def step(self, closure=None, stats=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not hasattr(self, "_step_cache"):
            self._step_cache = {}
            self._args_cache = {}
        if len(self._step_cache) > 64:  # parameters replaced by densification: drop stale entries
            live = {id(p) for g_ in self.param_groups for p in g_["params"]}
            self._step_cache = {k: v for k, v in self._step_cache.items() if k in live}
        entries = []
        dev = None
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                g = p.grad
                if g is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise _lib.GsplatError("FusedAdam needs contiguous fp32 device parameters")
                if g.is_sparse:
                    raise _lib.GsplatError("FusedAdam does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:  # torch.optim.Adam's lazy state init
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                t = self._next_step(p, state)
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                if not g.is_contiguous():
                    g = g.contiguous()
                entries.append((p, g, state["exp_avg"], state["exp_avg_sq"], (group["lr"] / bc1) * -1,
                                bc2 ** 0.5, group))
                dev = p.device
        st = keep = None
        if stats is not None:
            variables, radius = stats[0], stats[1]
            accumulate = stats[2] if len(stats) > 2 else True
            st, keep = _stats_struct(variables, radius, accumulate)
            dev = radius.device
        if dev is None:
            return loss
        L = _lib.load()
        stream = _stream(dev)
        first = True
        for b in range(0, max(len(entries), 1), MAX_TENSORS):
            chunk = entries[b:b + MAX_TENSORS]
            # one launch per group of <= 16 tensors sharing (beta1, beta2, eps)
            by_hyper = {}
            for e in chunk:
                grp = e[6]
                by_hyper.setdefault((grp["betas"][0], grp["betas"][1], grp["eps"]), []).append(e)
            if not by_hyper:
                by_hyper = {(0.9, 0.999, 1e-8): []}
            for (b1, b2, eps), es in by_hyper.items():
                # the launch's argument block is reused from step to step; only
                # the per-step fields are rewritten
                key = (b, b1, b2, eps, len(es))
                args = self._args_cache.get(key)
                if args is None:
                    args = self._args_cache[key] = _lib.GsAdamArgs(n_tensors=len(es), beta1=b1, beta2=b2, eps=eps)
                for k, (p, g, m, v, step_size, bc2s, _) in enumerate(es):
                    tk = args.t[k]
                    tk.param, tk.grad, tk.exp_avg, tk.exp_avg_sq = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
                    tk.numel, tk.step_size, tk.bc2_sqrt = p.numel(), step_size, bc2s
                sp = ctypes.byref(st) if (first and st is not None) else None
                _lib.check(L.gs_adam_step(ctypes.byref(args), sp, stream), "adam step")
                first = False
        if stats is not None:
            stats[0]["seen"] = stats[1] > 0
        del keep
        return loss
