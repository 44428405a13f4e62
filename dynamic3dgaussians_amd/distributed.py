"""Camera-sharded data parallelism for the per-timestep multi-camera step.

The reference trains one camera per optimizer step and has no distributed
code.  Here a step renders a batch of cameras; cameras are
sharded over ranks (camera c -> rank c mod N, one process per GPU), each rank
runs forward+backward for its cameras with the full Gaussian set replicated,
and ONE flat-bucket all_reduce(SUM) of every per-Gaussian gradient (plus the
densification statistics) over RCCL/xGMI precedes an identical Adam step on
every rank.  max_2D_radius needs MAX, so it travels in a second, small
all_reduce (train.py:288-290, external.py:136-140).
"""
from __future__ import annotations

import ctypes
import weakref
from typing import Dict, Iterable, List, Mapping, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _lib


def shard_cameras(n_cams: int, rank: int, world: int) -> List[int]:
    """Camera c goes to rank c mod world."""
    return [c for c in range(n_cams) if c % world == rank]


def shard_camera_windows(n_cams: int, rank: int, world: int, grid_x: int, grid_y: int,
                         row_cost: Optional[Sequence[Sequence[float]]] = None, piece_cost: float = 0.0,
                         whole_scale: Optional[Sequence[float]] = None
                         ) -> List[Tuple[int, Optional[Tuple[int, int, int, int]]]]:
    """Balanced split of an n_cams rig over `world` ranks with image sharding
    (gs_camera tile_*): the first world * (n_cams // world) cameras whole,
    camera c on rank c mod world, and the n_cams % world left-over cameras
    cut into bands of tile rows that even out the ranks' totals.

    The left-over cameras' tile rows are laid end to end (camera-major) and
    cut into `world` consecutive runs, run k to rank k, each as long as rank
    k needs to reach the common level of the balanced loads (the mean unless
    some rank's whole cameras alone exceed it) -- so a rank gets a few bands
    (one or two on the 27-camera rig over 8 ranks), not a band of every
    left-over camera.  `row_cost[c][y]` is the work of camera c's tile row y
    (e.g. its tile-list instances from a previous forward); without it every
    row of every camera costs the same (the pixel split).  `piece_cost`: the
    fixed work of rendering one more camera (its projection and binning
    launches, in row_cost units): a rank whose run spans two left-over
    cameras is charged it and given fewer rows (a few refinement passes).
    `whole_scale[k]` (measured-feedback balancing, rank_load_scale): a factor
    on rank k's whole-camera load, the rank's measured step per modelled unit
    relative to the mean -- the model counts instances, and cameras differ in
    blend work per instance.
    Returns
    [(camera, window or None)], window = (x0, y0, x1, y1) in tiles, rank-major
    deterministic (every rank computes the same cut).  The windows of a camera
    partition its tile grid, so the ranks' gradients sum to the rig's."""
    q, r = divmod(n_cams, world)
    cost = (lambda c, y: 1.0) if row_cost is None else (lambda c, y: max(float(row_cost[c][y]), 0.0))
    out = [(c, None) for c in range(q * world) if c % world == rank]
    if not r:
        return out
    whole = [sum(cost(c, y) for c in range(q * world) if c % world == k for y in range(grid_y))
             for k in range(world)]
    if whole_scale is not None:
        whole = [w * float(f) for w, f in zip(whole, whole_scale)]
    seq = [(c, y) for c in range(q * world, n_cams) for y in range(grid_y)]
    pre = [0.0]
    for c, y in seq:
        pre.append(pre[-1] + cost(c, y))
    left = pre[-1]

    def cut(base):
        # water-filling: the level T at which the ranks below it absorb
        # exactly the left-over work (ranks already above T get no rows)
        lv = sorted(base)
        T, acc_w = lv[-1] + left / world, 0.0
        for j, w in enumerate(lv):
            acc_w += w
            t = (acc_w + left) / (j + 1)
            if j + 1 == world or t <= lv[j + 1]:
                T = t
                break
        need = [max(0.0, T - w) for w in base]
        tot_need = sum(need)
        need = [n * left / tot_need for n in need] if tot_need > 0 else [left / world] * world
        # run k ends where the cumulative cost comes closest to the cumulative need
        bounds, acc, i = [0], 0.0, 0
        for k in range(world - 1):
            acc += need[k]
            while i < len(seq) and abs(pre[i + 1] - acc) <= abs(pre[i] - acc):
                i += 1
            i = max(i, bounds[-1])
            bounds.append(i)
        bounds.append(len(seq))
        return bounds

    def pieces(bounds, k):
        return len({c for c, _ in seq[bounds[k]:bounds[k + 1]]})

    def loads(bounds):
        return [whole[k] + pre[bounds[k + 1]] - pre[bounds[k]] + piece_cost * pieces(bounds, k)
                for k in range(world)]

    bounds = cut(whole)
    cands = [bounds]
    for _ in range(6 if piece_cost > 0 else 0):
        nb = cut([w + piece_cost * pieces(bounds, k) for k, w in enumerate(whole)])
        if nb in cands:
            break
        cands.append(nb)
        bounds = nb
    # the piece refinement can oscillate (a run gains or loses its second
    # camera between passes): keep the candidate whose largest modelled load
    # is least, then move single boundaries row by row while that improves it
    bounds = min(cands, key=lambda b: (max(loads(b)), cands.index(b)))
    if piece_cost > 0:
        best = max(loads(bounds))
        improved = True
        while improved:
            improved = False
            for k in range(1, world):
                for d in (-1, 1):
                    b = list(bounds)
                    b[k] += d
                    if not (b[k - 1] <= b[k] <= b[k + 1]):
                        continue
                    m = max(loads(b))
                    if m < best - 1e-9:
                        bounds, best, improved = b, m, True
    mine = seq[bounds[rank]:bounds[rank + 1]]
    for c in range(q * world, n_cams):
        ys = [y for cc, y in mine if cc == c]
        if ys:
            out.append((c, (0, ys[0], grid_x, ys[-1] + 1)))
    return out


def rank_load_scale(measured_ms: Sequence[float], model_load: Sequence[float]) -> List[float]:
    """Measured-feedback factors for shard_camera_windows(whole_scale=...):
    each rank's measured step per unit of modelled load (row_cost units),
    relative to the mean over the ranks.  Every rank must call it with the
    same numbers (gather the step times first), so every rank cuts the same
    windows."""
    rate = [m / max(l, 1e-30) for m, l in zip(measured_ms, model_load)]
    mean = sum(rate) / len(rate)
    return [r / mean for r in rate]


class StaleBucketError(RuntimeError):
    """A tensor the bucket was built over has been replaced or resized (the
    reference's densification rebinds variables[...] and the optimizer's
    Parameters, external.py:202-204, 273-275): build a new GradBucket."""


class GradBucket:
    """Flattens the .grad of a fixed list of parameters into one contiguous
    fp32 buffer, together with per-Gaussian running statistics (`extras`),
    all-reduces it with one collective and scatters the result back.

    Gradients are per-step quantities and are summed as they are.  The
    extras are RUNNING TOTALS that every rank holds identically at the start
    of a step (e.g. means2D_gradient_accum and denom, external.py:136-140):
    each rank adds its own cameras' contributions, so only the change since
    the last synchronisation point is summed over the ranks and added back to
    the common starting value.  Summing the totals themselves would multiply
    the history by world_size every step.  Synchronisation points are the
    construction, every all_reduce(), and resync() -- call it after changing
    the extras' VALUES identically on every rank outside a step.

    Densification (external.py:202-204, 273-275) does not change
    values in place: it binds NEW tensors into the variables dict and NEW
    Parameters into the optimizer, with a different Gaussian count.  A bucket
    cannot follow that; all_reduce() and resync() therefore check that every
    tensor is still the live object with the size the bucket was built for
    and raise StaleBucketError otherwise -- build a new GradBucket after every
    densification.  To let the check see replacements, pass the containers
    the caller rebinds: `params` may be a dict (name -> Parameter, e.g. the
    params dict the optimizer groups are built from) and `extras_from` a
    (dict, keys) pair (e.g. (variables, ["means2D_gradient_accum", "denom"])).
    `keys` restricts a dict of parameters to the trainable entries (e.g.
    without the reference's constant seg_colors).

    bind_grads=True makes every parameter's .grad a view into the flat
    buffer: the backward accumulates straight into the bucket, so
    all_reduce() needs no pack/unpack copies of the gradients.  Clear the
    gradients with zero_grad() (one fill of the buffer) instead of the
    optimizer's zero_grad(set_to_none=True), which would unbind them.

    track_reached=True (bound mode): a bound .grad exists whether or not the
    step's loss reached the parameter, so an optimizer would step every
    parameter (Adam moving an unreached one on its old moments) where the
    single-process run leaves .grad None and skips it.  The bucket notes on
    each rank which parameters autograd accumulated into (post-accumulate
    hooks), sums those flags over the ranks in the same all_reduce, and after
    it sets .grad = None on the parameters no rank reached (one small
    device->host read of the flags); zero_grad() binds them again.  The
    hooks hold the bucket only weakly and close() removes them: a parameter
    that survives a densification (e.g. the reference's cam_m / cam_c) must
    not keep every replaced bucket -- and its flat buffer -- alive, nor run
    their stale hooks in every later backward.
    """

    def __init__(self, params: Iterable[torch.Tensor] | Mapping[str, torch.Tensor],
                 extras: Dict[str, torch.Tensor] | None = None,
                 extras_from: tuple[Mapping[str, torch.Tensor], Sequence[str]] | None = None,
                 bind_grads: bool = False, keys: Sequence[str] | None = None, track_reached: bool = False,
                 n_aux: int = 0):
        if isinstance(params, Mapping):
            self._param_src, self._param_keys = params, list(keys if keys is not None else params.keys())
            self.params = [params[k] for k in self._param_keys]
        else:
            self._param_src, self._param_keys = None, None
            self.params = list(params)
        self.extras = dict(extras or {})
        self._extra_src = None
        if extras_from is not None:
            src, keys = extras_from
            self._extra_src = src
            for k in keys:
                self.extras[k] = src[k]
        self._param_numel = [p.numel() for p in self.params]
        self._extra_numel = {k: t.numel() for k, t in self.extras.items()}
        sizes = self._param_numel + list(self._extra_numel.values())
        self.sizes = sizes
        if not self.params and not self.extras:
            raise ValueError("GradBucket: nothing to exchange")
        dev = (self.params[0] if self.params else next(iter(self.extras.values()))).device
        self.track = bool(track_reached and bind_grads)
        n_flags = len(self.params) if self.track else 0
        # n_aux: a per-step slot summed as it is (all_reduce(aux=...)), e.g.
        # ShardedStep's reached-parameter flags riding with the statistics
        self.n_aux = int(n_aux)
        self._aux_at = sum(sizes) + n_flags
        self.flat = torch.zeros(sum(sizes) + n_flags + self.n_aux, dtype=torch.float32, device=dev)
        self.bound = bind_grads
        self._reached = [False] * len(self.params)
        self._unbound = set()
        self._hooks = []
        if self.track:
            for i, p in enumerate(self.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._hook(i)))
        self._views = []
        o = 0
        for p in self.params:
            n = p.numel()
            self._views.append(self.flat[o:o + n].view_as(p))
            o += n
        if bind_grads:
            for p, v in zip(self.params, self._views):
                p.grad = v
        self._base = {}
        self.resync()

    def _hook(self, i):
        ref = weakref.ref(self)

        def mark(_p):
            b = ref()
            if b is not None:
                b._reached[i] = True
        return mark

    def close(self) -> None:
        """Remove the reach-tracking hooks from the parameters (idempotent).
        Call it when the bucket is replaced (a new bucket per timestep or
        after a densification); a closed bucket no longer tracks reach."""
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- checks
    def check_live(self) -> None:
        """Raise StaleBucketError if a parameter or extra was replaced or
        resized since construction, or a bound gradient was unbound."""
        if self._param_src is not None:
            for k, p in zip(self._param_keys, self.params):
                if self._param_src.get(k) is not p:
                    raise StaleBucketError(f"parameter '{k}' was replaced (densification?): "
                                           "build a new GradBucket")
        for i, (p, n) in enumerate(zip(self.params, self._param_numel)):
            if p.numel() != n:
                raise StaleBucketError(f"parameter {i} changed size {n} -> {p.numel()}: build a new GradBucket")
        if self._extra_src is not None:
            for k, t in self.extras.items():
                if k in self._extra_src and self._extra_src[k] is not t:
                    raise StaleBucketError(f"statistic '{k}' was replaced (densification?): "
                                           "build a new GradBucket")
        for k, t in self.extras.items():
            if t.numel() != self._extra_numel[k]:
                raise StaleBucketError(f"statistic '{k}' changed size: build a new GradBucket")
        if self.bound:
            for i, (p, v) in enumerate(zip(self.params, self._views)):
                if i in self._unbound and p.grad is None:
                    continue  # unbound by all_reduce (reached by no rank); zero_grad() binds it again
                if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                    raise StaleBucketError(
                        f"parameter {i}'s .grad is no longer the bucket's view (zero_grad(set_to_none=True)?): "
                        "clear gradients with GradBucket.zero_grad()")

    # ---------------------------------------------------------------- grads
    def bind(self) -> None:
        """Bound mode: make every parameter's .grad this bucket's view (again):
        several buckets can take turns over the same parameters, e.g. a
        double-buffered gradient set whose all-reduce runs behind the next
        step (all_reduce_async)."""
        for p, v in zip(self.params, self._views):
            p.grad = v
        self._unbound.clear()

    def all_reduce_async(self, group=None):
        """One all_reduce(SUM) of a bound bucket without extras, left running:
        returns the work handle (wait() on it -- on the stream that consumes
        the gradients -- before using them), None without a process group
        (a world of one still runs the collective: bench.py's RCCL rehearsal).
        The gradients are summed in place in the bound views."""
        if not self.bound or self.extras or self.track:
            raise ValueError("all_reduce_async: bound gradients only (no extras, no reach tracking)")
        self.check_live()
        if not (dist.is_available() and dist.is_initialized()):
            return None
        return dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group, async_op=True)

    def zero_grad(self) -> None:
        """Bound mode: zero every gradient with one fill of the buffer."""
        if self.bound:
            for i in self._unbound:
                self.params[i].grad = self._views[i]
            self._unbound.clear()
            self._reached = [False] * len(self.params)
            n = sum(self._param_numel)
            self.flat[:n].zero_()
        else:
            for p in self.params:
                p.grad = None

    def resync(self) -> None:
        """Record the extras' current values as the common starting point of
        the next step (they must be identical on every rank)."""
        self.check_live()
        self._base = {k: t.detach().clone() for k, t in self.extras.items()}

    def pack(self):
        o = 0
        for p, v in zip(self.params, self._views):
            n = p.numel()
            if not self.bound:
                if p.grad is None:
                    v.zero_()
                else:
                    v.copy_(p.grad)
            o += n
        for k, t in self.extras.items():
            n = t.numel()
            # this rank's increment since the last synchronisation point
            torch.sub(t.reshape(-1), self._base[k].reshape(-1), out=self.flat[o:o + n])
            o += n
        if self.track:
            self.flat[o:o + len(self.params)].copy_(torch.tensor(self._reached, dtype=torch.float32))

    def unpack(self):
        o = 0
        for p, v in zip(self.params, self._views):
            n = p.numel()
            if not self.bound:
                if p.grad is None:
                    p.grad = torch.empty_like(p)
                p.grad.copy_(v)
            o += n
        for k, t in self.extras.items():
            n = t.numel()
            # common start + every rank's increment
            torch.add(self._base[k].reshape(-1), self.flat[o:o + n], out=t.reshape(-1))
            o += n

    def all_reduce(self, group=None, aux: Optional[torch.Tensor] = None):
        """pack -> one all_reduce(SUM) -> unpack.  Without a process group
        (or with one rank) the values stay as they are.  `aux`: n_aux floats
        summed over the ranks in the same collective, in place."""
        self.check_live()
        if aux is not None and aux.numel() != self.n_aux:
            raise ValueError(f"GradBucket: aux of {aux.numel()} floats, the bucket holds {self.n_aux}")
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
            self.resync()
            return
        self.pack()
        if aux is not None:
            self.flat[self._aux_at:].copy_(aux.reshape(-1))
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.unpack()
        if aux is not None:
            aux.reshape(-1).copy_(self.flat[self._aux_at:])
        if self.track:
            reached = self.flat[self._aux_at - len(self.params):self._aux_at].cpu()
            for i, p in enumerate(self.params):
                if reached[i] == 0:
                    p.grad = None
                    self._unbound.add(i)
        self.resync()


def all_reduce_max_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place MAX all-reduce (max_2D_radius)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t


class ShardedAdam:
    """Adam with the update sharded over the ranks (ZeRO stage 1), for the
    camera-sharded step: instead of an all_reduce of every gradient followed
    by the same full Adam update on every rank, one reduce_scatter(SUM) hands
    each rank the summed gradients of its 1/N slice of the parameters, the
    rank runs Adam on that slice only (the fused kernel of gs_optim.h, one
    launch), and one all_gather returns the updated slices to every rank.
    The ring moves the same bytes as the all_reduce (reduce-scatter + all-
    gather IS the ring all-reduce), the Adam step's HBM traffic (7 fp32 per
    element: param, grad, both moments read, three written) and its moments'
    memory drop N-fold -- at 300k Gaussians x 46 floats, Adam is 61 us of a
    1.4 ms rank step at N = 8, the largest per-rank fixed cost.

    Layout.  The parameters' storage moves into one flat fp32 buffer
    (`param_flat`, padded to N x chunk, chunk a multiple of `align`): each
    Parameter keeps its identity (its .data becomes a view), so the caller's
    dict, the rasterizer inputs and anything else holding the Parameters are
    unchanged.  Gradients live in `n_grad_buffers` flat buffers of the same
    layout (two for a gradient set exchanged behind the next step).  Two ways
    to fill one:
      * grad_views(k): {name: view} destinations for the camera batch's
        backward (GaussianRasterizerBatch(...)(..., grad_into=...)): the
        kernels write the summed gradients straight into the bucket -- no
        gradient tensors, no accumulation, no fill, no pack copy;
      * bind(k) + zero_grad(k): .grad of every parameter is its view and
        autograd accumulates into it (gradients from any autograd path).
    The padding is never written and stays zero.

    step(k) = reduce_scatter(k) + update(k) + all_gather(); the three are
    public so that an exchange can run behind other work (reduce_scatter with
    async_op=True, the update and the gather on a side stream).  Without a
    process group (or with `collectives=False`) nothing is exchanged: the
    rank updates its own slice of its own gradients -- a one-GPU stand-in for
    rank `rank` of an N-rank step (bench.py --proxy-world).  `emulate`
    (default: gloo with CUDA tensors, which gloo only all-reduces) runs the
    reduce-scatter / all-gather as all-reduces of the whole buffer.

    Adam is torch.optim.Adam's (amsgrad off, no weight decay; gs_optim.h):
    a step count per parameter (a parameter no rank's loss reached is skipped
    and keeps its count, as torch skips a .grad of None), bias corrections
    computed in double on the host, per-parameter learning rates `lr[name]`
    (update(lr=...) takes the current ones, e.g. from the reference
    optimizer's param_groups).  At N = 1 it is bit-identical to FusedAdam over
    the same parameters; at N > 1 the gradient sums are the collective's.
    Not the reference's optimizer object: load_state() takes the moments and
    step counts from one (torch.optim.Adam / FusedAdam state), export_state()
    writes them back (all-gathering the moments) so the reference's
    optimizer-state surgery (densification, external.py:157-213) can run on
    it, and replace() rebinds a same-size replacement tensor with zeroed
    moments (update_params_and_optimizer, external.py:143-155).
    """

    def __init__(self, params: Mapping[str, torch.Tensor], lr: Mapping[str, float], rank: Optional[int] = None,
                 world: Optional[int] = None, group=None, betas=(0.9, 0.999), eps: float = 1e-15,
                 n_grad_buffers: int = 1, align: int = 64, collectives: Optional[bool] = None,
                 emulate: Optional[bool] = None):
        self.names = list(params)
        self.params = [params[k] for k in self.names]
        if not self.params:
            raise ValueError("ShardedAdam: no parameters")
        self.lr = [float(lr[k]) for k in self.names]
        self.beta1, self.beta2 = float(betas[0]), float(betas[1])
        self.eps = float(eps)
        dist_on = dist.is_available() and dist.is_initialized()
        self.group = group
        world = (dist.get_world_size(group) if dist_on else 1) if world is None else int(world)
        rank = (dist.get_rank(group) if dist_on else 0) if rank is None else int(rank)
        if not 0 <= rank < world:
            raise ValueError(f"ShardedAdam: rank {rank} outside a world of {world}")
        self.collectives = (dist_on and world > 1) if collectives is None else bool(collectives)
        if self.collectives and not (dist_on and dist.get_world_size(group) == world
                                     and dist.get_rank(group) == rank):
            raise ValueError("ShardedAdam: collectives need the process group's own rank and world")
        self.world, self.rank = world, rank
        dev = self.params[0].device
        for k, p in zip(self.names, self.params):
            if p.dtype != torch.float32 or p.device != dev:
                raise ValueError(f"ShardedAdam: parameter '{k}' must be fp32 on {dev}")
        sizes = [p.numel() for p in self.params]
        self.total = sum(sizes)
        self.chunk = -(-self.total // (world * align)) * align
        self.lo, self.hi = rank * self.chunk, (rank + 1) * self.chunk
        n = world * self.chunk
        self.param_flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.offsets = []
        o = 0
        with torch.no_grad():
            for p, m in zip(self.params, sizes):
                self.param_flat[o:o + m].copy_(p.detach().reshape(-1))
                p.data = self.param_flat[o:o + m].view_as(p)
                self.offsets.append(o)
                o += m
        self.grad_flat = [torch.zeros(n, dtype=torch.float32, device=dev) for _ in range(max(1, n_grad_buffers))]
        # gloo moves CUDA tensors through all_reduce only: its rehearsals
        # (2 ranks on one GPU) emulate the reduce-scatter / all-gather with it
        if emulate is None:
            emulate = self.collectives and dev.type == "cuda" and dist.get_backend(group) == "gloo"
        self._emulate = bool(emulate) and self.collectives
        if self.collectives and not self._emulate:
            self.grad_shard = [torch.zeros(self.chunk, dtype=torch.float32, device=dev) for _ in self.grad_flat]
        else:
            self.grad_shard = [g[self.lo:self.hi] for g in self.grad_flat]
        self.exp_avg = torch.zeros(self.chunk, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(self.chunk, dtype=torch.float32, device=dev)
        self.steps = [0] * len(self.params)
        # the rank's slice as pieces of the parameters: (param index, flat start, flat end)
        self.pieces = []
        for i, (o, m) in enumerate(zip(self.offsets, sizes)):
            a, b = max(self.lo, o), min(self.hi, o + m)
            if a < b:
                self.pieces.append((i, a, b))
        self._args = {}

    # ------------------------------------------------------------ gradients
    def grad_views(self, k: int = 0) -> Dict[str, torch.Tensor]:
        """{name: view of gradient buffer k shaped like the parameter} (the
        same view objects on every call: the buffers never move)."""
        if not hasattr(self, "_gviews"):
            self._gviews = [{name: g[o:o + p.numel()].view_as(p)
                             for name, p, o in zip(self.names, self.params, self.offsets)} for g in self.grad_flat]
        return dict(self._gviews[k])

    def bind(self, k: int = 0) -> None:
        """Make every parameter's .grad its view into gradient buffer k."""
        for p, v in zip(self.params, self.grad_views(k).values()):
            p.grad = v

    def zero_grad(self, k: int = 0) -> None:
        """Zero gradient buffer k (accumulating fills: bind(); grad_views()
        destinations are written whole by the backward and need none)."""
        self.grad_flat[k].zero_()

    # ------------------------------------------------------------ exchange
    def reduce_scatter(self, k: int = 0, async_op: bool = False):
        """Sum gradient buffer k over the ranks into this rank's slice
        (grad_shard[k]).  Returns the work handle with async_op (wait() on
        it on the stream that runs update(k)), else None."""
        if not self.collectives:
            return None
        if self._emulate:
            return dist.all_reduce(self.grad_flat[k], op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
        return dist.reduce_scatter_tensor(self.grad_shard[k], self.grad_flat[k], op=dist.ReduceOp.SUM,
                                          group=self.group, async_op=async_op)

    def all_gather(self, async_op: bool = False):
        """Every rank's updated slice into every rank's param_flat (in place:
        this rank's slice is the input)."""
        if not self.collectives:
            return None
        if self._emulate:
            buf = torch.zeros_like(self.param_flat)
            buf[self.lo:self.hi].copy_(self.param_flat[self.lo:self.hi])
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
            self.param_flat.copy_(buf)
            return None
        return dist.all_gather_into_tensor(self.param_flat, self.param_flat[self.lo:self.hi], group=self.group,
                                           async_op=async_op)

    @property
    def t(self) -> int:
        """The largest per-parameter step count."""
        return max(self.steps)

    # ------------------------------------------------------------ update
    def update(self, k: int = 0, lr: Optional[Mapping[str, float]] = None,
               reached: Optional[Sequence[bool]] = None) -> None:
        """Adam on this rank's slice, from grad_shard[k] (one launch).
        `lr`: {name: learning rate} for this step (missing names keep the
        constructor's).  `reached`: per parameter (self.names order), whether
        any rank's loss reached it -- unreached parameters are neither
        updated nor counted (every rank must pass the same flags)."""
        lrs = self.lr if lr is None else [float(lr.get(n, l)) for n, l in zip(self.names, self.lr)]
        live = [True] * len(self.params) if reached is None else [bool(x) for x in reached]
        if len(live) != len(self.params):
            raise ValueError(f"ShardedAdam: {len(live)} reach flags for {len(self.params)} parameters")
        for i, on in enumerate(live):
            if on:
                self.steps[i] += 1
        entries = []
        g = self.grad_shard[k]
        for i, a, b in self.pieces:
            if not live[i]:
                continue
            t = self.steps[i]
            bc1 = 1.0 - self.beta1 ** t
            bc2s = (1.0 - self.beta2 ** t) ** 0.5
            s, e = a - self.lo, b - self.lo
            entries.append((self.param_flat[a:b], g[s:e], self.exp_avg[s:e], self.exp_avg_sq[s:e],
                            (lrs[i] / bc1) * -1, bc2s))
        self._apply((k, tuple(live)), entries)

    def _apply(self, k, entries) -> None:
        if not entries:
            return
        if len(entries) > _lib.GS_ADAM_MAX_TENSORS:
            raise _lib.GsplatError(f"ShardedAdam: {len(entries)} parameter pieces > {_lib.GS_ADAM_MAX_TENSORS}")
        if not self.param_flat.is_cuda:
            raise _lib.GsplatError("ShardedAdam: the update is the HIP kernel (device parameters only)")
        args = self._args.get(k)
        if args is None:  # the pointers are fixed for the optimizer's life; only the step fields change
            args = self._args[k] = _lib.GsAdamArgs(n_tensors=len(entries), beta1=self.beta1, beta2=self.beta2,
                                                   eps=self.eps)
            for j, (p, g, m, v, _, _) in enumerate(entries):
                tj = args.t[j]
                tj.param, tj.grad, tj.exp_avg, tj.exp_avg_sq = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
                tj.numel = p.numel()
        for j, (_, _, _, _, step_size, bc2s) in enumerate(entries):
            args.t[j].step_size, args.t[j].bc2_sqrt = step_size, bc2s
        _lib.check(_lib.load().gs_adam_step(ctypes.byref(args), None,
                                            torch.cuda.current_stream(self.param_flat.device).cuda_stream),
                   "sharded adam step")

    def step(self, k: int = 0, lr: Optional[Mapping[str, float]] = None,
             reached: Optional[Sequence[bool]] = None) -> None:
        """reduce_scatter(k) -> update(k) -> all_gather(), in line."""
        self.reduce_scatter(k)
        self.update(k, lr, reached)
        self.all_gather()

    # ------------------------------------------------------------ state
    def _slices(self, i: int):
        """(flat start, flat end) of this rank's pieces of parameter i."""
        return [(a, b) for j, a, b in self.pieces if j == i]

    @torch.no_grad()
    def load_state(self, optimizer) -> None:
        """The moments (this rank's slice) and step counts of a torch-style
        Adam's state (torch.optim.Adam / FusedAdam: state[p] = {'step',
        'exp_avg', 'exp_avg_sq'}); parameters without state start at zero."""
        for i, (p, o) in enumerate(zip(self.params, self.offsets)):
            st = optimizer.state.get(p)
            st = st if st else None
            for a, b in self._slices(i):
                s, e = a - self.lo, b - self.lo
                if st is None:
                    self.exp_avg[s:e].zero_()
                    self.exp_avg_sq[s:e].zero_()
                else:
                    self.exp_avg[s:e].copy_(st["exp_avg"].reshape(-1)[a - o:b - o])
                    self.exp_avg_sq[s:e].copy_(st["exp_avg_sq"].reshape(-1)[a - o:b - o])
            self.steps[i] = int(float(st["step"])) if st is not None else 0

    def _gather(self, x: torch.Tensor) -> torch.Tensor:
        """Every rank's chunk of `x` (a moment) as one world * chunk buffer."""
        full = torch.zeros(self.world * self.chunk, dtype=x.dtype, device=x.device)
        full[self.lo:self.hi].copy_(x)
        if self.world == 1:
            return full
        if not self.collectives:
            raise RuntimeError("ShardedAdam: exporting the moments of a rank of N needs the process group")
        if self._emulate:
            dist.all_reduce(full, op=dist.ReduceOp.SUM, group=self.group)
        else:
            dist.all_gather_into_tensor(full, x.contiguous(), group=self.group)
        return full

    @torch.no_grad()
    def export_state(self, optimizer) -> None:
        """Write the full moments and step counts into optimizer.state (a
        collective at N > 1: every rank calls it), e.g. before the
        reference's densification surgery or a checkpoint."""
        m, v = self._gather(self.exp_avg), self._gather(self.exp_avg_sq)
        for i, (p, o) in enumerate(zip(self.params, self.offsets)):
            if self.steps[i] == 0 and not optimizer.state.get(p):
                continue  # never stepped: the reference optimizer has no state for it either
            n = p.numel()
            optimizer.state[p] = {"step": torch.tensor(float(self.steps[i]), dtype=torch.float32),
                                  "exp_avg": m[o:o + n].view_as(p).clone(),
                                  "exp_avg_sq": v[o:o + n].view_as(p).clone()}

    @torch.no_grad()
    def replace(self, name: str, tensor: torch.Tensor, reset_moments: bool = True) -> None:
        """Rebind parameter `name` to `tensor` (same number of elements, e.g.
        a new Parameter from update_params_and_optimizer, external.py:143-155):
        its values move into the flat storage and its .data becomes the view;
        with reset_moments its moments are zeroed.  The step count is kept."""
        i = self.names.index(name)
        old, o = self.params[i], self.offsets[i]
        if tensor.numel() != old.numel():
            raise ValueError(f"ShardedAdam.replace: '{name}' has {tensor.numel()} elements, "
                             f"the layout {old.numel()}")
        if tensor.dtype != torch.float32 or tensor.device != self.param_flat.device:
            raise ValueError(f"ShardedAdam.replace: '{name}' must be fp32 on {self.param_flat.device}")
        n = tensor.numel()
        if tensor is not old:
            self.param_flat[o:o + n].copy_(tensor.detach().reshape(-1))
            tensor.data = self.param_flat[o:o + n].view_as(tensor)
            self.params[i] = tensor
        if reset_moments:
            for a, b in self._slices(i):
                self.exp_avg[a - self.lo:b - self.lo].zero_()
                self.exp_avg_sq[a - self.lo:b - self.lo].zero_()


class ShardedStep:
    """One rank's optimizer step of the camera-sharded training step
    (the reference's loss.backward() -> optimizer.step() ->
    zero_grad(), train.py:424-433, with a step's cameras sharded over the
    ranks): Adam sharded over the ranks (ZeRO stage 1, ShardedAdam) and, with
    `overlap`, the feature gradients' exchange and update run behind the next
    step.

    Geometry (every parameter but `feature_key`): reduce-scatter, Adam on the
    rank's slice, all-gather -- in line, on the step's critical path.
    Features (`overlap`, the 32 of 46 floats per Gaussian at F = 32): two
    gradient buffers, step k's backward writes buffer k % 2; finish() issues
    its reduce-scatter asynchronously and runs the update and the all-gather
    on a side stream, behind an event.  Step k+1's blend waits for that event
    (`feature_ready` -> GaussianRasterizer(..., feature_ready=...) ->
    gs_gaussians.feature_ready), so the projection and binning of step k+1
    overlap the exchange; step k+2 waits for it in begin() before its
    backward writes buffer k % 2 again.  Without `overlap` (no features, no
    CUDA, or overlap=False) one ShardedAdam steps every parameter in line.

    A step:

        zs.begin()
        out = rasterizer(..., feature_ready=zs.feature_ready, grad_into=zs.grad_into(arg_names))
        torch.autograd.backward(outputs, upstream)      # or: zs.bind_grads() before any autograd path,
        zs.finish()                                     #     or zs.load_grads() after it

    and zs.drain() before anything reads the features outside that pattern
    (another stream, the host, a checkpoint).  Moved out of bench.py's
    step_zero (round 5) so the training driver (timesteps.TimestepDriver)
    takes the same path the per-rank bench proxies measure.

    `adam_cls`: the ShardedAdam class (tests substitute a torch restatement
    of the update to run the plumbing on the CPU)."""

    def __init__(self, params: Mapping[str, torch.Tensor], lr: Mapping[str, float], rank: Optional[int] = None,
                 world: Optional[int] = None, group=None, eps: float = 1e-15, betas=(0.9, 0.999),
                 overlap: Optional[bool] = None, feature_key: str = "semantic_feature",
                 collectives: Optional[bool] = None, emulate: Optional[bool] = None, adam_cls=None):
        adam_cls = ShardedAdam if adam_cls is None else adam_cls
        self.names = list(params)
        dev = params[self.names[0]].device
        if overlap is None:
            overlap = feature_key in params and dev.type == "cuda"
        if overlap and (feature_key not in params or dev.type != "cuda" or len(self.names) < 2):
            raise ValueError("ShardedStep(overlap=True) needs CUDA parameters with a feature tensor "
                             f"'{feature_key}' and geometry")
        self.overlap = bool(overlap)
        self.feature_key = feature_key
        kw = dict(rank=rank, world=world, group=group, eps=eps, betas=betas, collectives=collectives,
                  emulate=emulate)
        if self.overlap:
            self.geo = adam_cls({k: params[k] for k in self.names if k != feature_key}, lr, **kw)
            self.feat = adam_cls({feature_key: params[feature_key]}, lr, n_grad_buffers=2, **kw)
            self.side = torch.cuda.Stream(device=dev)
        else:
            self.geo = adam_cls(dict(params), lr, **kw)
            self.feat = None
            self.side = None
        self.device = dev
        self.k = 0                   # steps finished
        self._done = [None, None]    # per feature buffer: the event of the last exchange that read it
        self._bound = False

    # ------------------------------------------------------------ layout
    @property
    def opts(self) -> List[ShardedAdam]:
        return [self.geo] + ([self.feat] if self.feat is not None else [])

    @property
    def params(self) -> Dict[str, torch.Tensor]:
        return {n: p for o in self.opts for n, p in zip(o.names, o.params)}

    @property
    def rank(self) -> int:
        return self.geo.rank

    @property
    def world(self) -> int:
        return self.geo.world

    def _buffers(self):
        """(optimizer, gradient buffer index) pairs of the current step."""
        return [(self.geo, 0)] + ([(self.feat, self.k % 2)] if self.feat is not None else [])

    # ------------------------------------------------------------ a step
    def begin(self) -> None:
        """Start step k: the current stream waits until step k-2's feature
        exchange no longer reads gradient buffer k % 2."""
        if self.feat is None:
            return
        pending = self._done[self.k % 2]
        if pending is not None:
            torch.cuda.current_stream(self.device).wait_event(pending)

    @property
    def feature_ready(self):
        """The event the step's blend waits for before reading the features
        (step k-1's feature update), or None."""
        return self._done[(self.k - 1) % 2] if self.feat is not None else None

    def grad_into(self, arg_names: Optional[Mapping[str, str]] = None) -> Dict[str, torch.Tensor]:
        """{name: view} destinations of this step's gradients, for the
        camera batch's backward (GaussianRasterizerBatch(...)(...,
        grad_into=...)); `arg_names` maps parameter names to the rasterizer's
        argument names.  Written whole by that backward: no zeroing."""
        out = {}
        for o, b in self._buffers():
            for n, v in o.grad_views(b).items():
                out[arg_names[n] if arg_names is not None else n] = v
        return out

    def bind_grads(self) -> None:
        """Every parameter's .grad becomes its (zeroed) view of this step's
        buffers: autograd accumulates the step's gradients into them."""
        for o, b in self._buffers():
            o.bind(b)
            o.zero_grad(b)
        self._bound = True

    @torch.no_grad()
    def load_grads(self) -> List[bool]:
        """Move the parameters' unbound .grad (from any autograd path) into
        this step's buffers and clear them; returns per parameter (names
        order of `params`) whether it had a gradient."""
        flags = {}
        for o, b in self._buffers():
            views = o.grad_views(b)
            for n, p in zip(o.names, o.params):
                g = p.grad
                flags[n] = g is not None
                if g is None:
                    views[n].zero_()
                else:
                    views[n].copy_(g)
                p.grad = None
        return [flags[n] for n in self.params]

    def _split(self, lr, reached):
        """Per-optimizer reach flags from flags in `params` order."""
        if reached is None:
            return [None for _ in self.opts]
        by_name = dict(zip(self.params, reached))
        return [[bool(by_name[n]) for n in o.names] for o in self.opts]

    def finish(self, lr: Optional[Mapping[str, float]] = None, reached: Optional[Sequence[bool]] = None,
               inline: bool = False) -> None:
        """The optimizer step of step k (geometry in line; with `overlap`
        and not `inline`, the features behind the next step).  `lr`,
        `reached`: as ShardedAdam.update (reached in `params` order)."""
        rg = self._split(lr, reached)
        if self._bound:  # the views stay the gradients' home only for this step
            for o in self.opts:
                for p in o.params:
                    p.grad = None
            self._bound = False
        if self.feat is None:
            self.geo.step(0, lr, rg[0])
            self.k += 1
            return
        kb = self.k % 2
        self.geo.step(0, lr, rg[0])
        if inline:
            self.feat.step(kb, lr, rg[1])
            self._done[kb] = None
            self.k += 1
            return
        main = torch.cuda.current_stream(self.device)
        work = self.feat.reduce_scatter(kb, async_op=True)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            if work is not None:
                work.wait()
            self.feat.update(kb, lr, rg[1])
            self.feat.all_gather()
            ev = torch.cuda.Event()
            ev.record(self.side)
        self._done[kb] = ev
        self.k += 1

    def drain(self) -> None:
        """The current stream waits for every pending feature update."""
        if self.feat is None:
            return
        cur = torch.cuda.current_stream(self.device)
        for ev in self._done:
            if ev is not None:
                cur.wait_event(ev)

    # ------------------------------------------------------------ state
    def load_state(self, optimizer) -> None:
        for o in self.opts:
            o.load_state(optimizer)

    def export_state(self, optimizer) -> None:
        """Full moments and step counts into optimizer.state (a collective)."""
        self.drain()
        for o in self.opts:
            o.export_state(optimizer)

    def replace(self, name: str, tensor: torch.Tensor, reset_moments: bool = True) -> None:
        self.drain()
        for o in self.opts:
            if name in o.names:
                o.replace(name, tensor, reset_moments)
                return
        raise KeyError(name)
