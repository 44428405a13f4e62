"""Per-timestep training driver for the camera-sharded step (BASELINE.json
configs[3]: the rig's cameras sharded over N ranks, T timesteps).

The reference trains a sequence timestep by timestep (train.py:392-432):
timestep 0 from the initial point cloud, every later timestep initialised
from the previous one by a constant-velocity extrapolation of the means and
rotations (`initialize_per_timestep`, train.py:294-314, with the optimizer
moments of the replaced tensors reset by `update_params_and_optimizer`,
external.py:143-155), and after timestep 0 the foreground neighbour graph
is built once (`initialize_post_first_timestep`, train.py:316-341).  Inside a
timestep it draws one camera per optimizer step (train.py:82-87, 422-433).

`TimestepDriver` runs the same loop with the multi-camera step of
SURVEY.md 8(e): every iteration renders ALL of the rig's cameras, camera c
on rank c mod N (distributed.shard_cameras), each rank's cameras as one
GaussianRasterizerBatch launch per stage; the per-Gaussian gradients and the
densification statistics travel in ONE GradBucket all_reduce(SUM) and
max_2D_radius in one all_reduce(MAX), then every rank takes the identical
optimizer step.  The loss is the mean over all rig cameras of a per-camera
image loss, so the summed gradient is the gradient of that mean whatever N
is; losses that do not render (neighbour terms, floor, background) are
computed identically on every rank and enter with weight 1/N so the SUM
counts them once.

The default image loss is the L1 term of the reference's photometric loss
(train.py:187, `l1_loss_v1` helpers.py:110-111); SSIM, masks, per-camera colour correction and
the neighbour losses (neighbor.neighbor_losses) are the caller's to pass as
`image_loss` / `extra_loss` -- they are not on the rasterizer path.
Densification at timestep 0 (external.py:215-292) is likewise the caller's
`densify` callback: it replaces tensors (variables[...] and the optimizer's
Parameters), after which the driver builds a new bucket.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from .distributed import GradBucket, ShardedStep, StaleBucketError, all_reduce_max_, shard_cameras

STATS = ("means2D_gradient_accum", "denom", "max_2D_radius")


def params2rendervar(params: Dict[str, torch.Tensor]) -> dict:
    """helpers.py:98-107: the rasterizer inputs of the Dynamic3DGaussians
    parameterisation (precomputed colours, normalised quaternions,
    sigmoid opacities, exp scales, a fresh means2D leaf)."""
    rv = {
        "means3D": params["means3D"],
        "colors_precomp": params["rgb_colors"],
        "rotations": torch.nn.functional.normalize(params["unnorm_rotations"]),
        "opacities": torch.sigmoid(params["logit_opacities"]),
        "scales": torch.exp(params["log_scales"]),
        "means2D": torch.zeros_like(params["means3D"], requires_grad=True),
    }
    if "semantic_feature" in params:  # the FSGS rasterizer's feature channels (G3 call)
        rv["semantic_feature"] = params["semantic_feature"]
    return rv


def update_params_and_optimizer(new_params: Dict[str, torch.Tensor], params: dict, optimizer) -> dict:
    """external.py:143-155: bind each new tensor as a fresh Parameter in its
    optimizer group (found by the group's 'name') and in `params`, with zeroed
    Adam moments and the step count kept."""
    for k, v in new_params.items():
        group = [g for g in optimizer.param_groups if g["name"] == k][0]
        old = group["params"][0]
        state = optimizer.state.pop(old, None)
        p = torch.nn.Parameter(v.detach().requires_grad_(True))
        group["params"][0] = p
        if state is not None:
            state["exp_avg"] = torch.zeros_like(v)
            state["exp_avg_sq"] = torch.zeros_like(v)
            optimizer.state[p] = state
        params[k] = p
    return params


def _fg_mask(params: dict) -> torch.Tensor:
    """train.py:299: foreground = seg_colors[:, 0] > 0.5 (every Gaussian when
    the parameterisation carries no seg colours)."""
    if "seg_colors" in params:
        return (params["seg_colors"][:, 0] > 0.5).detach()
    return torch.ones(params["means3D"].shape[0], dtype=torch.bool, device=params["means3D"].device)


def initialize_per_timestep(params: dict, variables: dict, optimizer) -> tuple:
    """train.py:294-314: constant-velocity initialisation of timestep t from
    t-1 and t-2 (means and normalised rotations), the previous timestep's
    state kept in `variables` for the neighbour / colour losses."""
    pts = params["means3D"]
    rot = torch.nn.functional.normalize(params["unnorm_rotations"])
    new_pts = pts + (pts - variables["prev_pts"])
    new_rot = torch.nn.functional.normalize(rot + (rot - variables["prev_rot"]))
    is_fg = _fg_mask(params)
    prev_inv_rot_fg = rot[is_fg].clone()
    prev_inv_rot_fg[:, 1:] = -1 * prev_inv_rot_fg[:, 1:]
    variables["prev_inv_rot_fg"] = prev_inv_rot_fg.detach()
    if "neighbor_indices" in variables:
        fg_pts = pts[is_fg]
        variables["prev_offset"] = (fg_pts[variables["neighbor_indices"]] - fg_pts[:, None]).detach()
    variables["prev_pts"] = pts.detach()
    variables["prev_rot"] = rot.detach()
    variables["prev_col"] = params["rgb_colors"].detach()
    params = update_params_and_optimizer({"means3D": new_pts, "unnorm_rotations": new_rot}, params, optimizer)
    return params, variables


def initialize_post_first_timestep(params: dict, variables: dict, optimizer, num_knn: int = 20,
                                   knn_fn: Optional[Callable] = None,
                                   params_to_fix: Sequence[str] = ("logit_opacities", "log_scales", "cam_m", "cam_c")
                                   ) -> dict:
    """train.py:316-341: the foreground k-nearest-neighbour graph with its
    weights exp(-2000 d^2) and distances (knn_fn(points, k) -> (sq_dist,
    indices); default knn.o3d_knn, the HIP search), the background's initial
    means / rotations, prev_pts / prev_rot, and lr = 0 for the fixed groups."""
    is_fg = _fg_mask(params)
    fg_pts = params["means3D"][is_fg].detach()
    if knn_fn is None:
        from .knn import o3d_knn as knn_fn
    sq, idx = knn_fn(fg_pts, num_knn)
    sq = torch.as_tensor(sq, device=fg_pts.device, dtype=torch.float32)
    variables["neighbor_indices"] = torch.as_tensor(idx, device=fg_pts.device).long().contiguous()
    variables["neighbor_weight"] = torch.exp(-2000 * sq).contiguous()
    variables["neighbor_dist"] = torch.sqrt(sq).contiguous()
    variables["init_bg_pts"] = params["means3D"][~is_fg].detach()
    variables["init_bg_rot"] = torch.nn.functional.normalize(params["unnorm_rotations"][~is_fg]).detach()
    variables["prev_pts"] = params["means3D"].detach()
    variables["prev_rot"] = torch.nn.functional.normalize(params["unnorm_rotations"]).detach()
    for g in optimizer.param_groups:
        if g.get("name") in params_to_fix:
            g["lr"] = 0.0
    return variables


def l1_image_loss(im, target) -> torch.Tensor:
    """helpers.py:110-111 l1_loss_v1 of every camera of a batch, summed:
    im, target [C, 3, H, W] -> sum_c mean |im_c - target_c| (one expression
    over the batch instead of C small ones).  With feature channels (a
    batch_renderer over parameters holding semantic_feature) im and target
    are (images, feature maps) pairs and the two L1 terms are added."""
    if isinstance(im, (tuple, list)):
        return sum(l1_image_loss(a, b) for a, b in zip(im, target))
    return torch.abs(im - target).mean(dim=(-3, -2, -1)).sum()


def batch_renderer(settings_all: Sequence):
    """The default `render`: GaussianRasterizerBatch over the given cameras
    (one launch per stage), densification statistics tracked.  Returns
    render(rendervar, cams, feature_ready=None) -> (images [C, 3, H, W],
    stats dict or None); with semantic_feature in the rendervar (the G3 call,
    label + features) the images are (colour [C, 3, H, W], features
    [C, F, H, W]) and the blend waits for `feature_ready` (ShardedStep's
    overlapped feature update) before reading the features."""
    from .rasterizer import GaussianRasterizerBatch
    cache = {}

    def render(rv, cams: List[int], feature_ready=None):
        key = tuple(cams)
        if key not in cache:
            cache[key] = GaussianRasterizerBatch([settings_all[c] for c in cams], track_densify=True)
        ras = cache[key]
        if "semantic_feature" in rv:  # label=None: every Gaussian's gradients kept (the G3 call's ones)
            im, _radius, feat, _depth, _alpha = ras(**rv, label=None, feature_ready=feature_ready)
            return (im, feat), ras.densify_stats
        im, _radius, _depth = ras(**rv)  # G1 call (train.py:142)
        return im, ras.densify_stats

    return render


class TimestepDriver:
    """One rank of the camera-sharded per-timestep training loop.

    params / variables / optimizer: the reference's dicts and optimizer
    (param groups named after the parameters, train.py:119-135); FusedAdam
    or torch.optim.Adam.  `n_cams`: cameras of the rig; this rank renders
    shard_cameras(n_cams, rank, world).  `image_loss(images, targets)` maps
    the rank's [C, 3, H, W] renders and targets to the SUM of its cameras'
    losses.  `render(rendervar, cams)` returns the
    cameras' images [C, 3, H, W] and optional densification statistics
    (default: batch_renderer(settings_all)).  `targets(t)` -> [n_cams, 3, H, W]
    images of timestep t, or only this rank's cameras' [C_rank, 3, H, W] with
    `targets_sharded=True` (a tuple of such tensors, e.g. images and feature
    maps, when the render returns a tuple).

    The optimizer step.  Two paths, the same arithmetic:
      * plain: ONE GradBucket all_reduce(SUM) of every gradient and the
        statistics, then `optimizer.step()` on every rank;
      * sharded (`sharded=True`; the default for world > 1 with device
        parameters): distributed.ShardedStep -- reduce-scatter, Adam on the
        rank's 1/N of the parameters (the fused HIP kernel), all-gather -- and,
        when the parameters hold `semantic_feature` (rendered through the G3
        call), the feature exchange and update behind the next step's
        projection and binning (its blend waits for them, `feature_ready`).
        The statistics and the reached-parameter flags travel in one small
        all_reduce.  While it is active the ShardedStep holds the Adam state:
        it is loaded from `optimizer` when the sharded step starts (and
        whenever a parameter was replaced from outside the driver), the
        per-timestep re-initialisation rebinds the replaced tensors in place
        with zeroed moments (update_params_and_optimizer, external.py:143-155),
        the learning rates are read from optimizer.param_groups every step,
        and sync_optimizer() (called at the end of run()) writes the state
        back into `optimizer`.  Densification (external.py:215-292, timestep
        0 only, train.py:436) does state surgery on the reference optimizer:
        the steps of timestep 0 take the plain path when a `densify` callback
        is given.
    `sharded` may also be a factory(params, lr, rank, world, group) ->
    ShardedStep (e.g. with a substituted update for CPU tests).

    Densification statistics: the loss divides every camera's image loss by
    n_cams (the rig's mean), so each camera's means2D gradient is 1/n_cams of
    a one-camera-per-step gradient (train.py:422-425); the statistic
    external.py:136-140 accumulates is the NORM of that gradient (compared
    with an absolute threshold, external.py:247-259), so the driver scales
    the increments by `stat_scale` (default n_cams): means2D_gradient_accum
    then holds per-view norms of an image loss of weight 1 that is the only
    term reaching means2D -- the loss of dyn_train.py (loss_weights['im'] =
    1).  The shipped train.py differs: it sets loss_weights['im'] = 0.0
    (train.py:284), and its means2D gradient comes from stat_im (weight
    0.01, averaged over the stat cameras sharing one means2D,
    train.py:186-243) plus depth; a caller reproducing that weighting
    passes its own `stat_scale`.  That train.py variant is parity unpinned:
    the reference ships no fixture of its statistics."""

    def __init__(self, params: dict, variables: dict, optimizer, n_cams: int, render: Callable,
                 rank: int = 0, world: int = 1, group=None,
                 image_loss: Callable = l1_image_loss, extra_loss: Optional[Callable] = None,
                 densify: Optional[Callable] = None, targets_sharded: bool = False,
                 stat_scale: Optional[float] = None, sharded=None):
        self.params, self.variables, self.optimizer = params, variables, optimizer
        self.n_cams = n_cams
        self.stat_scale = float(n_cams if stat_scale is None else stat_scale)
        self.targets_sharded = targets_sharded
        self.cams = shard_cameras(n_cams, rank, world)
        self.rank, self.world, self.group = rank, world, group
        self.render = render
        self.image_loss, self.extra_loss, self.densify = image_loss, extra_loss, densify
        dev = params["means3D"].device
        P = params["means3D"].shape[0]
        for k in STATS:
            if k not in variables:
                variables[k] = torch.zeros(P, dtype=torch.float32, device=dev)
        if sharded is None:
            sharded = world > 1 and dev.type == "cuda"
        self._sharded_factory = sharded if callable(sharded) else (self._default_sharded if sharded else None)
        self.zs: Optional[ShardedStep] = None
        self._stats = None
        self.bucket = None  # the plain path's, built at its first step

    # ------------------------------------------------------------ buckets
    def _keys(self):
        """The optimizer's parameters (seg_colors and other constants stay out)."""
        names = {g.get("name") for g in self.optimizer.param_groups}
        return [k for k in self.params if k in names]

    def _new_bucket(self):
        # the replaced bucket's reach hooks come off the parameters that
        # survive (GradBucket.close)
        if self.bucket is not None:
            self.bucket.close()
        # bound .grad views only when there is an exchange (N = 1: autograd
        # hands the backward's tensors to the leaves, no accumulate kernels)
        self.bucket = GradBucket(self.params, extras_from=(self.variables, list(STATS[:2])),
                                 bind_grads=self.world > 1,
                                 keys=self._keys(), track_reached=True)

    def _live_bucket(self):
        try:
            if self.bucket is None:
                raise StaleBucketError("no bucket")
            self.bucket.check_live()
        except StaleBucketError:
            self._new_bucket()
        return self.bucket

    def _lrs(self) -> Dict[str, float]:
        return {g["name"]: float(g["lr"]) for g in self.optimizer.param_groups if "name" in g}

    def _default_sharded(self, params, lr, rank, world, group):
        return ShardedStep(params, lr, rank=rank, world=world, group=group,
                           eps=float(self.optimizer.param_groups[0].get("eps", 1e-15)),
                           betas=tuple(self.optimizer.param_groups[0].get("betas", (0.9, 0.999))))

    def _sharded_on(self, t: int) -> bool:
        return self._sharded_factory is not None and not (t == 0 and self.densify is not None)

    def _live_sharded(self) -> ShardedStep:
        keys = self._keys()
        zs = self.zs
        if zs is not None:
            held = zs.params
            if list(held) != keys or any(self.params[k] is not held[k] for k in keys):
                zs.drain()
                zs = None  # a parameter replaced outside the driver: start again from the optimizer
        if zs is None:
            zs = self._sharded_factory({k: self.params[k] for k in keys}, self._lrs(), self.rank, self.world,
                                       self.group)
            zs.load_state(self.optimizer)
            self.zs = zs
        if self._stats is not None:
            try:
                self._stats.check_live()
            except StaleBucketError:
                self._stats = None
        if self._stats is None or self._stats.n_aux != len(keys):
            self._stats = GradBucket([], extras_from=(self.variables, list(STATS[:2])), n_aux=len(keys))
        return zs

    def sync_optimizer(self) -> None:
        """Write the sharded step's Adam state (moments, step counts) back
        into the reference optimizer (a collective at N > 1: every rank
        calls it).  No-op on the plain path."""
        if self.zs is not None:
            self.zs.export_state(self.optimizer)

    # ------------------------------------------------------------ a step
    def _loss(self, rv, targets, t, feature_ready=None):
        loss = None
        stats = None
        if self.cams:
            if feature_ready is not None:
                im, stats = self.render(rv, self.cams, feature_ready=feature_ready)
            else:
                im, stats = self.render(rv, self.cams)
            lead = targets[0] if isinstance(targets, (tuple, list)) else targets
            want = len(self.cams) if self.targets_sharded else self.n_cams
            if lead.shape[0] != want:
                raise ValueError(f"targets hold {lead.shape[0]} images; expected {want} "
                                 f"({'this rank' if self.targets_sharded else 'the rig'}'s cameras)")
            if self.targets_sharded or len(self.cams) == self.n_cams:
                tg = targets
            elif isinstance(targets, (tuple, list)):
                tg = type(targets)(x[self.cams] for x in targets)
            else:
                tg = targets[self.cams]
            loss = self.image_loss(im, tg) / self.n_cams
        if self.extra_loss is not None:
            le = self.extra_loss(self.params, self.variables, rv, t) / self.world
            loss = le if loss is None else loss + le
        return loss, stats

    def _add_stats(self, stats):
        v = self.variables
        if stats is not None:
            # this rank's cameras' statistics (external.py:136-140,
            # train.py:288-290); the bucket sums the increments
            v["means2D_gradient_accum"] += stats["means2D_gradient_accum"] * self.stat_scale
            v["denom"] += stats["denom"]
            torch.maximum(v["max_2D_radius"], stats["max_2D_radius"], out=v["max_2D_radius"])

    def step(self, targets, t: int = 0, i: int = 0) -> float:
        """One optimizer step over the whole rig.  Returns this rank's share of
        the loss (summed over the ranks: the step's loss)."""
        if self._sharded_on(t):
            return self._step_sharded(targets, t, i)
        if self.zs is not None:  # leaving the sharded step: the optimizer takes its state back
            self.sync_optimizer()
            self.zs = None
        bucket = self._live_bucket()
        bucket.zero_grad()
        rv = params2rendervar(self.params)
        loss, stats = self._loss(rv, targets, t)
        if loss is not None:
            loss.backward()
        with torch.no_grad():
            self._add_stats(stats)
            bucket.all_reduce(self.group)
            all_reduce_max_(self.variables["max_2D_radius"], self.group)
            if t == 0 and self.densify is not None:
                # external.py:215-292 with the statistics already accumulated
                # above (the caller's densify skips accumulate_mean2d_gradient).
                # Tensors it replaces come back as new Parameters without
                # .grad, which the step below skips, as in the reference; the
                # next step() sees the stale bucket and builds a new one.
                self.params, self.variables = self.densify(self.params, self.variables, self.optimizer, i)
            self.optimizer.step()
        return float(loss.detach()) if loss is not None else 0.0

    def _drop_bucket(self):
        """Leaving the plain path: its bound .grad views come off the
        parameters (the sharded step reads unbound gradients)."""
        if self.bucket is not None:
            self.bucket.close()
            for k in self._keys():
                self.params[k].grad = None
            self.bucket = None

    def _step_sharded(self, targets, t: int, i: int) -> float:
        self._drop_bucket()
        zs = self._live_sharded()
        zs.begin()
        rv = params2rendervar(self.params)
        loss, stats = self._loss(rv, targets, t, zs.feature_ready)
        if loss is not None:
            loss.backward()
        with torch.no_grad():
            reached = zs.load_grads()
            self._add_stats(stats)
            flags = torch.tensor([1.0 if r else 0.0 for r in reached], dtype=torch.float32,
                                 device=self.params["means3D"].device)
            self._stats.all_reduce(self.group, aux=flags)
            all_reduce_max_(self.variables["max_2D_radius"], self.group)
            # a parameter is updated iff some rank's loss reached it (the plain
            # path's GradBucket reach tracking); the summed flags are read only
            # when this rank's loss missed one
            union = None if all(reached) else (flags > 0).tolist()
            zs.finish(lr=self._lrs(), reached=union)
        return float(loss.detach()) if loss is not None else 0.0

    def timestep(self, t: int, iters: int, targets: torch.Tensor) -> List[float]:
        """train.py:411-433 for one timestep (timestep t > 0 is initialised
        from t-1 and t-2 first)."""
        if t > 0:
            zs = self.zs if self._sharded_on(t) else None
            if zs is not None:
                zs.drain()  # the features are not touched, but the exchange's buffers are left settled
            self.params, self.variables = initialize_per_timestep(self.params, self.variables, self.optimizer)
            if zs is not None:
                # the replaced means / rotations keep their flat storage; zeroed
                # moments, step counts kept (update_params_and_optimizer)
                for k in ("means3D", "unnorm_rotations"):
                    if k in zs.params:
                        zs.replace(k, self.params[k], reset_moments=True)
            else:
                self._drop_bucket()  # built again at the next plain step
        return [self.step(targets, t, i) for i in range(iters)]

    def run(self, n_timesteps: int, iters: Callable[[int], int], targets: Callable[[int], torch.Tensor],
            post_first: Optional[Callable] = None) -> List[List[float]]:
        """The whole sequence; `post_first(params, variables, optimizer)` runs
        after timestep 0 (default: nothing -- pass a wrapper of
        initialize_post_first_timestep to build the neighbour graph).  The
        optimizer holds the final Adam state on return (sync_optimizer)."""
        losses = []
        for t in range(n_timesteps):
            losses.append(self.timestep(t, iters(t), targets(t)))
            if t == 0:
                if post_first is not None:
                    self.variables = post_first(self.params, self.variables, self.optimizer)
                elif "prev_pts" not in self.variables:
                    self.variables["prev_pts"] = self.params["means3D"].detach()
                    self.variables["prev_rot"] = torch.nn.functional.normalize(
                        self.params["unnorm_rotations"]).detach()
        self.sync_optimizer()
        return losses


def world_info(group=None):
    """(rank, world) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1
