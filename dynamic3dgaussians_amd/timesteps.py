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

from .distributed import GradBucket, StaleBucketError, all_reduce_max_, shard_cameras

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


def l1_image_loss(im: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """helpers.py:110-111 l1_loss_v1 of every camera of a batch, summed:
    im, target [C, 3, H, W] -> sum_c mean |im_c - target_c| (one expression
    over the batch instead of C small ones)."""
    return torch.abs(im - target).mean(dim=(-3, -2, -1)).sum()


def batch_renderer(settings_all: Sequence):
    """The default `render`: GaussianRasterizerBatch over the given cameras
    (one launch per stage), densification statistics tracked.  Returns
    render(rendervar, cams) -> (images [C, 3, H, W], stats dict or None)."""
    from .rasterizer import GaussianRasterizerBatch
    cache = {}

    def render(rv, cams: List[int]):
        key = tuple(cams)
        if key not in cache:
            cache[key] = GaussianRasterizerBatch([settings_all[c] for c in cams], track_densify=True)
        ras = cache[key]
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
    `targets_sharded=True`.

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
                 stat_scale: Optional[float] = None):
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
        self.bucket = None
        self._new_bucket()

    def _new_bucket(self):
        # the replaced bucket's reach hooks come off the parameters that
        # survive (GradBucket.close)
        if self.bucket is not None:
            self.bucket.close()
        # the optimizer's parameters (seg_colors and other constants stay out)
        names = {g.get("name") for g in self.optimizer.param_groups}
        keys = [k for k in self.params if k in names]
        # bound .grad views only when there is an exchange (N = 1: autograd
        # hands the backward's tensors to the leaves, no accumulate kernels)
        self.bucket = GradBucket(self.params, extras_from=(self.variables, list(STATS[:2])),
                                 bind_grads=self.world > 1,
                                 keys=keys, track_reached=True)

    def _live_bucket(self):
        try:
            self.bucket.check_live()
        except StaleBucketError:
            self._new_bucket()
        return self.bucket

    def step(self, targets: torch.Tensor, t: int = 0, i: int = 0) -> float:
        """One optimizer step over the whole rig.  Returns this rank's share of
        the loss (summed over the ranks: the step's loss)."""
        bucket = self._live_bucket()
        bucket.zero_grad()
        rv = params2rendervar(self.params)
        loss = None
        stats = None
        if self.cams:
            im, stats = self.render(rv, self.cams)
            want = len(self.cams) if self.targets_sharded else self.n_cams
            if targets.shape[0] != want:
                raise ValueError(f"targets hold {targets.shape[0]} images; expected {want} "
                                 f"({'this rank' if self.targets_sharded else 'the rig'}'s cameras)")
            tg = targets if (self.targets_sharded or len(self.cams) == self.n_cams) else targets[self.cams]
            loss = self.image_loss(im, tg) / self.n_cams
        if self.extra_loss is not None:
            le = self.extra_loss(self.params, self.variables, rv, t) / self.world
            loss = le if loss is None else loss + le
        if loss is not None:
            loss.backward()
        with torch.no_grad():
            v = self.variables
            if stats is not None:
                # this rank's cameras' statistics (external.py:136-140,
                # train.py:288-290); the bucket sums the increments
                v["means2D_gradient_accum"] += stats["means2D_gradient_accum"] * self.stat_scale
                v["denom"] += stats["denom"]
                torch.maximum(v["max_2D_radius"], stats["max_2D_radius"], out=v["max_2D_radius"])
            bucket.all_reduce(self.group)
            all_reduce_max_(v["max_2D_radius"], self.group)
            if t == 0 and self.densify is not None:
                # external.py:215-292 with the statistics already accumulated
                # above (the caller's densify skips accumulate_mean2d_gradient).
                # Tensors it replaces come back as new Parameters without
                # .grad, which the step below skips, as in the reference; the
                # next step() sees the stale bucket and builds a new one.
                self.params, self.variables = self.densify(self.params, self.variables, self.optimizer, i)
            self.optimizer.step()
        return float(loss.detach()) if loss is not None else 0.0

    def timestep(self, t: int, iters: int, targets: torch.Tensor) -> List[float]:
        """train.py:411-433 for one timestep (timestep t > 0 is initialised
        from t-1 and t-2 first)."""
        if t > 0:
            self.params, self.variables = initialize_per_timestep(self.params, self.variables, self.optimizer)
            self._new_bucket()
        return [self.step(targets, t, i) for i in range(iters)]

    def run(self, n_timesteps: int, iters: Callable[[int], int], targets: Callable[[int], torch.Tensor],
            post_first: Optional[Callable] = None) -> List[List[float]]:
        """The whole sequence; `post_first(params, variables, optimizer)` runs
        after timestep 0 (default: nothing -- pass a wrapper of
        initialize_post_first_timestep to build the neighbour graph)."""
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
        return losses


def world_info(group=None):
    """(rank, world) of the default process group, (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1
