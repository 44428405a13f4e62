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

from typing import Dict, Iterable, List

import torch
import torch.distributed as dist


def shard_cameras(n_cams: int, rank: int, world: int) -> List[int]:
    """Camera c goes to rank c mod world."""
    return [c for c in range(n_cams) if c % world == rank]


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
    the extras identically on every rank outside a step (e.g. the
    densification reset of the accumulators, external.py:237-240).
    """

    def __init__(self, params: Iterable[torch.Tensor], extras: Dict[str, torch.Tensor] | None = None):
        self.params = [p for p in params]
        self.extras = dict(extras or {})
        sizes = [p.numel() for p in self.params] + [t.numel() for t in self.extras.values()]
        self.sizes = sizes
        dev = self.params[0].device
        self.flat = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)
        self._base = {}
        self.resync()

    def resync(self) -> None:
        """Record the extras' current values as the common starting point of
        the next step (they must be identical on every rank)."""
        self._base = {k: t.detach().clone() for k, t in self.extras.items()}

    def pack(self):
        o = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.flat[o:o + n].zero_()
            else:
                self.flat[o:o + n].copy_(p.grad.reshape(-1))
            o += n
        for k, t in self.extras.items():
            n = t.numel()
            # this rank's increment since the last synchronisation point
            torch.sub(t.reshape(-1), self._base[k].reshape(-1), out=self.flat[o:o + n])
            o += n

    def unpack(self):
        o = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.reshape(-1).copy_(self.flat[o:o + n])
            o += n
        for k, t in self.extras.items():
            n = t.numel()
            # common start + every rank's increment
            torch.add(self._base[k].reshape(-1), self.flat[o:o + n], out=t.reshape(-1))
            o += n

    def all_reduce(self, group=None):
        """pack -> one all_reduce(SUM) -> unpack.  Without a process group
        (or with one rank) the values stay as they are."""
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
            self.resync()
            return
        self.pack()
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.unpack()
        self.resync()


def all_reduce_max_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place MAX all-reduce (max_2D_radius)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t
