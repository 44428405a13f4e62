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
    fp32 buffer (plus extra per-Gaussian statistics), all-reduces it with one
    collective and scatters the result back."""

    def __init__(self, params: Iterable[torch.Tensor], extras: Dict[str, torch.Tensor] | None = None):
        self.params = [p for p in params]
        self.extras = dict(extras or {})
        sizes = [p.numel() for p in self.params] + [t.numel() for t in self.extras.values()]
        self.sizes = sizes
        dev = self.params[0].device
        self.flat = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)

    def pack(self):
        o = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                self.flat[o:o + n].zero_()
            else:
                self.flat[o:o + n].copy_(p.grad.reshape(-1))
            o += n
        for t in self.extras.values():
            n = t.numel()
            self.flat[o:o + n].copy_(t.reshape(-1))
            o += n

    def unpack(self):
        o = 0
        for p in self.params:
            n = p.numel()
            if p.grad is None:
                p.grad = torch.empty_like(p)
            p.grad.reshape(-1).copy_(self.flat[o:o + n])
            o += n
        for t in self.extras.values():
            n = t.numel()
            t.reshape(-1).copy_(self.flat[o:o + n])
            o += n

    def all_reduce(self, group=None):
        """pack -> one all_reduce(SUM) -> unpack.  No-op without a process group."""
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
            return
        self.pack()
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=group)
        self.unpack()


def all_reduce_max_(t: torch.Tensor, group=None) -> torch.Tensor:
    """In-place MAX all-reduce (max_2D_radius)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t
