"""Multi-process (gloo, CPU) tests of the camera-sharded data-parallel step:
the flat-bucket all-reduce must equal the sum of per-rank (per-camera)
gradients, max_2D_radius reduces with MAX, and camera sharding is a partition.
RCCL is exercised only by the GPU bench (bench.py --gpus N under torchrun)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dynamic3dgaussians_amd.distributed import GradBucket, all_reduce_max_, shard_cameras


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        P = 1000
        params = [torch.zeros(P, 3, requires_grad=True), torch.zeros(P, 4, requires_grad=True),
                  torch.zeros(P, 1, requires_grad=True), torch.zeros(P, 32, requires_grad=True)]
        cams = shard_cameras(27, rank, world)
        # per-camera gradient = deterministic function of the camera id
        for p in params:
            p.grad = torch.zeros_like(p)
        for c in cams:
            g = torch.Generator().manual_seed(100 + c)
            for p in params:
                p.grad += torch.randn(p.shape, generator=g)
        accum = torch.full((P,), float(rank + 1))
        bucket = GradBucket(params, extras={"means2D_gradient_accum": accum})
        bucket.all_reduce()
        radius = torch.arange(P, dtype=torch.float32) * (rank + 1)
        all_reduce_max_(radius)
        q.put((rank, [p.grad.clone() for p in params], accum.clone(), radius.clone(), cams))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bucket_all_reduce_equals_sum_of_camera_grads(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    # single-process reference: sum over all 27 cameras
    P = 1000
    shapes = [(P, 3), (P, 4), (P, 1), (P, 32)]
    ref = [torch.zeros(s) for s in shapes]
    for c in range(27):
        g = torch.Generator().manual_seed(100 + c)
        for r, s in zip(ref, shapes):
            r += torch.randn(s, generator=g)
    all_cams = sorted(c for r in res for c in r[4])
    assert all_cams == list(range(27))
    for rank, grads, accum, radius, _ in res:
        for a, b in zip(grads, ref):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
        assert torch.all(accum == sum(range(1, world + 1)))
        torch.testing.assert_close(radius, torch.arange(P, dtype=torch.float32) * world)


def test_shard_cameras_partition():
    for world in (1, 2, 4, 8):
        parts = [shard_cameras(27, r, world) for r in range(world)]
        flat = sorted(c for p in parts for c in p)
        assert flat == list(range(27))
        assert max(len(p) for p in parts) - min(len(p) for p in parts) <= 1


def test_bucket_noop_without_process_group():
    p = torch.zeros(5, requires_grad=True)
    p.grad = torch.ones(5)
    GradBucket([p]).all_reduce()
    assert torch.all(p.grad == 1)
