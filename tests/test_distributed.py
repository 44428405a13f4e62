"""Multi-process (gloo, CPU) tests of the camera-sharded data-parallel step:
the flat-bucket all-reduce must equal the sum of per-rank (per-camera)
gradients, max_2D_radius reduces with MAX, and camera sharding is a partition.
RCCL is exercised only by the GPU bench (bench.py --gpus N under torchrun)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dynamic3dgaussians_amd.distributed import GradBucket, StaleBucketError, all_reduce_max_, shard_cameras


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cam_norms(c, P):
    """Stand-in for one camera's |dL/dmeans2D| contributions (deterministic
    in the camera id)."""
    return torch.rand(P, generator=torch.Generator().manual_seed(500 + c))


def _worker(rank, world, port, q, bind=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        P = 1000
        params = [torch.zeros(P, 3, requires_grad=True), torch.zeros(P, 4, requires_grad=True),
                  torch.zeros(P, 1, requires_grad=True), torch.zeros(P, 32, requires_grad=True)]
        cams = shard_cameras(27, rank, world)
        # densification statistics: running totals, identical on every rank
        # at the start of the step; each rank adds its own cameras
        accum = torch.full((P,), 0.5)
        denom = torch.full((P,), 2.0)
        extras = {"means2D_gradient_accum": accum, "denom": denom}
        if bind:
            # gradients accumulate straight into the bucket's flat buffer
            bucket = GradBucket(params, extras=extras, bind_grads=True)
            bucket.zero_grad()
        else:
            for p in params:
                p.grad = torch.zeros_like(p)
        # per-camera gradient = deterministic function of the camera id
        for c in cams:
            g = torch.Generator().manual_seed(100 + c)
            for p in params:
                p.grad += torch.randn(p.shape, generator=g)
        if bind:
            assert params[1].grad.data_ptr() == bucket.flat[3 * P:].data_ptr()
        else:
            bucket = GradBucket(params, extras=extras)
        for c in cams:
            accum += _cam_norms(c, P)
            denom += (_cam_norms(c, P) > 0.5).float()
        bucket.all_reduce()
        radius = torch.arange(P, dtype=torch.float32) * (rank + 1)
        all_reduce_max_(radius)
        # numpy copies: tensors would travel as shared-memory handles that die
        # with this process
        q.put((rank, [p.grad.numpy().copy() for p in params], (accum.numpy().copy(), denom.numpy().copy()),
               radius.numpy().copy(), cams))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bind", [(2, False), (3, False), (2, True)])
def test_bucket_all_reduce_equals_sum_of_camera_grads(world, bind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, bind)) for r in range(world)]
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
        grads = [torch.from_numpy(g) for g in grads]
        accum = [torch.from_numpy(a) for a in accum]
        radius = torch.from_numpy(radius)
        for a, b in zip(grads, ref):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
        ref_acc = torch.full((P,), 0.5) + sum(_cam_norms(c, P) for c in range(27))
        ref_den = torch.full((P,), 2.0) + sum((_cam_norms(c, P) > 0.5).float() for c in range(27))
        torch.testing.assert_close(accum[0], ref_acc, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(accum[1], ref_den, rtol=0, atol=0)
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


def _multistep_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        P = 257
        p = torch.zeros(P, 3, requires_grad=True)
        accum, denom = torch.zeros(P), torch.zeros(P)
        bucket = GradBucket([p], extras={"accum": accum, "denom": denom})
        hist = []
        for step in range(3):
            cams = [step * 27 + c for c in shard_cameras(27, rank, world)]
            p.grad = torch.zeros_like(p)
            for c in cams:
                p.grad += _cam_norms(c, P)[:, None]
                accum += _cam_norms(c, P)
                denom += 1.0
            bucket.all_reduce()
            if step == 1:
                # an in-place reset of some accumulators, identical on every
                # rank, between steps -> resync (the reference's own reset binds
                # new tensors instead: test_bucket_detects_replaced_statistics)
                accum[::3] = 0.0
                denom[::3] = 0.0
                bucket.resync()
            hist.append((p.grad.numpy().copy(), accum.numpy().copy(), denom.numpy().copy()))
        q.put((rank, hist))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_bucket_statistics_over_steps_match_single_process(world):
    """Running densification statistics over several steps (with a reset in
    between) equal the single-process accumulation over all cameras: the
    bucket must sum per-step increments, not the totals."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multistep_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    P = 257
    accum, denom = torch.zeros(P), torch.zeros(P)
    ref = []
    for step in range(3):
        g = torch.zeros(P, 3)
        for c in range(step * 27, step * 27 + 27):
            g += _cam_norms(c, P)[:, None]
            accum += _cam_norms(c, P)
            denom += 1.0
        if step == 1:
            accum[::3] = 0.0
            denom[::3] = 0.0
        ref.append((g, accum.clone(), denom.clone()))
    for _, hist in res:
        for (g, a, d), (rg, ra, rd) in zip(hist, ref):
            g, a, d = torch.from_numpy(g), torch.from_numpy(a), torch.from_numpy(d)
            torch.testing.assert_close(g, rg, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(a, ra, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(d, rd, rtol=0, atol=0)


def test_bucket_detects_replaced_parameter():
    """Densification binds new Parameters (external.py:202-204, 273-275): a
    bucket built over the old ones must refuse to run, not silently reduce
    stale gradients."""
    params = {"means3D": torch.zeros(10, 3, requires_grad=True), "rgb": torch.zeros(10, 3, requires_grad=True)}
    b = GradBucket(params)
    b.all_reduce()  # live: fine
    params["means3D"] = torch.zeros(12, 3, requires_grad=True)
    with pytest.raises(StaleBucketError, match="means3D"):
        b.all_reduce()
    with pytest.raises(StaleBucketError):
        b.resync()
    # a same-object resize is caught too
    p = torch.zeros(10, requires_grad=True)
    b2 = GradBucket([p])
    p.data = torch.zeros(11)
    with pytest.raises(StaleBucketError, match="size"):
        b2.all_reduce()


def test_bucket_detects_replaced_statistics():
    """The densification reset binds new zero tensors into variables
    (external.py:273-275; remove_points at :202-204):
    a bucket tracking the old statistics must raise."""
    P = 10
    p = torch.zeros(P, requires_grad=True)
    variables = {"means2D_gradient_accum": torch.zeros(P), "denom": torch.zeros(P)}
    b = GradBucket([p], extras_from=(variables, ["means2D_gradient_accum", "denom"]))
    variables["denom"] += 1.0  # in place: still live
    b.all_reduce()
    variables["denom"] = torch.zeros(P)
    with pytest.raises(StaleBucketError, match="denom"):
        b.all_reduce()


def test_bound_gradients_accumulate_into_the_bucket():
    p = torch.ones(4, 3, requires_grad=True)
    q = torch.ones(5, requires_grad=True)
    b = GradBucket({"p": p, "q": q}, bind_grads=True)
    b.zero_grad()
    ((p * 2).sum() + (q * 3).sum()).backward()
    ((p * 1).sum()).backward()  # a second camera adds in place
    assert p.grad.data_ptr() == b.flat.data_ptr()
    assert torch.all(b.flat[:12] == 3) and torch.all(b.flat[12:] == 3)
    b.all_reduce()  # no process group: values unchanged, views intact
    assert torch.all(p.grad == 3)
    b.zero_grad()
    assert torch.all(b.flat == 0)
    p.grad = None  # what zero_grad(set_to_none=True) does
    with pytest.raises(StaleBucketError, match="zero_grad"):
        b.all_reduce()


def _reach_worker(rank, world, port, q):
    """a: reached on every rank; b: only on rank 0; c: on no rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a, b, c = (torch.nn.Parameter(torch.ones(5)) for _ in range(3))
        bucket = GradBucket({"a": a, "b": b, "c": c}, bind_grads=True, track_reached=True)
        out = []
        for step in range(2):
            bucket.zero_grad()
            bucket.check_live()
            loss = (a * (rank + 1)).sum()
            if rank == 0:
                loss = loss + 2 * b.sum()
            loss.backward()
            bucket.all_reduce()
            out.append([None if p.grad is None else p.grad.numpy().copy() for p in (a, b, c)])
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_bucket_unbinds_parameters_no_rank_reached():
    """with bound gradients every parameter has a .grad (a zero
    view) whether or not the loss reached it, so Adam would step unreached
    parameters on their old moments where one process leaves .grad None.
    track_reached=True: after the all-reduce a parameter reached by no rank
    has .grad None (the optimizer skips it), one reached by any rank keeps
    the summed gradient, and zero_grad() binds the gradients again."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reach_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        for ga, gb, gc in res[r]:
            assert (ga == 3.0).all()      # 1 + 2 from the two ranks
            assert (gb == 2.0).all()      # rank 0 only, still summed and bound
            assert gc is None             # no rank reached it


@pytest.mark.parametrize("n_cams,world,gx,gy", [(27, 8, 50, 50), (27, 2, 50, 50), (16, 8, 120, 68),
                                                 (3, 8, 120, 68), (5, 8, 4, 3)])
def test_shard_camera_windows_partition_every_camera(n_cams, world, gx, gy):
    """Image sharding of the rig: every camera's tile grid is covered exactly
    once over the ranks, whole cameras go c mod N, and the ranks' pixel
    shares differ by at most one tile row."""
    from dynamic3dgaussians_amd.distributed import shard_camera_windows
    cover = {c: [[0] * gx for _ in range(gy)] for c in range(n_cams)}
    load = []
    for r in range(world):
        sh = shard_camera_windows(n_cams, r, world, gx, gy)
        px = 0
        for c, w in sh:
            x0, y0, x1, y1 = w if w is not None else (0, 0, gx, gy)
            assert 0 <= x0 < x1 <= gx and 0 <= y0 < y1 <= gy
            for y in range(y0, y1):
                for x in range(x0, x1):
                    cover[c][y][x] += 1
            px += (x1 - x0) * (y1 - y0)
            if w is None:
                assert c % world == r
        load.append(px)
    assert all(v == 1 for c in cover for row in cover[c] for v in row)
    assert max(load) - min(load) <= gx


@pytest.mark.parametrize("n_cams,world,gy,seed", [(27, 8, 50, 0), (27, 8, 50, 1), (19, 4, 30, 2), (5, 8, 12, 3)])
def test_shard_camera_windows_balances_row_costs(n_cams, world, gy, seed):
    """With per-row work (row_cost) the left-over cameras' rows are cut so
    every rank's total work is the mean to within one row's cost -- except
    ranks whose whole cameras alone exceed the mean, which get no rows --
    and every camera is still covered exactly once."""
    from dynamic3dgaussians_amd.distributed import shard_camera_windows
    rng = np.random.default_rng(seed)
    gx = 7
    cost = rng.gamma(2.0, 1.0, (n_cams, gy)) * rng.uniform(0.5, 1.5, (n_cams, 1))
    cover = np.zeros((n_cams, gy), int)
    tot = []
    for r in range(world):
        t = 0.0
        for c, w in shard_camera_windows(n_cams, r, world, gx, gy, row_cost=cost):
            y0, y1 = (0, gy) if w is None else (w[1], w[3])
            if w is not None:
                assert (w[0], w[2]) == (0, gx)
            cover[c, y0:y1] += 1
            t += cost[c, y0:y1].sum()
        tot.append(t)
    assert (cover == 1).all()
    q = n_cams // world
    whole = np.array([cost[[c for c in range(q * world) if c % world == k]].sum() for k in range(world)])
    left = cost[q * world:].sum()
    lo, hi = whole.min(), whole.max() + left  # the balanced level: sum max(0, T - whole) = left
    for _ in range(200):
        T = 0.5 * (lo + hi)
        lo, hi = (T, hi) if np.maximum(0.0, T - whole).sum() < left else (lo, T)
    for k in range(world):
        if whole[k] < T - cost.max():
            assert abs(tot[k] - T) <= cost.max() * 1.0001 + 1e-6, (k, tot[k], T)
        else:
            assert tot[k] <= max(whole[k], T) + cost.max() * 1.0001 + 1e-6, (k, tot[k], T)
    assert max(tot) <= max(whole.max(), T) + cost.max() * 1.0001 + 1e-6
    # a fixed per-piece cost (ranks whose run spans two cameras get fewer
    # rows) keeps the partition
    cover[:] = 0
    for r in range(world):
        sh = shard_camera_windows(n_cams, r, world, gx, gy, row_cost=cost, piece_cost=cost.sum(1).mean() * 0.2)
        for c, w in sh:
            cover[c, (0 if w is None else w[1]):(gy if w is None else w[3])] += 1
    assert (cover == 1).all()
    # measured-feedback balance (bench.py --balance measured): a rank whose
    # measured step per modelled unit is 20 % above the mean gets less of the
    # left-over rows; the windows still partition every camera
    from dynamic3dgaussians_amd.distributed import rank_load_scale
    base = [sum(cost[c, (0 if w is None else w[1]):(gy if w is None else w[3])].sum() for c, w in
                shard_camera_windows(n_cams, r, world, gx, gy, row_cost=cost)) for r in range(world)]
    ms = [b * (1.2 if r == 1 else 1.0) for r, b in enumerate(base)]
    scale = rank_load_scale(ms, base)
    assert scale[1] > scale[0] and abs(np.mean(scale) - 1.0) < 1e-9
    cover[:] = 0
    got = []
    for r in range(world):
        sh = shard_camera_windows(n_cams, r, world, gx, gy, row_cost=cost, whole_scale=scale)
        got.append(sum(cost[c, (0 if w is None else w[1]):(gy if w is None else w[3])].sum() for c, w in sh))
        for c, w in sh:
            cover[c, (0 if w is None else w[1]):(gy if w is None else w[3])] += 1
    assert (cover == 1).all()
    if n_cams // world > 0:  # a rank with whole cameras to rescale
        assert got[1] <= base[1] + 1e-9


def _async_worker(rank, world, port, q):
    """bench.py's overlapped exchange on two alternating feature buckets."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = torch.nn.Parameter(torch.zeros(7, 3))
        buckets = [GradBucket({"f": f}, bind_grads=True) for _ in range(2)]
        works, out = [None, None], []
        for step in range(4):
            b = buckets[step % 2]
            if works[step % 2] is not None:  # the exchange of step - 2 read this buffer
                works[step % 2].wait()
            b.bind()
            b.zero_grad()
            (f * (rank + 1 + step)).sum().backward()
            works[step % 2] = b.all_reduce_async()
            prev = works[(step - 1) % 2]
            if prev is not None and step > 0:  # step - 1's exchange, consumed behind this step
                prev.wait()
                out.append(buckets[(step - 1) % 2].flat[:21].clone().numpy())
        works[3 % 2].wait()
        out.append(buckets[3 % 2].flat[:21].clone().numpy())
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_bucket_async_all_reduce_on_alternating_buffers():
    """GradBucket.all_reduce_async + bind(): each step's gradients land in
    the other buffer while the previous step's exchange may still run; every
    step's summed gradient comes out of its own buffer (ranks 1 + s and
    2 + s -> 3 + 2 s at step s)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_async_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert len(res[r]) == 4
        for s_, g in enumerate(res[r]):
            np.testing.assert_array_equal(g, np.full(21, 3.0 + 2 * s_, np.float32))


def test_replaced_bucket_releases_surviving_parameters_hooks():
    """with track_reached, each parameter carries a post-accumulate
    hook.  A parameter that survives a densification (the reference keeps
    cam_m / cam_c, external.py:185,253,263) must not keep the replaced bucket
    and its flat buffer alive, nor run its stale hook in later backwards:
    TimestepDriver closes the old bucket, and the hooks hold it weakly."""
    import gc
    import weakref

    from dynamic3dgaussians_amd.timesteps import TimestepDriver

    P = 64
    params = {"means3D": torch.nn.Parameter(torch.randn(P, 3)), "cam_m": torch.nn.Parameter(torch.zeros(1, 3))}
    opt = torch.optim.Adam([{"params": [v], "name": k, "lr": 1e-3} for k, v in params.items()])
    drv = TimestepDriver(params, {}, opt, 1, render=lambda rv, cams: (None, None), world=2)
    old = weakref.ref(drv._live_bucket())  # the plain path's bucket (built at its first step)
    # densification: means3D replaced, cam_m survives
    params["means3D"] = torch.nn.Parameter(torch.randn(2 * P, 3))
    opt.param_groups[0]["params"][0] = params["means3D"]
    drv._live_bucket()  # stale -> a new bucket
    gc.collect()
    assert old() is None, "the replaced bucket is still referenced (a surviving parameter's hook?)"
    # exactly one live hook on the surviving parameter: the new bucket's
    drv.bucket.zero_grad()
    (params["cam_m"].sum() * 2 + params["means3D"].sum()).backward()
    assert drv.bucket._reached == [True, True]
    n_hooks = len(params["cam_m"]._post_accumulate_grad_hooks or {})
    assert n_hooks == 1, n_hooks
    # a bucket closed by hand stops tracking; close() is idempotent
    b = GradBucket({"cam_m": params["cam_m"]}, bind_grads=True, track_reached=True)
    b.close()
    b.close()
    assert len(params["cam_m"]._post_accumulate_grad_hooks or {}) == 1
