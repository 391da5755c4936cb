"""world_size-2 gloo test of the view-sharded data-parallel step (burn_raymarching_amd.parallel)
on CPU. The per-rank compute is the fp64 oracle (test infrastructure standing in for the HIP
train kernel, which needs a GPU); what is under test is the product's sharding, global-N loss
normalisation and the single sum all-reduce: the reduced gradient must equal one process
training on all views."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

W = 12
M = 6
S = 8
K = 20.0
VPG = 2
RING = 6


def _setup():
    from burn_raymarching_amd.model import ring_cameras, synthetic_scene
    from oracle import oracle as orc
    sc = synthetic_scene(M, 2)
    tgt_sc = synthetic_scene(M, 3)
    cams = ring_cameras(RING)
    rays = [orc.camera_rays(W, W, *c, precision="f64") for c in cams]
    targets = [orc.render_diff(o, d, tgt_sc, S, K) for o, d in rays]
    return orc, sc, rays, targets


def _pack(g):
    """Packed layout [centers 3M | colors 3M | radius M | light 3 | ambient 1], in fp64."""
    return np.concatenate([np.asarray(g[k], np.float64).reshape(-1)
                           for k in ("centers", "colors", "radius", "light_dir", "ambient")])


def _worker(rank, world, port, out_dir, global_views=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    from burn_raymarching_amd.parallel import Shard, ViewShardedStep
    orc, sc, rays, targets = _setup()

    def step_fn(views, inv_count, grads_out, loss_out):
        o = np.concatenate([rays[v][0] for v in views])
        d = np.concatenate([rays[v][1] for v in views])
        tg = np.concatenate([targets[v] for v in views])
        _, loss_sum, g = orc.train_step(o, d, tg, sc, S, K, 0.25, inv_count=inv_count)
        grads_out.copy_(torch.from_numpy(_pack(g)).to(grads_out.dtype))
        loss_out.fill_(loss_sum)

    shard = Shard(rank, world, 0 if global_views else VPG, RING, global_views)
    dp = ViewShardedStep(shard, W * W, 7 * M + 4, "cpu", step_fn)
    dp.buf = dp.buf.double()
    dp.grads = dp.buf[:7 * M + 4]
    dp.loss = dp.buf[7 * M + 4:]
    for step in range(3):
        dp(step)
        np.save(os.path.join(out_dir, f"r{rank}_s{step}.npy"), dp.buf.numpy())
        np.save(os.path.join(out_dir, f"views_r{rank}_s{step}.npy"), np.array(dp.shard.views(step)))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_view_sharded_allreduce_equals_single_process():
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, _free_port(), tmp), nprocs=world, join=True)
        orc, sc, rays, targets = _setup()
        for step in range(3):
            a = np.load(os.path.join(tmp, f"r0_s{step}.npy"))
            b = np.load(os.path.join(tmp, f"r1_s{step}.npy"))
            assert np.array_equal(a, b)  # every rank holds the same reduced gradient
            v0 = list(np.load(os.path.join(tmp, f"views_r0_s{step}.npy")))
            v1 = list(np.load(os.path.join(tmp, f"views_r1_s{step}.npy")))
            assert not set(v0) & set(v1) and len(v0) == len(v1) == VPG
            views = v0 + v1
            o = np.concatenate([rays[v][0] for v in views])
            d = np.concatenate([rays[v][1] for v in views])
            tg = np.concatenate([targets[v] for v in views])
            _, loss_sum, g = orc.train_step(o, d, tg, sc, S, K, 0.25)
            ref = _pack(g)
            assert np.allclose(a[:-1], ref, rtol=1e-10, atol=1e-13)
            assert abs(a[-1] - loss_sum) <= 1e-10 * abs(loss_sum)


def test_shard_rotation_covers_ring():
    from burn_raymarching_amd.parallel import Shard
    seen = set()
    for step in range(3):
        for r in range(2):
            seen.update(Shard(r, 2, 1, 6).views(step))
    assert seen == set(range(6))


@pytest.mark.timeout(300)
def test_strong_scaling_uneven_split_equals_single_process():
    """Strong scaling (bench.py --global-views): 3 views per step over 2 ranks (2 + 1), the
    global-N normalisation and the one all-reduce give the single-process gradient of the step's
    3 views; the step's views are disjoint across ranks and rotate over the ring."""
    world, gv = 2, 3
    with tempfile.TemporaryDirectory() as tmp:
        mp.spawn(_worker, args=(world, _free_port(), tmp, gv), nprocs=world, join=True)
        orc, sc, rays, targets = _setup()
        for step in range(3):
            a = np.load(os.path.join(tmp, f"r0_s{step}.npy"))
            b = np.load(os.path.join(tmp, f"r1_s{step}.npy"))
            assert np.array_equal(a, b)
            v0 = list(np.load(os.path.join(tmp, f"views_r0_s{step}.npy")))
            v1 = list(np.load(os.path.join(tmp, f"views_r1_s{step}.npy")))
            assert len(v0) == 2 and len(v1) == 1 and not set(v0) & set(v1)
            views = v0 + v1
            assert views == [(step * gv + j) % RING for j in range(gv)]
            o = np.concatenate([rays[v][0] for v in views])
            d = np.concatenate([rays[v][1] for v in views])
            tg = np.concatenate([targets[v] for v in views])
            _, loss_sum, g = orc.train_step(o, d, tg, sc, S, K, 0.25)
            assert np.allclose(a[:-1], _pack(g), rtol=1e-10, atol=1e-13)
            assert abs(a[-1] - loss_sum) <= 1e-10 * abs(loss_sum)


def test_shard_counts_strong_and_weak():
    from burn_raymarching_amd.parallel import Shard
    for world, gv in ((2, 5), (3, 7), (8, 80), (8, 3)):
        counts = [Shard(r, world, 0, 100, gv).count() for r in range(world)]
        assert sum(counts) == gv and max(counts) - min(counts) <= 1
        seen = []
        for r in range(world):
            seen += Shard(r, world, 0, 100, gv).views(4)
        assert seen == [(4 * gv + j) % 100 for j in range(gv)]
    weak = Shard(1, 4, 10, 80)
    assert weak.count() == 10 and weak.views_total == 40


def test_rank_share_alone_has_fixed_views_and_global_count():
    """bench.py --as-rank R/N: one process runs rank R's share of an N-rank strong step -- the same
    views every step when the step covers the whole ring (what rank R renders at N ranks), the
    global ray count in the seed, and no collective (no process group exists here)."""
    import torch
    from burn_raymarching_amd.parallel import Shard, ViewShardedStep
    calls, opt = [], []
    shard = Shard(3, 8, 0, 80, 80)
    dp = ViewShardedStep(shard, 100, 5, "cpu", lambda v, ic, g, l: calls.append((list(v), ic)),
                         optim_fn=lambda g: opt.append(1), collective=False)
    for step in range(3):
        dp(step)
    assert [c[0] for c in calls] == [list(range(30, 40))] * 3
    assert all(c[1] == 1.0 / (3.0 * 100 * 80) for c in calls) and len(opt) == 3
