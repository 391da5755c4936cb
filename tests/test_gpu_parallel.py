"""The view-sharded data-parallel step (burn_raymarching_amd.parallel.ViewShardedStep, SURVEY.md
§8(e)) with the REAL HIP train kernel: two rank processes share the one GPU of the test box and
all-reduce over gloo (RCCL refuses two ranks on one device; the collective's place in the step
is the same). Each rank runs rm_train_step_camera on its own views with the global-N loss
scaling, then the replicated optimizer. Checked: both ranks hold bit-identical reduced buffers
and parameters after every step, and the reduced gradient and loss equal one process training
on all the views (to fp32 summation order), step after step (reference step:
train.rs:169-199)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

W = 64
M = 32
S = 16
K = 24.0
VPG = 2
RING = 4
STEPS = 3
LR = 0.05


def _setup(torch, color_dtype="f32"):
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import render as rmr
    sc = rmm.synthetic_scene(M, 21)
    cams = rmm.ring_cameras(RING)
    targets = rmr.render_diff_camera(cams, W, W, rmm.scene_tensors(rmm.synthetic_scene(M, 22)), K, S)
    targets = targets.view(RING, W * W, 3)
    model = rmm.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"],
                                          color_dtype=color_dtype)
    opt = rmm.Adam(model)

    def step_fn(views, inv_count, grads_out, loss_out):
        tg = torch.cat([targets[v] for v in views])
        rmr.train_step_camera([cams[v] for v in views], W, W, tg, model.scene(), K, 0.5, S, inv_count=inv_count,
                              grads_packed=grads_out, loss=loss_out)

    return model, opt, step_fn


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from burn_raymarching_amd.parallel import Shard, ViewShardedStep
    model, opt, step_fn = _setup(torch)
    dp = ViewShardedStep(Shard(rank, world, VPG, RING), W * W, 7 * M + 4, "cuda", step_fn,
                         optim_fn=lambda g: opt.step(g, LR))
    for step in range(STEPS):
        dp(step)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f"buf_r{rank}_s{step}.npy"), dp.buf.cpu().numpy())
        np.save(os.path.join(out_dir, f"raw_r{rank}_s{step}.npy"), model.raw.cpu().numpy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_sharded_hip_step_equals_single_process():
    import torch
    from burn_raymarching_amd.parallel import Shard, ViewShardedStep
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, _free_port(), tmp), nprocs=world, join=True, start_method="spawn")
        # one process over all RING views per step (world 1, VPG * 2 views): the same views
        model, opt, step_fn = _setup(torch)
        dp = ViewShardedStep(Shard(0, 1, VPG * world, RING), W * W, 7 * M + 4, "cuda", step_fn,
                             optim_fn=lambda g: opt.step(g, LR))
        for step in range(STEPS):
            b0 = np.load(os.path.join(tmp, f"buf_r0_s{step}.npy"))
            b1 = np.load(os.path.join(tmp, f"buf_r1_s{step}.npy"))
            assert np.array_equal(b0, b1), step  # every rank holds the same reduced gradient
            r0 = np.load(os.path.join(tmp, f"raw_r0_s{step}.npy"))
            assert np.array_equal(r0, np.load(os.path.join(tmp, f"raw_r1_s{step}.npy"))), step
            if step > 0:  # continue the single process from the ranks' parameters (no drift)
                model.raw.copy_(torch.from_numpy(np.load(os.path.join(tmp, f"raw_r0_s{step - 1}.npy"))).cuda())
                model.invalidate()
            dp(step)
            torch.cuda.synchronize()
            ref = dp.buf.cpu().numpy()
            g_ref, g = ref[:-1], b0[:-1]
            assert np.abs(g - g_ref).max() <= 1e-5 * np.abs(g_ref).max(), (step, np.abs(g - g_ref).max())
            assert abs(b0[-1] - ref[-1]) <= 1e-5 * abs(ref[-1])
            # the single-process views of this step are the union of the two ranks' views
            assert sorted(Shard(0, 1, VPG * world, RING).views(step)) == sorted(
                Shard(0, world, VPG, RING).views(step) + Shard(1, world, VPG, RING).views(step))
