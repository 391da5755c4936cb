"""BASELINE configs[1] on its stated poses: "256x256, 64 spheres, 32 steps, 10 views
(data/cameras.json)" (BASELINE.md:24-25). The camera-mode kernels on the ten poses of the reference's
data/cameras.json (tests/golden/cameras.json: eight at y = 0.5 around the scene, one from the top,
one from below; train.rs:62-85 loads them) against the fp64 oracle on the same rays:

  * forward and backward (a seeded N(0,1) dL/dout) on all ten poses at 128x128;
  * the fused train step at the full 256x256 on two of the poses (a ring view and the top view)
    against the reference's own target images for them (data/target_0.png, target_8.png, linear
    RGB as util.rs:21-33 loads them), twice (the second call in the cost order of the first).

Tolerances: tests/conftest.py (forward max 1e-3 / mean 1e-5 linear RGB; check_grads)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, check_grads, gpu_available, record_margin

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

M, S, K = 64, 32, 32.0


def _poses():
    cams = json.load(open(os.path.join(GOLDEN, "cameras.json")))
    return [(c["origin"], c["target"], c["fov"]) for c in cams], cams


def _rays(oracle, cams, w):
    rays = [oracle.camera_rays(w, w, *c, precision="f32") for c in cams]
    return np.concatenate([r[0] for r in rays]), np.concatenate([r[1] for r in rays])


def _dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


def test_forward_backward_on_reference_poses(oracle):
    from burn_raymarching_amd import model, render
    cams, _ = _poses()
    assert len(cams) == 10
    W = 128
    sc = model.synthetic_scene(M, 0)
    o, d = _rays(oracle, cams, W)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = model.scene_tensors(sc)
    out = render.render_diff_camera(cams, W, W, s, K, S).cpu().numpy()
    e = np.abs(out.astype(np.float64) - oracle.render_diff(o64, d64, sc, S, K))
    record_margin("fwd_max", e.max(), 1e-3)
    record_margin("fwd_mean", e.mean(), 1e-5)
    assert e.max() <= 1e-3 and e.mean() <= 1e-5, (e.max(), e.mean())
    g = np.random.default_rng(21).normal(size=o.shape).astype(np.float32)
    got = render.render_diff_backward_camera(cams, W, W, s, K, _dev(g), S)
    check_grads(got, oracle.render_diff_backward(o64, d64, sc, S, K, g.astype(np.float64)))


def test_train_step_on_reference_targets(oracle):
    from burn_raymarching_amd import host, model, render
    cams, entries = _poses()
    W = 256
    pick = [0, 8]
    sub = [cams[i] for i in pick]
    targets = np.concatenate([host.image_load(os.path.join(GOLDEN, os.path.basename(entries[i]["file"])))
                              for i in pick])
    sc = model.synthetic_scene(M, 0)
    o, d = _rays(oracle, sub, W)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = model.scene_tensors(sc)
    for _ in range(2):
        loss, g, _ = render.train_step_camera(sub, W, W, _dev(targets), s, K, 0.5, S)
    _, loss_ref, g_ref = oracle.train_step(o64, d64, targets.astype(np.float64), sc, S, K, 0.5)
    got = loss.cpu().numpy()[0]
    assert abs(got - loss_ref) <= 1e-4 * abs(loss_ref), (got, loss_ref)
    check_grads(g, g_ref, mode="train")
