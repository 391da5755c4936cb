"""GPU parity tests: the HIP kernels (through the C ABI of include/raymarch.h) against the
CPU oracle (fp64 restatement of the reference) and the reference's own fixtures.

Tolerances (stated against the fp64 oracle; the fp32 reference-order restatement itself
sits at forward max 1.3e-4 / mean 5e-7 and gradient max-rel 6e-4, light_dir 2.7e-3):
  forward  linear RGB: max |d| <= 1e-3, mean |d| <= 1e-5
  PNG fixtures:        +-1 LSB
  gradients:           conftest.check_grads -- max |d| <= GRAD_TOL * max |g64| per parameter
                       group, plus relative-L2 and per-element relative bounds for the
                       per-sphere groups (set from the fp32 reference-order oracle's own error)
"""
import json
import os

import numpy as np
import pytest

from conftest import DANGO, FINAL1_CAMERA, GOLDEN, check_grads, final1_scene, gpu_available, load_png, record_margin

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

FWD_MAX, FWD_MEAN = 1e-3, 1e-5


@pytest.fixture(scope="module")
def rm():
    import torch
    from burn_raymarching_amd import _build
    _build.build_lib()
    from burn_raymarching_amd import model, render
    torch.cuda.init()
    return render, model


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


def host(t):
    return t.detach().cpu().numpy()


def scene_dev(rm, sc):
    render, _ = rm
    return render.Scene(dev(sc["centers"]), dev(sc["colors"]), dev(sc["radius"]), dev(sc["light_dir"]),
                        dev(sc["ambient"]))


def check_fwd(got, ref):
    e = np.abs(got.astype(np.float64) - ref)
    assert np.isfinite(got).all()
    record_margin("fwd_max", e.max(), FWD_MAX)
    record_margin("fwd_mean", e.mean(), FWD_MEAN)
    assert e.max() <= FWD_MAX and e.mean() <= FWD_MEAN, (e.max(), e.mean())


CASES = [  # (width, spheres, steps, k, seed)
    (64, 8, 16, 32.0, 0),   # BASELINE configs[0] shape
    (64, 8, 40, 5.0, 1),    # reference step count, early-training k
    (48, 64, 32, 32.0, 2),
    (40, 300, 16, 32.0, 3),  # M not a multiple of 32 and > 256
    (24, 1024, 64, 32.0, 5),  # BASELINE configs[3] sphere and step counts
    (16, 4096, 128, 32.0, 6),  # configs[4]: 4096 spheres, 128 steps (multi-block record kernel)
]


def rays_for(oracle, width, seed, precision="f32"):
    from burn_raymarching_amd.model import ring_cameras
    eye, tgt, fov = ring_cameras(7)[seed % 7]
    return oracle.camera_rays(width, width, eye, tgt, fov, precision=precision)


@pytest.mark.parametrize("width,m,steps,k,seed", CASES)
def test_forward_matches_oracle(rm, oracle, width, m, steps, k, seed):
    render, model = rm
    sc = model.synthetic_scene(m, seed)
    o, d = rays_for(oracle, width, seed)
    ref = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), sc, steps, k, precision="f64")
    out = render.render_diff_forward(dev(o), dev(d), scene_dev(rm, sc), k, steps)
    check_fwd(host(out), ref)


@pytest.mark.parametrize("small", ["0", "1"])
def test_camera_mode_equals_array_mode(rm, oracle, monkeypatch, small):
    """In-kernel camera rays are bit-identical to camera.rs rays, in the general kernel and in the
    small-scene kernel (RM_SMALL; both modes of a call take the same kernel)."""
    monkeypatch.setenv("RM_SMALL", small)
    render, model = rm
    sc = model.synthetic_scene(32, 5)
    cams = model.ring_cameras(3)
    outs = render.render_diff_camera(cams, 40, 24, scene_dev(rm, sc), 32.0, 20)
    for v, (eye, tgt, fov) in enumerate(cams):
        o, d = oracle.camera_rays(40, 24, eye, tgt, fov, precision="f32")
        arr = render.render_diff_forward(dev(o), dev(d), scene_dev(rm, sc), 32.0, 20)
        a = host(outs[v * 960:(v + 1) * 960])
        b = host(arr)
        assert np.array_equal(a, b)  # in-kernel rays are bit-identical to camera.rs rays


def test_final1_png_fixture_gpu(rm, oracle):
    """steps/final_1.png through the HIP forward (camera mode), +-1 LSB."""
    render, _ = rm
    out = render.render_diff_camera([FINAL1_CAMERA], 256, 256, scene_dev(rm, final1_scene()), 32.0, 40)
    png = oracle.to_png_bytes(host(out)).reshape(256, 256, 3).astype(int)
    ref = load_png(os.path.join(GOLDEN, "final_1.png")).astype(int)
    diff = np.abs(png - ref)
    assert diff.max() <= 1, diff.max()
    assert (diff > 0).sum() <= 64


@pytest.mark.parametrize("width,m,steps,k,seed", CASES)
def test_backward_matches_oracle(rm, oracle, width, m, steps, k, seed):
    render, model = rm
    sc = model.synthetic_scene(m, seed)
    o, d = rays_for(oracle, width, seed)
    g = np.random.default_rng(seed + 10).normal(size=o.shape).astype(np.float32)
    ref = oracle.render_diff_backward(o.astype(np.float64), d.astype(np.float64), sc, steps, k,
                                      g.astype(np.float64), precision="f64")
    got = render.render_diff_backward(dev(o), dev(d), scene_dev(rm, sc), k, dev(g), steps)
    check_grads(got, ref)


def test_backward_reuses_saved_t_bitwise(rm, oracle):
    render, model = rm
    sc = model.synthetic_scene(24, 9)
    o, d = rays_for(oracle, 32, 9)
    s = scene_dev(rm, sc)
    out, t = render.render_diff_forward(dev(o), dev(d), s, 20.0, 24, return_t=True)
    g = dev(np.random.default_rng(2).normal(size=o.shape))
    a = render.render_diff_backward(dev(o), dev(d), s, 20.0, g, 24)
    b = render.render_diff_backward(dev(o), dev(d), s, 20.0, g, 24, t_march=t)
    for key in a:
        assert np.array_equal(host(a[key]), host(b[key])), key


def test_autograd_function(rm, oracle):
    import torch
    render, model = rm
    sc = model.synthetic_scene(16, 4)
    o, d = rays_for(oracle, 24, 4)
    params = [dev(sc[k]).requires_grad_(True) for k in ("centers", "colors", "radius", "light_dir", "ambient")]
    out = render.render_diff(dev(o), dev(d), *params, 32.0, 16)
    g = dev(np.random.default_rng(5).normal(size=o.shape))
    (out * g).sum().backward()
    ref = oracle.render_diff_backward(o.astype(np.float64), d.astype(np.float64), sc, 16, 32.0,
                                      host(g).astype(np.float64), precision="f64")
    got = dict(zip(("centers", "colors", "radius", "light_dir", "ambient"), [p.grad for p in params]))
    check_grads(got, ref)
    assert torch.equal(out.detach(), render.render_diff_forward(dev(o), dev(d), scene_dev(rm, sc), 32.0, 16))


@pytest.mark.parametrize("m,progress", [(8, 0.1), (64, 0.9)])
def test_train_step_matches_oracle(rm, oracle, m, progress):
    render, model = rm
    sc = model.synthetic_scene(m, 11)
    tgt_sc = model.synthetic_scene(m, 12)
    o, d = rays_for(oracle, 48, 3)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    targets = oracle.render_diff(o64, d64, tgt_sc, 16, 32.0, precision="f64")
    out_ref, loss_ref, g_ref = oracle.train_step(o64, d64, targets, sc, 16, 20.0, progress)
    loss, g, out = render.train_step(dev(o), dev(d), dev(targets), scene_dev(rm, sc), 20.0, progress, 16,
                                     with_out=True)
    check_fwd(host(out), out_ref)
    assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref) + 1e-3
    check_grads(g, g_ref, mode="train")


def test_train_step_camera_matches_array(rm, oracle):
    render, model = rm
    sc = model.synthetic_scene(40, 13)
    cams = model.ring_cameras(2, offset=1)
    rays = [oracle.camera_rays(32, 32, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    targets = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), model.synthetic_scene(40, 14), 16,
                                 32.0, precision="f64").astype(np.float32)
    s = scene_dev(rm, sc)
    la, ga, _ = render.train_step(dev(o), dev(d), dev(targets), s, 32.0, 0.5, 16)
    lb, gb, _ = render.train_step_camera(cams, 32, 32, dev(targets), s, 32.0, 0.5, 16)
    assert abs(host(la)[0] - host(lb)[0]) <= 1e-5 * abs(host(la)[0]) + 1e-6
    for key in ga:
        a, b = host(ga[key]), host(gb[key])
        assert np.abs(a - b).max() <= 1e-4 * max(np.abs(a).max(), 1e-12), key


def test_multi_tile_spheres(rm, oracle):
    """M = 1100 > one 1024-sphere LDS tile: the per-sweep restaging path."""
    render, model = rm
    sc = model.synthetic_scene(1100, 21, radius_range=(0.01, 0.04))
    o, d = rays_for(oracle, 16, 1)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    ref = oracle.render_diff(o64, d64, sc, 8, 32.0, precision="f64")
    s = scene_dev(rm, sc)
    check_fwd(host(render.render_diff_forward(dev(o), dev(d), s, 32.0, 8)), ref)
    g = np.random.default_rng(0).normal(size=o.shape)
    gref = oracle.render_diff_backward(o64, d64, sc, 8, 32.0, g, precision="f64")
    check_grads(render.render_diff_backward(dev(o), dev(d), s, 32.0, dev(g), 8), gref)


def test_ragged_sizes_and_single_sphere(rm, oracle):
    render, model = rm
    for n, m in ((1, 1), (257, 13), (1000, 33)):
        sc = model.synthetic_scene(m, n)
        o, d = rays_for(oracle, 32, 2)
        o, d = o[:n], d[:n]
        o64, d64 = o.astype(np.float64), d.astype(np.float64)
        s = scene_dev(rm, sc)
        check_fwd(host(render.render_diff_forward(dev(o), dev(d), s, 32.0, 12)),
                  oracle.render_diff(o64, d64, sc, 12, 32.0, precision="f64"))
        g = np.random.default_rng(n).normal(size=o.shape)
        check_grads(render.render_diff_backward(dev(o), dev(d), s, 32.0, dev(g), 12),
                    oracle.render_diff_backward(o64, d64, sc, 12, 32.0, g, precision="f64"))


def test_zero_rays(rm):
    import torch
    render, model = rm
    s = scene_dev(rm, model.synthetic_scene(4, 0))
    e = torch.zeros((0, 3), device="cuda")
    assert render.render_diff_forward(e, e, s, 32.0, 8).shape == (0, 3)
    g = render.render_diff_backward(e, e, s, 32.0, e, 8)
    for v in g.values():
        assert torch.count_nonzero(v) == 0


def test_deterministic_bitwise(rm, oracle):
    render, model = rm
    sc = model.synthetic_scene(64, 6)
    o, d = rays_for(oracle, 64, 6)
    s = scene_dev(rm, sc)
    g = dev(np.random.default_rng(3).normal(size=o.shape))
    a = render.render_diff_backward(dev(o), dev(d), s, 32.0, g, 16)
    b = render.render_diff_backward(dev(o), dev(d), s, 32.0, g, 16)
    for key in a:
        assert np.array_equal(host(a[key]), host(b[key])), key


def test_invalid_arguments_raise(rm):
    import torch
    render, model = rm
    from burn_raymarching_amd.native import RaymarchError
    s = scene_dev(rm, model.synthetic_scene(4, 0))
    r = torch.zeros((8, 3), device="cuda")
    with pytest.raises(RaymarchError, match="smooth_k"):
        render.render_diff_forward(r, r, s, 0.0, 8)
    with pytest.raises(RaymarchError, match="steps"):
        render.render_diff_forward(r, r, s, 32.0, -1)
    with pytest.raises(ValueError):
        render.render_diff_forward(torch.zeros((8, 2), device="cuda"), r, s, 32.0, 8)
    with pytest.raises(ValueError):
        render.render_diff_camera([], 4, 4, s, 32.0, 8)
    import ctypes
    from burn_raymarching_amd import native
    ctx = render.context()
    march = native.march_params(8, 32.0)
    rc = ctx._lib.rm_render_diff_camera(ctx.handle, native.cameras([([0, 0, -2], [0, 0, 0], 50.0)]), 0, 4, 4,
                                        ctypes.byref(s.c_struct()), ctypes.byref(march),
                                        ctypes.c_void_p(r.data_ptr()), None)
    assert rc == 1 and b"num_views" in ctx._lib.rm_last_error(ctx.handle)


def test_sublaunch_split_large_batch(rm, oracle, monkeypatch):
    """More ray blocks than one launch takes (here capped at 4096 blocks = 1,048,576 rays with
    RM_MAX_BLOCKS_PER_LAUNCH; 16384 by default): split into sub-launches, gradients accumulated."""
    monkeypatch.setenv("RM_MAX_BLOCKS_PER_LAUNCH", "4096")
    render, model = rm
    sc = model.synthetic_scene(8, 17)
    cams = model.ring_cameras(2)
    w = 740  # 2 * 740^2 = 1,095,200 rays
    s = scene_dev(rm, sc)
    rays = [oracle.camera_rays(w, w, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    g = np.random.default_rng(1).normal(size=o.shape).astype(np.float32)
    got = render.render_diff_backward(dev(o), dev(d), s, 32.0, dev(g), 4)
    ref = oracle.render_diff_backward(o.astype(np.float64), d.astype(np.float64), sc, 4, 32.0,
                                      g.astype(np.float64), precision="f64")
    check_grads(got, ref)


def test_activation_and_optimizer_match_torch(rm):
    """rm_scene_activate (scene.rs:41-45) and rm_optimizer_step (chain rule + training.rs:38-82
    penalties + Burn Adam with coupled weight decay) against torch autograd / formulas."""
    import torch
    from oracle import autodiff_ref as ad
    render, model = rm
    rng = np.random.default_rng(0)
    m = 9
    raw = {"centers": rng.normal(scale=0.7, size=(m, 3)), "colors": rng.normal(size=(m, 3)),
           "radius": rng.normal(size=(m,)) * 1.5, "light_dir": np.array([0.2, 1.0, -0.3]),
           "ambient": np.array([-1.4])}
    raw["radius"][0] = 2.0  # softplus > 1: large-radius penalty branch
    sm = model.SceneModel.from_raw(raw["centers"], raw["colors"], raw["radius"], raw["light_dir"], raw["ambient"])
    act = host(sm.activated_packed())
    tr = {k: torch.tensor(np.asarray(v, np.float64).reshape((m, 3) if k in ("centers", "colors") else (-1, 1)
                                                           if k == "radius" else (-1,)), requires_grad=True)
          for k, v in raw.items()}
    a = ad.activate(tr)
    exp_act = np.concatenate([a["centers"].detach().numpy().ravel(), a["colors"].detach().numpy().ravel(),
                              a["radius"].detach().numpy().ravel(), a["light_dir"].detach().numpy().ravel(),
                              a["ambient"].detach().numpy().ravel()])
    assert np.abs(act - exp_act).max() < 2e-6
    # gradient w.r.t. activated params -> chain + penalties -> Adam (2 steps)
    gact = rng.normal(size=7 * m + 4)
    opt = model.Adam(sm, weight_decay=1e-5, with_penalties=True)
    pen = torch.zeros(1, device="cuda")
    theta = np.concatenate([np.asarray(raw[k], np.float64).ravel() for k in
                            ("centers", "colors", "radius", "light_dir", "ambient")])
    mom1 = np.zeros_like(theta)
    mom2 = np.zeros_like(theta)
    for step in (1, 2):
        opt.step(dev(gact), lr=0.05, penalty_out=pen)
        tr = {k: torch.tensor(v, requires_grad=True) for k, v in model.unpack(theta.copy(), m).items()}
        tr["radius"] = tr["radius"]
        acts = ad.activate({**tr, "radius": tr["radius"]})
        flat = torch.cat([acts[k].reshape(-1) for k in ("centers", "colors", "radius", "light_dir", "ambient")])
        zero = torch.zeros((1, 3), dtype=torch.float64)
        pen_loss = ad.compute_loss({**tr, "radius": tr["radius"].reshape(-1, 1)}, zero, zero, 0.0)
        (flat * torch.tensor(gact)).sum().add(pen_loss).backward()
        grad = np.concatenate([tr[k].grad.numpy().ravel() for k in
                               ("centers", "colors", "radius", "light_dir", "ambient")])
        grad = grad + 1e-5 * theta
        mom1 = 0.9 * mom1 + 0.1 * grad
        mom2 = 0.999 * mom2 + 0.001 * grad * grad
        mh = mom1 / (1 - 0.9 ** step)
        vh = mom2 / (1 - 0.999 ** step)
        theta = theta - 0.05 * mh / (np.sqrt(vh) + 1e-5)
        assert abs(host(pen)[0] - pen_loss.item()) < 1e-5 * max(1.0, abs(pen_loss.item()))
        got = host(sm.raw).astype(np.float64)
        assert np.abs(got - theta).max() < 2e-4, np.abs(got - theta).max()
        # the optimizer's fused activation output == rm_scene_activate of the updated params
        fused = host(sm._act).copy()
        sm.invalidate()
        assert np.array_equal(fused, host(sm.activated_packed()))
        theta = got  # continue from the device state (fp32 rounding)


def test_metric_size_properties(rm, oracle):
    """512x512, 256 spheres, 32 steps (the metric workload): finiteness, exact linearity in g
    (power-of-two scaling commutes with the fixed-order reductions), and a strided sample of
    rays against the fp64 oracle."""
    import torch
    render, model = rm
    sc = model.synthetic_scene(256, 0)
    s = scene_dev(rm, sc)
    cam = model.ring_cameras(4)[0]
    out = render.render_diff_camera([cam], 512, 512, s, 32.0, 32)
    assert torch.isfinite(out).all()
    o, d = oracle.camera_rays(512, 512, *cam, precision="f32")
    idx = np.arange(0, 512 * 512, 61)
    ref = oracle.render_diff(o[idx].astype(np.float64), d[idx].astype(np.float64), sc, 32, 32.0, precision="f64")
    check_fwd(host(out)[idx], ref)
    g = torch.randn((512 * 512, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(0))
    a = render.render_diff_backward_camera([cam], 512, 512, s, 32.0, g, 32)
    b = render.render_diff_backward_camera([cam], 512, 512, s, 32.0, 2.0 * g, 32)
    for key in a:
        assert torch.isfinite(a[key]).all()
        assert torch.equal(2.0 * a[key], b[key]), key
