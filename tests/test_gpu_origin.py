"""Shared origin step (camera mode, default; RM_MARCH_PER_RAY_ORIGIN / env RM_PER_RAY_ORIGIN=1
turns it off): every ray of a view starts its march at the eye (camera.rs:83-85), so the first
step's soft-min D(eye) is one value per view. The record kernel evaluates it once per view by
the march's own code path for that step and every ray starts from it. With it on and off the
images, march t, loss and every gradient are equal (==), and the work counters show the shared
steps as steps a wave did not run."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def mods():
    import torch
    from burn_raymarching_amd import model, native, render
    torch.cuda.init()
    return torch, model, native, render


def _both(monkeypatch, fn):
    # the general kernel's origin step (small camera calls of <= 32 spheres otherwise take the
    # small-scene kernel, which marches every step per ray)
    monkeypatch.setenv("RM_SMALL", "0")
    monkeypatch.setenv("RM_PER_RAY_ORIGIN", "1")
    per_ray = fn()
    monkeypatch.setenv("RM_PER_RAY_ORIGIN", "0")
    shared = fn()
    return per_ray, shared


# (views, W, H, M, k, steps): 16x16-tiled views; 40x24 in row order (ray blocks straddle two
# views); M = 600 (records built by several blocks + rm_prep_finish); k = 5; the reference's 40
@pytest.mark.parametrize("views,w,h,m,k,steps", [(2, 64, 64, 64, 32.0, 32), (3, 40, 24, 40, 5.0, 16),
                                                 (2, 48, 48, 600, 32.0, 12), (1, 64, 64, 256, 32.0, 40)])
def test_train_step_identical_with_shared_origin(mods, monkeypatch, views, w, h, m, k, steps):
    torch, model, native, render = mods
    sc = model.scene_tensors(model.synthetic_scene(m, 3), "cuda")
    cams = model.ring_cameras(10)[:views]
    tgt = render.render_diff_camera(cams, w, h, model.scene_tensors(model.synthetic_scene(m, 4), "cuda"), 32.0, steps)

    def run():
        out = torch.empty_like(tgt)
        march = native.march_params(steps, k)
        loss, g, _ = render.train_step_camera(cams, w, h, tgt, sc, k, 0.3, steps, out=out, march=march)
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    (l0, g0, o0), (l1, g1, o1) = _both(monkeypatch, run)
    assert torch.isfinite(o1).all()
    assert torch.equal(o0, o1)
    assert torch.equal(l0, l1)
    for key in g0:
        assert torch.equal(g0[key], g1[key]), key


def test_forward_t_and_backward_identical(mods, monkeypatch):
    torch, model, native, render = mods
    sc = model.scene_tensors(model.synthetic_scene(128, 7), "cuda")
    cams = model.ring_cameras(10)[3:6]
    (o0, t0), (o1, t1) = _both(monkeypatch, lambda: render.render_diff_camera(cams, 64, 64, sc, 32.0, 32,
                                                                              return_t=True))
    assert torch.equal(o0, o1) and torch.equal(t0, t1)
    g = torch.randn((3 * 4096, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(4))
    b0, b1 = _both(monkeypatch, lambda: render.render_diff_backward_camera(cams, 64, 64, sc, 32.0, g, 32))
    for key in b0:
        assert torch.equal(b0[key], b1[key]), key


def test_stats_count_shared_steps(mods, monkeypatch):
    torch, model, native, render = mods
    sc = model.scene_tensors(model.synthetic_scene(64, 2), "cuda")
    cams = model.ring_cameras(10)[:2]

    def saved():
        ctx = render.context()
        ctx.stats(True)
        ctx.collect_stats(reset=True)
        render.render_diff_camera(cams, 64, 64, sc, 32.0, 32)
        st = ctx.collect_stats(reset=True)
        ctx.stats(False)
        return st

    s0, s1 = _both(monkeypatch, saved)
    assert s0["waves"] == s1["waves"] == 2 * 4096 // 64
    assert s0["waves_exited"] == s1["waves_exited"]
    # every wave that did not leave at step 0 takes its first step from the shared value
    assert s0["steps_saved"] < s1["steps_saved"] <= s0["steps_saved"] + s1["waves"]


@pytest.mark.parametrize("views,m", [(16, 256), (5, 512), (1, 8), (40, 64), (128, 40)])
def test_origins_up_to_16_views(mods, monkeypatch, views, m):
    """Per-view origin steps for up to 128 views per call (one wave per view in rm_origin_kernel;
    beyond 16 views the camera bases come from the context's device table): images, loss and
    gradients equal (==) to the per-ray first step."""
    torch, model, native, render = mods
    sc = model.scene_tensors(model.synthetic_scene(m, 6), "cuda")
    cams = model.ring_cameras(max(16, views))[:views]
    tgt = render.render_diff_camera(cams, 32, 32, model.scene_tensors(model.synthetic_scene(m, 9), "cuda"), 32.0, 24)

    def run():
        out = torch.empty_like(tgt)
        loss, g, _ = render.train_step_camera(cams, 32, 32, tgt, sc, 32.0, 0.3, 24, out=out,
                                              march=native.march_params(24, 32.0))
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    per_ray, shared = _both(monkeypatch, run)
    assert torch.equal(shared[0], per_ray[0])
    assert torch.equal(shared[2], per_ray[2])
    for key in shared[1]:
        assert torch.equal(shared[1][key], per_ray[1][key]), key


@pytest.mark.parametrize("views,m", [(17, 48), (40, 48), (128, 48), (20, 300)])
def test_many_views_per_call(mods, monkeypatch, views, m):
    """A call of more than 16 views (device camera table, kInlineCams) renders what calls of at most
    16 views render, bit for bit (per-ray outputs), and its train step's gradient equals the sum of
    the smaller calls' to fp32 rounding (another block order in the reduction). 300 spheres at
    these sizes take the split march (its four-wave origin step included)."""
    import numpy as np
    torch, model, native, render = mods
    monkeypatch.setenv("RM_SMALL", "0")
    sc = model.scene_tensors(model.synthetic_scene(m, 3), "cuda")
    cams = model.ring_cameras(views)
    one = render.render_diff_camera(cams, 32, 32, sc, 32.0, 24)
    parts = torch.cat([render.render_diff_camera(cams[i:i + 16], 32, 32, sc, 32.0, 24) for i in range(0, views, 16)])
    assert torch.equal(one, parts)
    tgt = render.render_diff_camera(cams, 32, 32, model.scene_tensors(model.synthetic_scene(m, 4), "cuda"), 32.0, 24)
    n = views * 32 * 32
    _, g1, _ = render.train_step_camera(cams, 32, 32, tgt, sc, 32.0, 0.3, 24, inv_count=1.0 / (3 * n))
    acc = None
    for i in range(0, views, 16):
        _, g, _ = render.train_step_camera(cams[i:i + 16], 32, 32, tgt[i * 1024:(i + 16) * 1024], sc, 32.0, 0.3, 24,
                                           inv_count=1.0 / (3 * n))
        acc = {k: v.clone() for k, v in g.items()} if acc is None else {k: acc[k] + g[k] for k in g}
    for k in g1:
        a, b = g1[k].cpu().numpy(), acc[k].cpu().numpy()
        assert np.abs(a - b).max() <= 1e-5 * max(np.abs(b).max(), 1e-12), k
