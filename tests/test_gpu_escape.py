"""RM_MARCH_SKIP_ESCAPED: skipping ray blocks that provably escape the scene changes nothing.

With the skip on and off (env RM_SKIP_ESCAPED read by native.march_params; both legs in the
default 16x16-tile pixel order) the forward image,
the train-step loss and every gradient are equal (==; only the sign of an exact zero may
differ), and the stats counter shows that blocks were actually skipped."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def mods():
    import torch
    from burn_raymarching_amd import model, native, render
    torch.cuda.init()
    return torch, model, native, render


def _scene(mods, m, seed, radius_range=(0.03, 0.12)):
    torch, model, _, render = mods
    return model.scene_tensors(model.synthetic_scene(m, seed, radius_range), "cuda")


def _both(monkeypatch, fn):
    # the escape pre-pass runs with 256-ray blocks only (the library never splits a launch that
    # uses it), so the reference leg is the unsplit march too
    monkeypatch.setenv("RM_SPLIT", "0")
    monkeypatch.setenv("RM_SKIP_ESCAPED", "0")
    full = fn()
    monkeypatch.setenv("RM_SKIP_ESCAPED", "1")
    skip = fn()
    return full, skip


def _skipped(render, fn):
    ctx = render.context()
    ctx.stats(True)
    ctx.collect_stats(reset=True)
    fn()
    st = ctx.collect_stats(reset=True)
    ctx.stats(False)
    return st["blocks"], st["blocks_skipped"]


@pytest.mark.parametrize("m,k,steps,size", [(64, 32.0, 32, 128), (256, 32.0, 32, 96), (40, 5.0, 16, 64),
                                            (300, 32.0, 40, 80)])
def test_train_step_identical_with_skip(mods, monkeypatch, m, k, steps, size):
    torch, model, native, render = mods
    sc = _scene(mods, m, 3)
    cams = model.ring_cameras(10)[:2]
    tgt = render.render_diff_camera(cams, size, size, _scene(mods, m, 4), 32.0, steps)

    def run():
        out = torch.empty_like(tgt)
        loss, g, _ = render.train_step_camera(cams, size, size, tgt, sc, k, 0.3, steps, out=out)
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    (l0, g0, o0), (l1, g1, o1) = _both(monkeypatch, run)
    assert torch.equal(o0, o1)
    assert torch.equal(l0, l1)
    for key in g0:
        assert torch.equal(g0[key], g1[key]), key
    blocks, skipped = _skipped(render, run)
    assert blocks == 2 * size * size // 256
    if k == 32.0:
        assert skipped > 0  # the ring views have escaping corners at k = 32


def test_forward_and_backward_identical_with_skip(mods, monkeypatch):
    torch, model, native, render = mods
    sc = _scene(mods, 128, 7)
    cams = model.ring_cameras(10)[3:6]
    out0, out1 = _both(monkeypatch, lambda: render.render_diff_camera(cams, 64, 64, sc, 32.0, 32))
    assert torch.equal(out0, out1)
    # with return_t the march t is needed for every ray, so nothing is skipped
    monkeypatch.setenv("RM_SKIP_ESCAPED", "1")
    blocks, skipped = _skipped(render, lambda: render.render_diff_camera(cams, 64, 64, sc, 32.0, 32, return_t=True))
    assert skipped == 0
    _, t = render.render_diff_camera(cams, 64, 64, sc, 32.0, 32, return_t=True)
    g = torch.randn((4096, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(0))
    for t_march in (None, t[:4096]):
        b0, b1 = _both(monkeypatch, lambda: render.render_diff_backward_camera(cams[:1], 64, 64, sc, 32.0, g, 32,
                                                                             t_march=t_march))
        for key in b0:
            assert torch.equal(b0[key], b1[key]), key


def test_camera_inside_scene_never_skips(mods, monkeypatch):
    torch, model, native, render = mods
    sc = _scene(mods, 64, 2)
    cams = [([0.05, 0.02, 0.0], [1.0, 0.0, 0.0], 60.0)]
    monkeypatch.setenv("RM_SKIP_ESCAPED", "1")
    blocks, skipped = _skipped(render, lambda: render.render_diff_camera(cams, 32, 32, sc, 32.0, 16))
    assert skipped == 0
    out0, out1 = _both(monkeypatch, lambda: render.render_diff_camera(cams, 32, 32, sc, 32.0, 16))
    assert torch.equal(out0, out1)


def test_escaped_rays_are_exactly_zero_in_the_oracle(mods, oracle):
    """The certificate's premise, checked independently: rays the GPU renders as exactly 0
    (every ray of a skipped block) are black in the f64 oracle too."""
    torch, model, native, render = mods
    sc_np = model.synthetic_scene(64, 3)
    sc = model.scene_tensors(sc_np, "cuda")
    eye, tgt, fov = model.ring_cameras(10)[0]
    out = render.render_diff_camera([(eye, tgt, fov)], 64, 64, sc, 32.0, 32).cpu().numpy()
    o, d = oracle.camera_rays(64, 64, eye, tgt, fov)
    ref = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), sc_np, 32, 32.0, precision="f64")
    zero = (out == 0).all(1)
    assert zero.sum() > 500
    assert np.abs(ref[zero]).max() < 1e-30
