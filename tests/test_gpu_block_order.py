"""Centre-out block dispatch (default in tiled camera mode; RM_MARCH_NATURAL_ORDER / env
RM_NATURAL_ORDER=1 turns it off) changes no result: gradient partials are indexed by the
tile, not by the dispatch position, so images, loss and gradients are equal (==) either way --
for square and non-square images, one or many views, and launches split into several chunks."""
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def mods():
    import torch
    from burn_raymarching_amd import model, render
    torch.cuda.init()
    return torch, model, render


def _both(monkeypatch, fn):
    monkeypatch.setenv("RM_NATURAL_ORDER", "1")
    natural = fn()
    monkeypatch.setenv("RM_NATURAL_ORDER", "0")
    ordered = fn()
    return natural, ordered


# (views, W, H): square, non-square (odd tile rows), and 5 x 512^2 = 5120 blocks, which the
# library splits into a 4-view and a 1-view launch (RM_MAX_BLOCKS_PER_LAUNCH = 4096)
@pytest.mark.parametrize("views,w,h", [(2, 128, 128), (3, 160, 96), (1, 48, 208), (5, 512, 512)])
def test_train_step_identical_in_any_dispatch_order(mods, monkeypatch, views, w, h):
    monkeypatch.setenv("RM_MAX_BLOCKS_PER_LAUNCH", "4096")
    torch, model, render = mods
    m, steps = 96, 32
    sc = model.scene_tensors(model.synthetic_scene(m, 5), "cuda")
    cams = model.ring_cameras(10)[:views]
    tgt = render.render_diff_camera(cams, w, h, model.scene_tensors(model.synthetic_scene(m, 6), "cuda"), 32.0, steps)

    def run():
        out = torch.empty_like(tgt)
        loss, g, _ = render.train_step_camera(cams, w, h, tgt, sc, 32.0, 0.5, steps, out=out)
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    (l0, g0, o0), (l1, g1, o1) = _both(monkeypatch, run)
    assert torch.equal(o0, o1)
    assert torch.equal(l0, l1)
    for key in g0:
        assert torch.equal(g0[key], g1[key]), key


def test_forward_and_backward_identical_in_any_dispatch_order(mods, monkeypatch):
    torch, model, render = mods
    sc = model.scene_tensors(model.synthetic_scene(128, 7), "cuda")
    cams = model.ring_cameras(10)[2:6]
    o0, o1 = _both(monkeypatch, lambda: render.render_diff_camera(cams, 96, 64, sc, 32.0, 32))
    assert torch.equal(o0, o1)
    g = torch.randn((4 * 96 * 64, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(2))
    b0, b1 = _both(monkeypatch, lambda: render.render_diff_backward_camera(cams, 96, 64, sc, 32.0, g, 32))
    for key in b0:
        assert torch.equal(b0[key], b1[key]), key


def test_cost_ordered_dispatch_identical(mods, monkeypatch):
    """Cost-ordered dispatch (default for repeated train/backward calls over the same views; the
    order comes from the block lists the previous call appended to by cost class, RM_MARCH_STATIC_ORDER / env
    RM_STATIC_ORDER=1 turns it off): the second call of a pair uses it, and its images, loss and
    gradients equal (==) the static centre-out order's."""
    torch, model, render = mods
    sc = model.scene_tensors(model.synthetic_scene(96, 8), "cuda")
    cams = model.ring_cameras(10)[1:5]
    tgt = render.render_diff_camera(cams, 128, 128, model.scene_tensors(model.synthetic_scene(96, 9), "cuda"), 32.0, 32)

    def run():
        out = torch.empty_like(tgt)
        loss, g, _ = render.train_step_camera(cams, 128, 128, tgt, sc, 32.0, 0.5, 32, out=out)
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    monkeypatch.setenv("RM_STATIC_ORDER", "1")
    l0, g0, o0 = run()
    monkeypatch.setenv("RM_STATIC_ORDER", "0")
    run()                  # establishes the cost history
    for i in range(4):     # dispatched by cost; the block lists rotate through three sets
        if i == 2:         # a call over other views in between: its lists must not be used here
            render.train_step_camera(cams[:2], 128, 128, tgt[:2 * 128 * 128], sc, 32.0, 0.5, 32)
            run()
        l1, g1, o1 = run()
        assert torch.equal(o0, o1)
        assert torch.equal(l0, l1)
        for key in g0:
            assert torch.equal(g0[key], g1[key]), key
    g = torch.randn((4 * 128 * 128, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(3))
    monkeypatch.setenv("RM_STATIC_ORDER", "1")
    b0 = render.render_diff_backward_camera(cams, 128, 128, sc, 32.0, g, 32)
    monkeypatch.setenv("RM_STATIC_ORDER", "0")
    render.render_diff_backward_camera(cams, 128, 128, sc, 32.0, g, 32)
    b1 = render.render_diff_backward_camera(cams, 128, 128, sc, 32.0, g, 32)
    for key in b0:
        assert torch.equal(b0[key], b1[key]), key


def test_cost_order_across_rotating_view_sets(mods, monkeypatch):
    """A caller rotating through view sets of the same shape (BASELINE configs[4]: one view per
    step over a ring) reads, on every call, the lists the previous call -- over other views --
    appended: a valid permutation of the same blocks, so the images, loss and gradients equal (==)
    the static order's on every call."""
    torch, model, render = mods
    sc = model.scene_tensors(model.synthetic_scene(96, 8), "cuda")
    ring = model.ring_cameras(8)
    sets = [ring[2 * i:2 * i + 2] for i in range(4)]
    tgt = render.render_diff_camera(ring[:2], 64, 64, model.scene_tensors(model.synthetic_scene(96, 9), "cuda"),
                                    32.0, 32)

    def run(cams):
        out = torch.empty_like(tgt)
        loss, g, _ = render.train_step_camera(cams, 64, 64, tgt, sc, 32.0, 0.5, 32, out=out)
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    monkeypatch.setenv("RM_STATIC_ORDER", "1")
    ref = [run(c) for c in sets]
    monkeypatch.setenv("RM_STATIC_ORDER", "0")
    for _ in range(3):
        for c, (l0, g0, o0) in zip(sets, ref):
            l1, g1, o1 = run(c)
            assert torch.equal(o0, o1) and torch.equal(l0, l1)
            for key in g0:
                assert torch.equal(g0[key], g1[key]), key
