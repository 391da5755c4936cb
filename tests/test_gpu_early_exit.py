"""Escaped-ray early exit (default; RM_MARCH_NO_EARLY_EXIT / env RM_NO_EARLY_EXIT=1 turns it
off): a wave whose rays all recede from the scene at a distance where the mask is exactly 0
stops marching and contributes out = 0 and zero gradient terms. With the exit on and off the
image, the train-step loss and every gradient are equal (==), and the counters show exits."""
import numpy as np
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
    monkeypatch.setenv("RM_NO_EARLY_EXIT", "1")
    full = fn()
    monkeypatch.setenv("RM_NO_EARLY_EXIT", "0")
    fast = fn()
    return full, fast


def _stats(render, fn):
    ctx = render.context()
    ctx.stats(True)
    ctx.collect_stats(reset=True)
    fn()
    st = ctx.collect_stats(reset=True)
    ctx.stats(False)
    return st


@pytest.mark.parametrize("m,k,steps,size,msharp", [(64, 32.0, 32, 128, 15.0), (256, 32.0, 32, 96, 15.0),
                                                   (40, 5.0, 40, 64, 15.0), (300, 32.0, 40, 80, 15.0),
                                                   (64, 32.0, 32, 64, 4.0), (1024, 32.0, 128, 48, 15.0)])
def test_train_step_identical_with_early_exit(mods, monkeypatch, m, k, steps, size, msharp):
    torch, model, render = mods
    sc = model.scene_tensors(model.synthetic_scene(m, 3), "cuda")
    cams = model.ring_cameras(10)[:2]
    tgt = render.render_diff_camera(cams, size, size, model.scene_tensors(model.synthetic_scene(m, 4), "cuda"),
                                    32.0, steps)
    from burn_raymarching_amd import native

    def run():
        out = torch.empty_like(tgt)
        march = native.march_params(steps, k, mask_sharpness=msharp)
        loss, g, _ = render.train_step_camera(cams, size, size, tgt, sc, k, 0.3, steps, out=out, march=march)
        torch.cuda.synchronize()
        return loss.clone(), {key: v.clone() for key, v in g.items()}, out

    (l0, g0, o0), (l1, g1, o1) = _both(monkeypatch, run)
    # finite at every step count: the march's t cap keeps rays that leave radially from
    # overflowing (configs[4] has 128 steps)
    assert torch.isfinite(o1).all() and torch.isfinite(l1).all()
    assert all(torch.isfinite(v).all() for v in g1.values())
    assert torch.equal(o0, o1)
    assert torch.equal(l0, l1)
    for key in g0:
        assert torch.equal(g0[key], g1[key]), key
    monkeypatch.setenv("RM_NO_EARLY_EXIT", "0")
    st = _stats(render, run)
    # one count per 64-ray wave, or per split ray group (split march: 32 rays, RM_SPLIT_RAYS)
    assert st["waves"] in (2 * size * size // 64, 2 * size * size // 32)
    if k == 32.0:
        assert st["waves_exited"] > 0 and st["steps_saved"] > 0
    # the backward sweeps' ray counts (rays with non-zero seeds): the same rays with the exit off,
    # the second sweep's a subset of the first's
    rays = 2 * size * size
    assert 0 < st["seeded_rays_a"] <= st["seeded_rays"] <= rays
    monkeypatch.setenv("RM_NO_EARLY_EXIT", "1")
    st_off = _stats(render, run)
    assert (st_off["seeded_rays"], st_off["seeded_rays_a"]) == (st["seeded_rays"], st["seeded_rays_a"])


def test_forward_backward_and_render_identical(mods, monkeypatch):
    torch, model, render = mods
    sc_np = model.synthetic_scene(128, 7)
    sc = model.scene_tensors(sc_np, "cuda")
    cams = model.ring_cameras(10)[3:6]
    out0, out1 = _both(monkeypatch, lambda: render.render_diff_camera(cams, 64, 64, sc, 32.0, 32))
    assert torch.equal(out0, out1)
    g = torch.randn((3 * 4096, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(0))
    b0, b1 = _both(monkeypatch, lambda: render.render_diff_backward_camera(cams, 64, 64, sc, 32.0, g, 32))
    for key in b0:
        assert torch.equal(b0[key], b1[key]), key
    c, col, r = (torch.tensor(sc_np[k2], device="cuda") for k2 in ("centers", "colors", "radius"))
    r0, r1 = _both(monkeypatch, lambda: render.render_camera(cams, 64, 64, c, col, r))
    assert torch.equal(r0, r1)
    # with return_t the full march is needed for every ray: no early exit
    monkeypatch.setenv("RM_NO_EARLY_EXIT", "0")
    st = _stats(render, lambda: render.render_diff_camera(cams, 64, 64, sc, 32.0, 32, return_t=True))
    assert st["waves_exited"] == 0


def test_t_march_contract_against_oracle(mods, oracle):
    """t_march (include/raymarch.h): the reference march t (renderer_diff.rs:20-26) to fp32
    rounding for every ray whose mask is not provably 0; a ray that provably escapes steps by the
    escape bound, so its t is at most the reference's and its out is exactly 0. Both t give the
    same image (the saved-t backward is bit-exact: test_gpu_parity.py)."""
    torch, model, render = mods
    sc_np = model.synthetic_scene(48, 8)
    cam = model.ring_cameras(10)[2]
    o, d = oracle.camera_rays(40, 40, *cam, precision="f32")
    s = model.scene_tensors(sc_np, "cuda")
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()  # noqa: E731
    out, t = render.render_diff_forward(dev(o), dev(d), s, 32.0, 40, return_t=True)
    ref, t_ref = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), sc_np, 40, 32.0, precision="f64",
                                    with_t=True)
    t_gpu = t.cpu().numpy().astype(np.float64)
    out_gpu = out.cpu().numpy()
    t_ref = np.asarray(t_ref, np.float64).reshape(-1)
    close = np.abs(t_gpu - t_ref) <= 1e-3 * np.maximum(1.0, np.abs(t_ref))
    bounded = (t_gpu <= t_ref * (1 + 1e-5) + 1e-4) & np.all(out_gpu == 0.0, axis=1)
    assert np.all(close | bounded), np.flatnonzero(~(close | bounded))[:8]
    assert close.sum() > 0 and np.isfinite(t_gpu).all()
    # where the ray still sees the scene (reference mask not negligible) t is the reference's
    seen = np.abs(ref).max(axis=1) > 1e-6
    assert np.all(close[seen])


@pytest.mark.parametrize("steps", [40, 128])
@pytest.mark.parametrize("small", ["0", "1"])
def test_receding_rays_stay_finite(mods, oracle, monkeypatch, steps, small):
    """A view that looks away from the scene: where the reference's fp32 march
    loses the rays at 128 steps (tests/test_oracle.py::test_reference_f32_march_breaks_for_receding_rays)
    the kernels -- general and small-scene -- return the fp64 restatement's exact 0 through the t
    cap: forward with t_march, and the train step's loss and sphere gradients, exit on and off."""
    torch, model, render = mods
    monkeypatch.setenv("RM_SMALL", small)
    sc = model.scene_tensors(model.synthetic_scene(16, seed=0), "cuda")
    eye = np.float32([0.0, 0.5, 2.5])
    o, d = oracle.camera_rays(8, 8, eye, eye * 2.0, 50.0, precision="f32")
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()  # noqa: E731
    out, t = render.render_diff_forward(dev(o), dev(d), sc, 32.0, steps, return_t=True)
    assert torch.isfinite(t).all() and float(t.max()) <= 1e15
    assert float(out.abs().max()) == 0.0
    tgt = torch.full_like(out, 0.25)
    for exit_off in ("1", "0"):
        monkeypatch.setenv("RM_NO_EARLY_EXIT", exit_off)
        loss, g, out2 = render.train_step(dev(o), dev(d), tgt, sc, 32.0, 0.5, steps, with_out=True)
        torch.cuda.synchronize()
        assert torch.isfinite(loss).all() and float(out2.abs().max()) == 0.0
        for key in ("centers", "colors", "radius"):
            assert float(g[key].abs().max()) == 0.0, key
        assert all(torch.isfinite(v).all() for v in g.values())
