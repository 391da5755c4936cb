"""GPU parity at the configurations the benchmark numbers are quoted on, through the C ABI,
against the fp64 oracle (oracle/rm_oracle_impl.h restating renderer_diff.rs:20-90,
scene.rs:60-128, sdf.rs:30-44 and training.rs:17-34).

  * the bench workload itself: camera-mode fused train step at 512x512, 256 spheres, 32 march
    steps, k = 32, with the early exit and the cost-ordered dispatch on (bench.py's defaults),
    every output and all five gradients against the oracle's train_step on the same rays;
  * BASELINE configs[2] (256 spheres, 64 steps) at a reduced ray count: forward, backward,
    train step;
  * the two march paths the default scene never takes: the vector-only march
    (RM_MARCH_VALU_ONLY) and the running-max log-sum-exp shift (RM_MARCH_FORCE_MAX_SHIFT);
  * the fp16 colour / fp32 SDF path of BASELINE configs[4] (RM_MARCH_COLOR_F16) at 4096
    spheres and 128 steps;
  * recovery of the cost-ordered dispatch from list counts a failed launch left uncleared.

Tolerances are the ones of tests/test_gpu_parity.py (forward max 1e-3 / mean 1e-5 linear RGB;
gradients by conftest.check_grads: 3e-3 of the largest fp64 component per group, relative L2 and
per-element relative bounds for the per-sphere groups), except where stated.
"""
import numpy as np
import pytest

from conftest import check_grads, gpu_available, record_margin

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

FWD_MAX, FWD_MEAN = 1e-3, 1e-5
KEYS = ("centers", "colors", "radius", "light_dir", "ambient")


@pytest.fixture(scope="module")
def rm():
    import torch
    from burn_raymarching_amd import _build
    _build.build_lib()
    from burn_raymarching_amd import model, native, render
    torch.cuda.init()
    return render, model, native


def dev(x, dtype=None):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()
    return t if dtype is None else t.to(dtype)


def host(t):
    return t.detach().float().cpu().numpy()


def scene_dev(render, sc, color_f16=False):
    import torch
    return render.Scene(dev(sc["centers"]), dev(sc["colors"], torch.float16 if color_f16 else None),
                        dev(sc["radius"]), dev(sc["light_dir"]), dev(sc["ambient"]))


def check_fwd(got, ref, fmax=FWD_MAX, fmean=FWD_MEAN):
    e = np.abs(got.astype(np.float64) - ref)
    assert np.isfinite(got).all()
    record_margin("fwd_max", e.max(), fmax)
    record_margin("fwd_mean", e.mean(), fmean)
    assert e.max() <= fmax and e.mean() <= fmean, (e.max(), e.mean())


def cam_rays(oracle, cams, width, height):
    rays = [oracle.camera_rays(width, height, *c, precision="f32") for c in cams]
    return np.concatenate([r[0] for r in rays]), np.concatenate([r[1] for r in rays])


def test_bench_workload_train_step_full_views(rm, oracle):
    """bench.py's step on two full 512x512 views of its camera ring (scene seed 0, radii
    U[0.03, 0.12], 256 spheres, 32 steps, k = 32, progress 0.5): three consecutive calls -- the
    2nd and 3rd dispatch their blocks in the cost order of the call before -- are bitwise equal,
    and the 3rd matches the fp64 oracle's train_step: image, loss and all five gradients."""
    import torch
    render, model, _ = rm
    W = H = 512
    M, S, K, prog = 256, 32, 32.0, 0.5
    sc = model.synthetic_scene(M, 0, radius_range=(0.03, 0.12))
    tsc = model.synthetic_scene(M, 1, radius_range=(0.03, 0.12))
    cams = model.ring_cameras(10)[:2]
    o, d = cam_rays(oracle, cams, W, H)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    targets = oracle.render_diff(o64, d64, tsc, S, K, precision="f64").astype(np.float32)
    s = scene_dev(render, sc)
    tg = dev(targets)
    runs = []
    ctx = render.context()
    for _ in range(3):
        out = torch.empty((2 * W * H, 3), device="cuda")
        loss, g, _ = render.train_step_camera(cams, W, H, tg, s, K, prog, S, out=out)
        runs.append((host(loss), {k: host(v) for k, v in g.items()}, host(out)))
    counts, nxt = ctx.order_counts()
    assert sum(counts[(nxt + 2) % 3]) == 2 * (W // 16) * (H // 16)  # the cost order is in use
    for r in runs[1:]:
        assert np.array_equal(r[0], runs[0][0]) and np.array_equal(r[2], runs[0][2])
        for k in KEYS:
            assert np.array_equal(r[1][k], runs[0][1][k]), k
    out_ref, loss_ref, g_ref = oracle.train_step(o64, d64, targets.astype(np.float64), sc, S, K, prog)
    loss, g, out = runs[2]
    check_fwd(out, out_ref)
    assert abs(loss[0] - loss_ref) <= 1e-4 * abs(loss_ref), (loss[0], loss_ref)
    check_grads(g, g_ref, mode="train")


@pytest.mark.parametrize("mode", ["forward", "backward", "train"])
def test_config2_s64(rm, oracle, mode):
    """BASELINE configs[2]: 256 spheres, 64 march steps, k = 32, on one 256x256 view of the ring
    (a quarter of the 512x512 rays of one view; camera mode, early exit, cost order)."""
    render, model, _ = rm
    W = H = 256
    M, S, K = 256, 64, 32.0
    sc = model.synthetic_scene(M, 2)
    cams = model.ring_cameras(10, offset=3)[:1]
    o, d = cam_rays(oracle, cams, W, H)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = scene_dev(render, sc)
    if mode == "forward":
        check_fwd(host(render.render_diff_camera(cams, W, H, s, K, S)), oracle.render_diff(o64, d64, sc, S, K))
    elif mode == "backward":
        g = np.random.default_rng(7).normal(size=o.shape).astype(np.float32)
        got = render.render_diff_backward_camera(cams, W, H, s, K, dev(g), S)
        check_grads(got, oracle.render_diff_backward(o64, d64, sc, S, K, g.astype(np.float64)))
    else:
        targets = oracle.render_diff(o64, d64, model.synthetic_scene(M, 3), S, K).astype(np.float32)
        for _ in range(2):  # the 2nd call runs in the cost order of the 1st
            loss, g, _ = render.train_step_camera(cams, W, H, dev(targets), s, K, 0.25, S)
        out_ref, loss_ref, g_ref = oracle.train_step(o64, d64, targets.astype(np.float64), sc, S, K, 0.25)
        assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref)
        check_grads(g, g_ref, mode="train")


@pytest.mark.parametrize("flag", ["RM_VALU_ONLY", "RM_FORCE_MAX_SHIFT"])
@pytest.mark.parametrize("steps", [32, 64])
def test_forced_march_paths(rm, oracle, monkeypatch, flag, steps):
    """The vector-only march and the running-max shift, forced, at 256 spheres (the metric's and
    configs[2]'s step counts): forward, backward and train step against the oracle, and the
    forced path really differs from the default one in the last bits."""
    import torch
    render, model, _ = rm
    W = H = 64
    M, K = 256, 32.0
    sc = model.synthetic_scene(M, 4)
    cams = model.ring_cameras(10, offset=1)[:2]
    o, d = cam_rays(oracle, cams, W, H)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = scene_dev(render, sc)
    default_out = render.render_diff_camera(cams, W, H, s, K, steps)
    monkeypatch.setenv(flag, "1")
    out = render.render_diff_camera(cams, W, H, s, K, steps)
    assert not torch.equal(out, default_out)
    check_fwd(host(out), oracle.render_diff(o64, d64, sc, steps, K))
    g = np.random.default_rng(8).normal(size=o.shape).astype(np.float32)
    check_grads(render.render_diff_backward_camera(cams, W, H, s, K, dev(g), steps),
                oracle.render_diff_backward(o64, d64, sc, steps, K, g.astype(np.float64)))
    targets = oracle.render_diff(o64, d64, model.synthetic_scene(M, 5), steps, K).astype(np.float32)
    loss, gt, _ = render.train_step(dev(o), dev(d), dev(targets), s, K, 0.75, steps)
    _, loss_ref, g_ref = oracle.train_step(o64, d64, targets.astype(np.float64), sc, steps, K, 0.75)
    assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref)
    check_grads(gt, g_ref, mode="train")


def _round_f16(sc):
    r = dict(sc)
    r["colors"] = sc["colors"].astype(np.float16).astype(np.float32)
    return r


@pytest.mark.parametrize("mode", ["forward", "backward", "train"])
def test_color_f16_config4(rm, oracle, mode):
    """fp16 colour / fp32 SDF (configs[4]: 4096 spheres, radii U[0.01, 0.04], 128 steps) on a
    32x32 view. Against the fp64 oracle on the fp16-rounded colours: the fp32 tolerances (the
    path computes in fp32 on exactly those colours). Against the unrounded colours: forward max
    1e-3 / mean 1e-4 (colour rounding is 2^-11 relative), gradients 4e-3."""
    render, model, _ = rm
    W = H = 32
    M, S, K = 4096, 128, 32.0
    sc = model.synthetic_scene(M, 6, radius_range=(0.01, 0.04))
    sc16 = _round_f16(sc)
    cams = model.ring_cameras(10, offset=2)[:1]
    o, d = cam_rays(oracle, cams, W, H)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = scene_dev(render, sc, color_f16=True)
    assert s.color_f16
    if mode == "forward":
        out = host(render.render_diff_camera(cams, W, H, s, K, S))
        check_fwd(out, oracle.render_diff(o64, d64, sc16, S, K))
        check_fwd(out, oracle.render_diff(o64, d64, sc, S, K), fmean=1e-4)
        ref32 = host(render.render_diff_camera(cams, W, H, scene_dev(render, sc16), K, S))
        assert np.array_equal(out, ref32)  # == the fp32 path fed the rounded colours
    elif mode == "backward":
        g = np.random.default_rng(9).normal(size=o.shape).astype(np.float32)
        got = render.render_diff_backward_camera(cams, W, H, s, K, dev(g), S)
        check_grads(got, oracle.render_diff_backward(o64, d64, sc16, S, K, g.astype(np.float64)))
        check_grads(got, oracle.render_diff_backward(o64, d64, sc, S, K, g.astype(np.float64)), scale=4.0 / 3.0)
    else:
        targets = oracle.render_diff(o64, d64, model.synthetic_scene(M, 7, radius_range=(0.01, 0.04)), S,
                                     K).astype(np.float32)
        loss, g, _ = render.train_step_camera(cams, W, H, dev(targets), s, K, 0.5, S)
        _, loss_ref, g_ref = oracle.train_step(o64, d64, targets.astype(np.float64), sc16, S, K, 0.5)
        assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref)
        check_grads(g, g_ref, mode="train")


def test_color_f16_full_size_properties(rm):
    """configs[4] at its full 512x512 / 4096 spheres / 128 steps: the fp16-colour render equals
    the fp32 render of the rounded colours bit for bit, stays within the colour rounding of the
    unrounded fp32 render, and its train step is finite and exactly linear in inv_count."""
    import torch
    render, model, _ = rm
    W = H = 512
    M, S, K = 4096, 128, 32.0
    sc = model.synthetic_scene(M, 0, radius_range=(0.01, 0.04))
    cams = model.ring_cameras(10)[:1]
    s16 = scene_dev(render, sc, color_f16=True)
    out16 = render.render_diff_camera(cams, W, H, s16, K, S)
    assert torch.equal(out16, render.render_diff_camera(cams, W, H, scene_dev(render, _round_f16(sc)), K, S))
    out32 = render.render_diff_camera(cams, W, H, scene_dev(render, sc), K, S)
    assert (out16 - out32).abs().max().item() <= 2.0 ** -11 * max(out32.abs().max().item(), 1e-6)
    tg = torch.zeros((W * H, 3), device="cuda")
    la, ga, _ = render.train_step_camera(cams, W, H, tg, s16, K, 0.5, S, inv_count=1.0 / (3 * W * H))
    lb, gb, _ = render.train_step_camera(cams, W, H, tg, s16, K, 0.5, S, inv_count=2.0 / (3 * W * H))
    assert torch.equal(la, lb)
    for k in KEYS:
        assert torch.isfinite(ga[k]).all(), k
        assert torch.equal(2.0 * ga[k], gb[k]), k


def test_optimizer_f16_colours(rm):
    """rm_optimizer_step_f16 == rm_optimizer_step, plus the updated activated colours rounded to
    fp16 (the next render's colour tensor)."""
    import torch
    render, model, _ = rm
    sc = model.synthetic_scene(37, 3)
    ma = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
    mb = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"],
                                         color_dtype="f16")
    assert mb.scene().color_f16 and not ma.scene().color_f16
    oa, ob = model.Adam(ma), model.Adam(mb)
    g = torch.randn(model.packed_size(37), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    for _ in range(3):
        oa.step(g, 0.05)
        ob.step(g, 0.05)
    assert torch.equal(ma.raw, mb.raw)
    col = ma.activated_packed()[3 * 37:6 * 37].view(37, 3)
    assert torch.equal(mb.scene().colors, col.half())


def test_stale_order_counts_recover(rm, oracle, monkeypatch):
    """A launch that leaves the next list set's counts uncleared (what a failed launch in the
    rotation leaves; RM_DEBUG_SKIP_ORDER_CLEAR) makes the launch that reads that set fall back
    to the static centre-out order; results stay bit-identical to the static order throughout,
    and the cost order is back two launches later."""
    import torch
    render, model, native = rm
    W = H = 128
    M, S, K = 64, 24, 32.0
    sc = model.synthetic_scene(M, 8)
    cams = model.ring_cameras(10, offset=5)[:3]
    s = scene_dev(render, sc)
    nblk = 3 * (W // 16) * (H // 16)
    tg = torch.rand((3 * W * H, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(2))
    static = native.march_params(S, K, flags=native.RM_MARCH_STATIC_ORDER)
    ref = render.train_step_camera(cams, W, H, tg, s, K, 0.5, S, march=static)
    ctx = render.context()

    def step():
        loss, g, _ = render.train_step_camera(cams, W, H, tg, s, K, 0.5, S)
        assert torch.equal(loss, ref[0])
        for k in KEYS:
            assert torch.equal(g[k], ref[1][k]), k
        counts, nxt = ctx.order_counts()
        return sum(counts[(nxt + 2) % 3])  # what the next launch reads

    for _ in range(4):
        assert step() == nblk
    monkeypatch.setenv("RM_DEBUG_SKIP_ORDER_CLEAR", "1")
    step()
    monkeypatch.delenv("RM_DEBUG_SKIP_ORDER_CLEAR")
    assert step() > nblk  # appended on top of stale counts: the next launch takes the static order
    totals = [step() for _ in range(3)]
    assert totals[-1] == nblk and totals[-2] == nblk


def test_shared_march_struct_f16_then_f32(rm):
    """A march struct shared by an fp16-colour scene and an fp32 scene (bench.py reuses one): the
    caller's struct is never modified, so the fp32 call after the fp16 one reads fp32 colours."""
    import torch
    render, model, native = rm
    sc = model.synthetic_scene(64, 3)
    cams = model.ring_cameras(4)[:1]
    march = native.march_params(16, 32.0)
    s16, s32 = scene_dev(render, sc, color_f16=True), scene_dev(render, sc)
    tg = torch.zeros((64 * 64, 3), device="cuda")
    render.train_step_camera(cams, 64, 64, tg, s16, 32.0, 0.5, 16, march=march)
    assert march.flags & native.RM_MARCH_COLOR_F16 == 0
    out_a, out_b = torch.empty_like(tg), torch.empty_like(tg)
    render.train_step_camera(cams, 64, 64, tg, s32, 32.0, 0.5, 16, march=march, out=out_a)
    render.train_step_camera(cams, 64, 64, tg, s32, 32.0, 0.5, 16, out=out_b)
    assert torch.equal(out_a, out_b)
