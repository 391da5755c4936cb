"""The small-scene kernel (rm_small_kernel, M <= 32; csrc/rm_small.h) through the C ABI against the
fp64 oracle, at the shape of the reference's own training loop: ray-array train steps of a random
16,384-ray batch drawn from the pixels of several views (dataset.rs:47-82), 7-20 spheres, 40 march
steps (renderer_diff.rs:20-26), k annealed 5 -> 32 (train.rs:174). Also: every sphere-count bucket
edge, ragged and multi-launch ray counts (the in-kernel last-block reduction and the partial-record
path), forward / backward / t_march, fp16 colours, accumulate, camera mode (RM_SMALL=1), bitwise
determinism, and agreement with the general kernel (RM_SMALL=0). Tolerances: tests/conftest.py."""
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


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


def host(t):
    return t.detach().float().cpu().numpy()


def check_fwd(got, ref):
    e = np.abs(got.astype(np.float64) - ref)
    assert np.isfinite(got).all()
    record_margin("fwd_max", e.max(), FWD_MAX)
    record_margin("fwd_mean", e.mean(), FWD_MEAN)
    assert e.max() <= FWD_MAX and e.mean() <= FWD_MEAN, (e.max(), e.mean())


def batch(oracle, model, n, seed, views=6, size=96):
    """n rays drawn uniformly (seeded) from the pixels of `views` ring views, as the dataset's
    uniform share draws them (dataset.rs:54-61)."""
    cams = model.ring_cameras(views, offset=seed % 3)
    rays = [oracle.camera_rays(size, size, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    idx = np.random.default_rng(seed).integers(0, o.shape[0], n)
    return o[idx], d[idx]


def train_scene(model, m, seed):
    # the reference's scenes after prune/split: a few larger spheres (train.rs:103-126, training.rs:185-222)
    return model.synthetic_scene(m, seed, radius_range=(0.08, 0.3))


@pytest.mark.parametrize("k", [5.0, 32.0])
@pytest.mark.parametrize("m", [7, 9, 20])
def test_reference_training_call(rm, oracle, monkeypatch, m, k):
    """The reference loop's call: rm_train_step on 16,384 random rays, S = 40 (default path)."""
    render, model, _ = rm
    monkeypatch.delenv("RM_SMALL", raising=False)
    n, steps = 16384, 40
    sc = train_scene(model, m, 30 + m)
    o, d = batch(oracle, model, n, m)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    targets = oracle.render_diff(o64, d64, train_scene(model, 5, 7), steps, 32.0)
    out_ref, loss_ref, g_ref = oracle.train_step(o64, d64, targets, sc, steps, k, 0.4)
    loss, g, out = render.train_step(dev(o), dev(d), dev(targets), model.scene_tensors(sc), k, 0.4, steps,
                                     with_out=True)
    check_fwd(host(out), out_ref)
    assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref) + 1e-3
    check_grads(g, g_ref, mode="train")


@pytest.mark.parametrize("lpr", ["1", "2"])
@pytest.mark.parametrize("m", [4, 9, 32])
def test_lanes_per_ray(rm, oracle, monkeypatch, m, lpr):
    """Train steps with one lane per ray and with the march split over two lanes (RM_SMALL_LPR,
    the default for <= 32,768 rays): both against the oracle, and within fp32 rounding of each other."""
    render, model, _ = rm
    monkeypatch.setenv("RM_SMALL_LPR", lpr)
    n, steps = 16384, 40
    sc = train_scene(model, m, 60 + m)
    o, d = batch(oracle, model, n, 100 + m)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    targets = oracle.render_diff(o64, d64, train_scene(model, 5, 8), steps, 32.0)
    out_ref, loss_ref, g_ref = oracle.train_step(o64, d64, targets, sc, steps, 24.0, 0.6)
    loss, g, out = render.train_step(dev(o), dev(d), dev(targets), model.scene_tensors(sc), 24.0, 0.6, steps,
                                     with_out=True)
    check_fwd(host(out), out_ref)
    assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref) + 1e-3
    check_grads(g, g_ref, mode="train")


@pytest.mark.parametrize("m", [1, 4, 8, 12, 16, 17, 24, 32])
@pytest.mark.parametrize("n", [1, 257, 4096])
def test_bucket_edges_forward_backward(rm, oracle, m, n):
    render, model, _ = rm
    sc = model.synthetic_scene(m, m + n)
    o, d = batch(oracle, model, n, m * 7 + n, views=3, size=48)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = model.scene_tensors(sc)
    out, t = render.render_diff_forward(dev(o), dev(d), s, 24.0, 20, return_t=True)
    check_fwd(host(out), oracle.render_diff(o64, d64, sc, 20, 24.0))
    g = np.random.default_rng(n).normal(size=o.shape)
    gref = oracle.render_diff_backward(o64, d64, sc, 20, 24.0, g)
    got = render.render_diff_backward(dev(o), dev(d), s, 24.0, dev(g), 20)
    if n >= 257:
        check_grads(got, gref)
    else:  # one ray: a handful of terms; normwise bound only (relative bounds need a population)
        for key in KEYS:
            a, b = host(got[key]).reshape(-1), gref[key].reshape(-1)
            assert np.abs(a - b).max() <= 3e-3 * max(np.abs(b).max(), 1e-12), key
    # the saved t gives the same gradients bit for bit
    got_t = render.render_diff_backward(dev(o), dev(d), s, 24.0, dev(g), 20, t_march=t)
    for key in KEYS:
        assert np.array_equal(host(got[key]), host(got_t[key])), key


@pytest.mark.parametrize("n", [65536, 70000, 300000])
def test_many_blocks_and_sublaunches(rm, oracle, monkeypatch, n):
    """> kSmallFinalMaxBlocks blocks: partial records + rm_reduce_partials / rm_finalize_grads;
    with RM_MAX_BLOCKS_PER_LAUNCH the call splits into launches that accumulate."""
    render, model, _ = rm
    if n == 300000:
        monkeypatch.setenv("RM_MAX_BLOCKS_PER_LAUNCH", "400")
    sc = train_scene(model, 11, 5)
    o, d = batch(oracle, model, n, 3, views=8, size=128)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    targets = oracle.render_diff(o64, d64, train_scene(model, 4, 9), 16, 32.0)
    out_ref, loss_ref, g_ref = oracle.train_step(o64, d64, targets, sc, 16, 20.0, 0.7)
    loss, g, out = render.train_step(dev(o), dev(d), dev(targets), model.scene_tensors(sc), 20.0, 0.7, 16,
                                     with_out=True)
    check_fwd(host(out), out_ref)
    assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref) + 1e-3
    check_grads(g, g_ref, mode="train")


def test_deterministic_and_accumulate(rm, oracle):
    """Repeated calls are bitwise equal (fixed-order lane / wave / block sums, the last block's
    reduction included); accumulate = 1 adds exactly the same gradient again (2x, exact)."""
    import ctypes
    import torch
    render, model, native = rm
    sc = train_scene(model, 13, 1)
    o, d = batch(oracle, model, 16384, 11)
    tg = dev(np.random.default_rng(2).uniform(size=o.shape))
    s = model.scene_tensors(sc)
    runs = [render.train_step(dev(o), dev(d), tg, s, 12.0, 0.2, 40) for _ in range(3)]
    for r in runs[1:]:
        assert torch.equal(r[0], runs[0][0])
        for key in KEYS:
            assert torch.equal(r[1][key], runs[0][1][key]), key
    loss, g, _ = runs[0]
    g2 = {k: v.clone() for k, v in g.items()}
    cg = native.RmGrads(*(g2[k].data_ptr() for k in KEYS))
    l2 = loss.clone()
    ctx = render.context()
    march = s.march_for(native.march_params(40, 12.0))
    od, dd = dev(o), dev(d)  # held: the call reads them asynchronously
    ctx.check(ctx._lib.rm_train_step(ctx.handle, ctypes.c_void_p(od.data_ptr()), ctypes.c_void_p(dd.data_ptr()),
                                     ctypes.c_void_p(tg.data_ptr()), 16384, 0.2, 1.0 / (3 * 16384),
                                     ctypes.byref(s.c_struct()), ctypes.byref(march), ctypes.byref(cg),
                                     ctypes.c_void_p(l2.data_ptr()), None, 1), "rm_train_step")
    torch.cuda.synchronize()
    assert torch.equal(l2, 2.0 * loss)
    for key in KEYS:
        assert torch.equal(g2[key], 2.0 * g[key]), key


def test_color_f16_small(rm, oracle):
    """fp16 colours through the small kernel: equal to the fp32 path on the rounded colours."""
    import torch
    render, model, _ = rm
    sc = train_scene(model, 10, 4)
    o, d = batch(oracle, model, 5000, 4)
    rounded = dict(sc, colors=sc["colors"].astype(np.float16).astype(np.float32))
    s16 = render.Scene(dev(sc["centers"]), dev(sc["colors"]).half(), dev(sc["radius"]), dev(sc["light_dir"]),
                       dev(sc["ambient"]))
    a = render.render_diff_forward(dev(o), dev(d), s16, 32.0, 40)
    b = render.render_diff_forward(dev(o), dev(d), model.scene_tensors(rounded), 32.0, 40)
    assert torch.equal(a, b)


@pytest.mark.parametrize("m", [6, 20])
def test_camera_mode_small(rm, oracle, monkeypatch, m):
    """Camera mode through the small kernel (RM_SMALL=1): bit-identical to array mode on the
    camera.rs rays, and against the oracle."""
    import torch
    render, model, _ = rm
    monkeypatch.setenv("RM_SMALL", "1")
    sc = train_scene(model, m, 2)
    cams = model.ring_cameras(3)
    out = render.render_diff_camera(cams, 48, 32, model.scene_tensors(sc), 32.0, 40)
    rays = [oracle.camera_rays(48, 32, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    arr = render.render_diff_forward(dev(o), dev(d), model.scene_tensors(sc), 32.0, 40)
    assert torch.equal(out, arr)
    check_fwd(host(out), oracle.render_diff(o.astype(np.float64), d.astype(np.float64), sc, 40, 32.0))
    tg = dev(np.random.default_rng(1).uniform(size=o.shape))
    _, ga, _ = render.train_step(dev(o), dev(d), tg, model.scene_tensors(sc), 32.0, 0.5, 40)
    _, gb, _ = render.train_step_camera(cams, 48, 32, tg, model.scene_tensors(sc), 32.0, 0.5, 40)
    for key in KEYS:
        a, b = host(ga[key]), host(gb[key])
        assert np.abs(a - b).max() <= 1e-5 * max(np.abs(a).max(), 1e-12), key


def test_small_and_general_kernel_agree(rm, oracle, monkeypatch):
    """The small kernel and the general kernel (RM_SMALL=0) on the same call: both within the
    oracle's bounds, and within fp32 rounding of each other."""
    render, model, _ = rm
    sc = train_scene(model, 9, 3)
    o, d = batch(oracle, model, 16384, 5)
    tg = dev(np.random.default_rng(3).uniform(size=o.shape))
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("RM_SMALL", flag)
        loss, g, out = render.train_step(dev(o), dev(d), tg, model.scene_tensors(sc), 24.0, 0.3, 40, with_out=True)
        res[flag] = (host(loss)[0], {k: host(v) for k, v in g.items()}, host(out))
    assert abs(res["1"][0] - res["0"][0]) <= 1e-4 * abs(res["0"][0])
    assert np.abs(res["1"][2] - res["0"][2]).max() <= 1e-3
    for key in KEYS:
        a, b = res["1"][1][key], res["0"][1][key]
        assert np.abs(a - b).max() <= 3e-3 * max(np.abs(b).max(), 1e-12), key


def _iteration(torch, native, render, model, src, fg, nu, nf, sc, steps, fused, monkeypatch):
    """`steps` training iterations (train.rs:169-198) through rm_train_iteration (fused: one launch
    when eligible), through rm_sample_batch + rm_train_step + rm_optimizer_step (fused False), or
    through rm_train_step_sampled + rm_optimizer_step (fused "sampled": a data-parallel rank's
    calls around its all-reduce)."""
    import ctypes
    monkeypatch.setenv("RM_FUSED_ITER", "0" if fused is False else "1")
    m = sc["centers"].shape[0]
    sm = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
    raw = sm.raw.clone()
    act = sm.activated_packed().clone()
    npk = model.packed_size(m)
    grad = torch.zeros(npk, device="cuda")
    mom = [torch.zeros(npk, device="cuda") for _ in range(2)]
    loss = torch.zeros(2, device="cuda")
    ctx = render.context()
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    o, d, t = src
    n = nu + nf
    out = []
    for it in range(1, steps + 1):
        k = 5.0 + 27.0 * it / steps
        march = native.march_params(40, k)
        args = (o.shape[0], p(fg), fg.numel(), nu, nf, 11, 1, it, it / steps, 1.0 / (3 * n))
        if fused in ("prepared", "prepared_other_step"):
            # the optimizer's gradient-independent part in the sampled launch; "prepared_other_step"
            # prepares for another step number, so the optimizer call must compute it itself
            s = native.RmScene()
            ctx._lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
            g = native.RmGrads()
            ctx._lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
            prep_step = it if fused == "prepared" else it + 1
            ctx.check(ctx._lib.rm_train_step_sampled_prepared(ctx.handle, p(o), p(d), p(t), *args, ctypes.byref(s),
                                                              ctypes.byref(march), ctypes.byref(g), p(loss), p(raw),
                                                              prep_step, 1, ctypes.c_void_p(loss.data_ptr() + 4)),
                      "rm_train_step_sampled_prepared")
            ctx.check(ctx._lib.rm_optimizer_step(ctx.handle, p(raw), p(grad), p(mom[0]), p(mom[1]), m, it, 0.01, 1e-5, 1,
                                                 ctypes.c_void_p(loss.data_ptr() + 4), p(act)), "rm_optimizer_step")
        elif fused == "sampled":
            s = native.RmScene()
            ctx._lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
            g = native.RmGrads()
            ctx._lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
            ctx.check(ctx._lib.rm_train_step_sampled(ctx.handle, p(o), p(d), p(t), *args, ctypes.byref(s),
                                                     ctypes.byref(march), ctypes.byref(g), p(loss)),
                      "rm_train_step_sampled")
            ctx.check(ctx._lib.rm_optimizer_step(ctx.handle, p(raw), p(grad), p(mom[0]), p(mom[1]), m, it, 0.01, 1e-5, 1,
                                                 ctypes.c_void_p(loss.data_ptr() + 4), p(act)), "rm_optimizer_step")
        elif fused:
            ctx.check(ctx._lib.rm_train_iteration(ctx.handle, p(o), p(d), p(t), *args, ctypes.byref(march), p(act),
                                                  p(grad), p(raw), p(mom[0]), p(mom[1]), m, it, 0.01, 1e-5, 1,
                                                  p(loss), ctypes.c_void_p(loss.data_ptr() + 4)), "rm_train_iteration")
        else:
            b = [torch.empty((n, 3), device="cuda") for _ in range(3)]
            ctx.check(ctx._lib.rm_sample_batch(ctx.handle, p(o), p(d), p(t), *args[:8], p(b[0]), p(b[1]), p(b[2]),
                                               None), "rm_sample_batch")
            s = native.RmScene()
            ctx._lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
            g = native.RmGrads()
            ctx._lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
            ctx.check(ctx._lib.rm_train_step(ctx.handle, p(b[0]), p(b[1]), p(b[2]), n, it / steps, 1.0 / (3 * n),
                                             ctypes.byref(s), ctypes.byref(march), ctypes.byref(g), p(loss), None, 0),
                      "rm_train_step")
            ctx.check(ctx._lib.rm_optimizer_step(ctx.handle, p(raw), p(grad), p(mom[0]), p(mom[1]), m, it, 0.01, 1e-5, 1,
                                                 ctypes.c_void_p(loss.data_ptr() + 4), p(act)), "rm_optimizer_step")
            torch.cuda.synchronize()
        out.append([x.clone() for x in (raw, act, grad, mom[0], mom[1], loss)])
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("m,nu,nf", [(7, 13107, 3277), (20, 9000, 7384), (32, 13107, 3277), (40, 13107, 3277),
                                     (9, 40000, 0)])
def test_train_iteration_equals_three_calls(rm, oracle, monkeypatch, m, nu, nf):
    """rm_train_iteration = rm_sample_batch -> rm_train_step -> rm_optimizer_step, bit for bit, over
    five iterations with penalties and k annealed (train.rs:169-198). One launch for M <= 32 and
    <= 16,384 rays; M = 40 and 40,000 rays run the three calls inside the entry point."""
    import torch
    render, model, native = rm
    rng = np.random.default_rng(m)
    cams = model.ring_cameras(4)
    rays = [oracle.camera_rays(64, 64, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    tg = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), train_scene(model, 6, 2), 24, 32.0)
    src = [dev(o), dev(d), dev(tg)]
    fg = torch.from_numpy(np.flatnonzero(tg.sum(1) > 0.01).astype(np.int32)).cuda()
    sc = train_scene(model, m, 40 + m)
    a = _iteration(torch, native, render, model, src, fg, nu, nf, sc, 5, True, monkeypatch)
    b = _iteration(torch, native, render, model, src, fg, nu, nf, sc, 5, False, monkeypatch)
    names = ("raw", "act", "grad", "adam_m", "adam_v", "loss")
    for it, (xa, xb) in enumerate(zip(a, b)):
        for name, u, v in zip(names, xa, xb):
            assert torch.equal(u, v), (it, name, (u - v).abs().max().item())
    assert torch.isfinite(a[-1][0]).all() and a[-1][5][0] > 0


@pytest.mark.parametrize("m,nu,nf", [(7, 13107, 3277), (32, 9000, 7384), (40, 13107, 3277), (9, 40000, 0)])
def test_train_step_sampled_equals_two_calls(rm, oracle, monkeypatch, m, nu, nf):
    """rm_train_step_sampled = rm_sample_batch -> rm_train_step, bit for bit (the gradient, the loss
    and, through the optimizer after it, the parameters), over five iterations with k annealed:
    the data-parallel rank's step before its all-reduce. One launch (the small kernel without its
    optimizer block) for M <= 32 and <= 16,384 rays; M = 40 and 40,000 rays run the two calls."""
    import torch
    render, model, native = rm
    cams = model.ring_cameras(4)
    rays = [oracle.camera_rays(64, 64, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    tg = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), train_scene(model, 6, 2), 24, 32.0)
    src = [dev(o), dev(d), dev(tg)]
    fg = torch.from_numpy(np.flatnonzero(tg.sum(1) > 0.01).astype(np.int32)).cuda()
    sc = train_scene(model, m, 60 + m)
    a = _iteration(torch, native, render, model, src, fg, nu, nf, sc, 5, "sampled", monkeypatch)
    b = _iteration(torch, native, render, model, src, fg, nu, nf, sc, 5, False, monkeypatch)
    names = ("raw", "act", "grad", "adam_m", "adam_v", "loss")
    for it, (xa, xb) in enumerate(zip(a, b)):
        for name, u, v in zip(names, xa, xb):
            assert torch.equal(u, v), (it, name, (u - v).abs().max().item())
    assert torch.isfinite(a[-1][2]).all() and a[-1][5][0] > 0


def test_train_step_sampled_arguments_and_empty_batch(rm):
    """rm_train_step_sampled's argument checks (dataset arrays, sampling sizes, foreground list,
    scene / march / grads: RM_ERR_INVALID_ARG, nothing launched) and an empty batch (no rays: the
    gradient and the loss sum are written as zeros, as rm_train_step with no rays writes them)."""
    import ctypes
    import torch
    render, model, native = rm
    ctx = render.context()
    lib = ctx._lib
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    m = 7
    src = torch.rand(64, 3, device="cuda")
    fg = torch.arange(8, dtype=torch.int32, device="cuda")
    act = torch.rand(model.packed_size(m), device="cuda")
    grad = torch.full((model.packed_size(m),), 7.0, device="cuda")
    loss = torch.full((1,), 7.0, device="cuda")
    s = native.RmScene()
    lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
    g = native.RmGrads()
    lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
    march = native.march_params(16, 32.0)

    def call(o, d, t, num_src, fgp, num_fg, nu, nf, scene=ctypes.byref(s), mp=ctypes.byref(march), gp=ctypes.byref(g)):
        return lib.rm_train_step_sampled(ctx.handle, o, d, t, num_src, fgp, num_fg, nu, nf, 1, 1, 1, 0.5, 1.0 / 3,
                                         scene, mp, gp, p(loss))
    assert call(None, p(src), p(src), 64, None, 0, 8, 0) == 1  # NULL dataset array
    assert call(p(src), p(src), p(src), 0, None, 0, 8, 0) == 1  # no source rows
    assert call(p(src), p(src), p(src), 64, None, 0, 8, -1) == 1  # negative count
    assert call(p(src), p(src), p(src), 64, None, 0, 4, 4) == 1  # n_fg > 0 without foreground indices
    assert call(p(src), p(src), p(src), 64, p(fg), 8, 4, 4, scene=None) == 1
    assert call(p(src), p(src), p(src), 64, p(fg), 8, 4, 4, gp=None) == 1
    torch.cuda.synchronize()
    assert torch.all(grad == 7.0) and loss.item() == 7.0  # nothing ran
    ctx.check(call(p(src), p(src), p(src), 64, p(fg), 8, 0, 0), "rm_train_step_sampled (empty)")
    torch.cuda.synchronize()
    assert torch.all(grad == 0.0) and loss.item() == 0.0


@pytest.mark.parametrize("m", [7, 24])
def test_train_step_sampled_color_f16(rm, oracle, m):
    """An fp16-colour model (RM_MARCH_COLOR_F16: the scene's colours are halves) through
    rm_train_step_sampled -- the multi-rank driver's step for every model, the fp16 growth runs
    included -- equals rm_sample_batch + rm_train_step bit for bit (gradient and loss sum)."""
    import ctypes
    import torch
    render, model, native = rm
    ctx = render.context()
    lib = ctx._lib
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    cams = model.ring_cameras(3)
    rays = [oracle.camera_rays(48, 48, *c, precision="f32") for c in cams]
    o = dev(np.concatenate([r[0] for r in rays]))
    d = dev(np.concatenate([r[1] for r in rays]))
    tg = dev(np.random.default_rng(m).uniform(size=(o.shape[0], 3)))
    fg = torch.arange(0, o.shape[0], 3, dtype=torch.int32, device="cuda")
    sc = train_scene(model, m, 70 + m)
    act = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"],
                                          sc["ambient"]).activated_packed().clone()
    col_h = act[3 * m:6 * m].half().contiguous()
    s = native.RmScene()
    lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
    s.colors = col_h.data_ptr()
    march = native.march_params(40, 20.0)
    march.flags |= native.RM_MARCH_COLOR_F16
    nu, nf = 5000, 1500
    out = []
    for sampled in (True, False):
        grad = torch.zeros(model.packed_size(m), device="cuda")
        loss = torch.zeros(1, device="cuda")
        g = native.RmGrads()
        lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
        args = (o.shape[0], p(fg), fg.numel(), nu, nf, 5, 2, 9)
        if sampled:
            ctx.check(lib.rm_train_step_sampled(ctx.handle, p(o), p(d), p(tg), *args, 0.4, 1.0 / (3 * (nu + nf)),
                                                ctypes.byref(s), ctypes.byref(march), ctypes.byref(g), p(loss)),
                      "rm_train_step_sampled")
        else:
            b = [torch.empty((nu + nf, 3), device="cuda") for _ in range(3)]
            ctx.check(lib.rm_sample_batch(ctx.handle, p(o), p(d), p(tg), *args, p(b[0]), p(b[1]), p(b[2]), None),
                      "rm_sample_batch")
            ctx.check(lib.rm_train_step(ctx.handle, p(b[0]), p(b[1]), p(b[2]), nu + nf, 0.4, 1.0 / (3 * (nu + nf)),
                                        ctypes.byref(s), ctypes.byref(march), ctypes.byref(g), p(loss), None, 0),
                      "rm_train_step")
        torch.cuda.synchronize()
        out.append((grad.clone(), loss.clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    assert torch.isfinite(out[0][0]).all() and out[0][1].item() > 0


@pytest.mark.parametrize("m,nu,nf,mode", [(7, 13107, 3277, "prepared"), (32, 9000, 7384, "prepared"),
                                          (9, 13107, 3277, "prepared_other_step"), (40, 13107, 3277, "prepared"),
                                          (9, 40000, 0, "prepared")])
def test_train_step_sampled_prepared(rm, oracle, monkeypatch, m, nu, nf, mode):
    """rm_train_step_sampled_prepared -> rm_optimizer_step (the data-parallel step: the optimizer's
    gradient-independent part in the sampled launch's extra block, the update alone after the
    all-reduce) = rm_sample_batch -> rm_train_step -> rm_optimizer_step, bit for bit, with the
    penalty loss; a preparation for another step number, more than 32 spheres and more than
    16,384 rays fall back to the full optimizer step, with the same bits."""
    import torch
    render, model, native = rm
    cams = model.ring_cameras(4)
    rays = [oracle.camera_rays(64, 64, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    tg = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), train_scene(model, 6, 2), 24, 32.0)
    src = [dev(o), dev(d), dev(tg)]
    fg = torch.from_numpy(np.flatnonzero(tg.sum(1) > 0.01).astype(np.int32)).cuda()
    sc = train_scene(model, m, 80 + m)
    a = _iteration(torch, native, render, model, src, fg, nu, nf, sc, 5, mode, monkeypatch)
    b = _iteration(torch, native, render, model, src, fg, nu, nf, sc, 5, False, monkeypatch)
    names = ("raw", "act", "grad", "adam_m", "adam_v", "loss")
    for it, (xa, xb) in enumerate(zip(a, b)):
        for name, u, v in zip(names, xa, xb):
            assert torch.equal(u, v), (it, name, (u - v).abs().max().item())
    assert a[-1][5][1] > 0  # the penalty share was written


def _f16_steps(torch, native, render, model, src, fg, nu, nf, sc, steps, monkeypatch, prepare):
    """`steps` data-parallel steps of an fp16-colour model (configs[4]'s colour format):
    rm_train_step_sampled_prepared -> rm_optimizer_step_f16 (colors_f16_out: the next render's
    colours); prepare False runs the same calls with RM_OPT_PREPARE=0 (the full optimizer)."""
    import ctypes
    monkeypatch.setenv("RM_OPT_PREPARE", "1" if prepare else "0")
    m = sc["centers"].shape[0]
    sm = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
    raw = sm.raw.clone()
    act = sm.activated_packed().clone()
    col_h = act[3 * m:6 * m].half().contiguous()
    npk = model.packed_size(m)
    grad = torch.zeros(npk, device="cuda")
    mom = [torch.zeros(npk, device="cuda") for _ in range(2)]
    loss = torch.zeros(2, device="cuda")
    ctx = render.context()
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    o, d, t = src
    n = nu + nf
    out = []
    for it in range(1, steps + 1):
        march = native.march_params(40, 5.0 + 27.0 * it / steps)
        march.flags |= native.RM_MARCH_COLOR_F16
        s = native.RmScene()
        ctx._lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
        s.colors = col_h.data_ptr()
        g = native.RmGrads()
        ctx._lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
        ctx.check(ctx._lib.rm_train_step_sampled_prepared(ctx.handle, p(o), p(d), p(t), o.shape[0], p(fg), fg.numel(),
                                                          nu, nf, 13, 1, it, it / steps, 1.0 / (3 * n), ctypes.byref(s),
                                                          ctypes.byref(march), ctypes.byref(g), p(loss), p(raw), it, 1,
                                                          ctypes.c_void_p(loss.data_ptr() + 4)),
                  "rm_train_step_sampled_prepared")
        ctx.check(ctx._lib.rm_optimizer_step_f16(ctx.handle, p(raw), p(grad), p(mom[0]), p(mom[1]), m, it, 0.01, 1e-5,
                                                 1, ctypes.c_void_p(loss.data_ptr() + 4), p(act), p(col_h)),
                  "rm_optimizer_step_f16")
        out.append([x.clone() for x in (raw, act, col_h, grad, mom[0], mom[1], loss)])
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("m", [7, 24])
def test_train_step_sampled_prepared_color_f16(rm, oracle, monkeypatch, m):
    """The multi-rank driver's prepared step on an fp16-colour model (configs[4] growth runs:
    rm_optimizer_step_f16 -> rm_optimizer_post_small with colors_f16_out) equals the full optimizer
    (RM_OPT_PREPARE=0) bit for bit: raw parameters, moments, activated values, the fp16 colours
    of the next render, gradient and losses, over five steps."""
    import torch
    render, model, native = rm
    cams = model.ring_cameras(4)
    rays = [oracle.camera_rays(64, 64, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    tg = oracle.render_diff(o.astype(np.float64), d.astype(np.float64), train_scene(model, 6, 2), 24, 32.0)
    src = [dev(o), dev(d), dev(tg)]
    fg = torch.from_numpy(np.flatnonzero(tg.sum(1) > 0.01).astype(np.int32)).cuda()
    sc = train_scene(model, m, 90 + m)
    a = _f16_steps(torch, native, render, model, src, fg, 13107, 3277, sc, 5, monkeypatch, True)
    b = _f16_steps(torch, native, render, model, src, fg, 13107, 3277, sc, 5, monkeypatch, False)
    names = ("raw", "act", "colors_f16", "grad", "adam_m", "adam_v", "loss")
    for it, (xa, xb) in enumerate(zip(a, b)):
        for name, u, v in zip(names, xa, xb):
            assert torch.equal(u, v), (it, name, (u.float() - v.float()).abs().max().item())
    assert a[-1][6][1] > 0


def test_prepared_step_dropped_by_another_call(rm, oracle, monkeypatch):
    """A preparation is dropped by any other library call before the optimizer step:
    prepare on the parameters, change them on the host side and call rm_scene_activate, then
    rm_optimizer_step -- it must compute on the changed parameters (equal to RM_OPT_PREPARE=0 with
    the same change), not apply the factors prepared on the old ones."""
    import ctypes
    import torch
    render, model, native = rm
    m, nu, nf = 7, 6000, 2000
    cams = model.ring_cameras(2)
    rays = [oracle.camera_rays(48, 48, *c, precision="f32") for c in cams]
    o = dev(np.concatenate([r[0] for r in rays]))
    d = dev(np.concatenate([r[1] for r in rays]))
    tg = dev(np.random.default_rng(5).uniform(size=(o.shape[0], 3)))
    fg = torch.arange(0, o.shape[0], 2, dtype=torch.int32, device="cuda")
    sc = train_scene(model, m, 123)
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    res = []
    for prepare in ("1", "0"):
        monkeypatch.setenv("RM_OPT_PREPARE", prepare)
        ctx = render.context()
        sm = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
        raw = sm.raw.clone()
        act = sm.activated_packed().clone()
        npk = model.packed_size(m)
        grad = torch.zeros(npk, device="cuda")
        mom = [torch.zeros(npk, device="cuda") for _ in range(2)]
        loss = torch.zeros(2, device="cuda")
        s = native.RmScene()
        ctx._lib.rm_scene_from_packed(p(act), m, ctypes.byref(s))
        g = native.RmGrads()
        ctx._lib.rm_grads_from_packed(p(grad), m, ctypes.byref(g))
        march = native.march_params(40, 20.0)
        ctx.check(ctx._lib.rm_train_step_sampled_prepared(ctx.handle, p(o), p(d), p(tg), o.shape[0], p(fg), fg.numel(),
                                                          nu, nf, 3, 1, 1, 0.5, 1.0 / (3 * (nu + nf)), ctypes.byref(s),
                                                          ctypes.byref(march), ctypes.byref(g), p(loss), p(raw), 1, 1,
                                                          ctypes.c_void_p(loss.data_ptr() + 4)),
                  "rm_train_step_sampled_prepared")
        torch.cuda.synchronize()
        raw.add_(0.25)  # a host-side change of the parameters (e.g. a broadcast) between the calls
        ctx.check(ctx._lib.rm_scene_activate(ctx.handle, p(raw), m, p(act)), "rm_scene_activate")
        ctx.check(ctx._lib.rm_optimizer_step(ctx.handle, p(raw), p(grad), p(mom[0]), p(mom[1]), m, 1, 0.01, 1e-5, 1,
                                             ctypes.c_void_p(loss.data_ptr() + 4), p(act)), "rm_optimizer_step")
        torch.cuda.synchronize()
        res.append([x.clone() for x in (raw, act, mom[0], mom[1], loss)])
    for name, u, v in zip(("raw", "act", "adam_m", "adam_v", "loss"), *res):
        assert torch.equal(u, v), (name, (u - v).abs().max().item())
