"""Split march (RM_MARCH_SPLIT / env RM_SPLIT=1): 32 rays per block (RM_SPLIT_RAYS) held by all four waves, each
wave summing a quarter of the sphere row blocks per march step, the quarters added in wave order.

  * against the fp64 oracle (forward, backward, train step) at sphere counts whose row blocks
    split evenly (256), unevenly (300: quarters of 4, 6, 4, 6 row blocks) and over many tiles
    (1100), and the split path really runs (its images differ from the unsplit ones in the last
    bits);
  * bit-for-bit properties the unsplit march has too: early exit on / off, shared origin step /
    per-ray first step, three consecutive train calls (the 2nd and 3rd in the cost order of the
    call before), camera mode in row order / array mode on the same rays, ragged ray counts;
  * the automatic choice (>= 256 spheres and <= 262,144 rays per launch, or >= 512 spheres and
    <= 1,048,576 rays) and RM_MARCH_NO_SPLIT.
Tolerances as in tests/test_gpu_parity.py.
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


def cam_rays(oracle, cams, w, h):
    rays = [oracle.camera_rays(w, h, *c, precision="f32") for c in cams]
    return np.concatenate([r[0] for r in rays]), np.concatenate([r[1] for r in rays])


@pytest.mark.parametrize("m", [256, 300, 1100])
def test_split_against_oracle(rm, oracle, monkeypatch, m):
    import torch
    render, model, _ = rm
    W = H = 48
    S, K = 32, 32.0
    sc = model.synthetic_scene(m, 11, radius_range=(0.02, 0.08))
    cams = model.ring_cameras(10, offset=4)[:2]
    o, d = cam_rays(oracle, cams, W, H)
    o64, d64 = o.astype(np.float64), d.astype(np.float64)
    s = model.scene_tensors(sc)
    monkeypatch.setenv("RM_SPLIT", "0")
    unsplit = render.render_diff_camera(cams, W, H, s, K, S)
    monkeypatch.setenv("RM_SPLIT", "1")
    out = render.render_diff_camera(cams, W, H, s, K, S)
    assert not torch.equal(out, unsplit)  # the quarters' sums are added in another order
    check_fwd(host(out), oracle.render_diff(o64, d64, sc, S, K))
    g = np.random.default_rng(3).normal(size=o.shape).astype(np.float32)
    check_grads(render.render_diff_backward_camera(cams, W, H, s, K, dev(g), S),
                oracle.render_diff_backward(o64, d64, sc, S, K, g.astype(np.float64)))
    targets = oracle.render_diff(o64, d64, model.synthetic_scene(m, 12, radius_range=(0.02, 0.08)), S,
                                 K).astype(np.float32)
    for _ in range(2):  # the 2nd call in the cost order of the 1st
        loss, gt, _ = render.train_step_camera(cams, W, H, dev(targets), s, K, 0.4, S)
    _, loss_ref, g_ref = oracle.train_step(o64, d64, targets.astype(np.float64), sc, S, K, 0.4)
    assert abs(host(loss)[0] - loss_ref) <= 1e-4 * abs(loss_ref)
    check_grads(gt, g_ref, mode="train")


def _train(render, native, cams, w, h, tg, s, k, steps, flags=0):
    import torch
    out = torch.empty_like(tg)
    loss, g, _ = render.train_step_camera(cams, w, h, tg, s, k, 0.3, steps, out=out,
                                          march=native.march_params(steps, k, flags=flags))
    torch.cuda.synchronize()
    return host(loss), {key: host(v) for key, v in g.items()}, host(out)


def _equal(a, b):
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2])
    for key in KEYS:
        assert np.array_equal(a[1][key], b[1][key]), key


def test_split_bitwise_properties(rm, monkeypatch):
    render, model, native = rm
    W = H = 64
    M, S, K = 300, 40, 32.0
    sc = model.scene_tensors(model.synthetic_scene(M, 13))
    cams = model.ring_cameras(10, offset=6)[:2]
    tg = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(M, 14)), K, S)
    monkeypatch.setenv("RM_SPLIT", "1")
    base = _train(render, native, cams, W, H, tg, sc, K, S)
    # three consecutive calls: the later ones in the cost order of the one before
    _equal(base, _train(render, native, cams, W, H, tg, sc, K, S))
    _equal(base, _train(render, native, cams, W, H, tg, sc, K, S))
    # early exit off
    _equal(base, _train(render, native, cams, W, H, tg, sc, K, S, flags=native.RM_MARCH_NO_EARLY_EXIT))
    # per-ray first step instead of the shared origin step
    _equal(base, _train(render, native, cams, W, H, tg, sc, K, S, flags=native.RM_MARCH_PER_RAY_ORIGIN))
    # static dispatch order
    _equal(base, _train(render, native, cams, W, H, tg, sc, K, S, flags=native.RM_MARCH_STATIC_ORDER))


def test_split_array_mode_and_ragged(rm, oracle, monkeypatch):
    """Array mode on the rays of a row-order camera launch gives the same image bit for bit, and
    ragged ray counts (a last block with 1..63 rays) stay within the oracle's tolerance."""
    import torch
    render, model, native = rm
    W, H = 40, 24
    M, S, K = 256, 24, 32.0
    sc = model.synthetic_scene(M, 15)
    s = model.scene_tensors(sc)
    cams = model.ring_cameras(10, offset=2)[:1]
    monkeypatch.setenv("RM_SPLIT", "1")
    monkeypatch.setenv("RM_ROW_ORDER", "1")
    cam_out = render.render_diff_camera(cams, W, H, s, K, S)
    o, d = cam_rays(oracle, cams, W, H)
    arr_out = render.render_diff_forward(dev(o), dev(d), s, K, S)
    assert torch.equal(cam_out, arr_out)
    for n in (1, 63, 65, 777):
        out = render.render_diff_forward(dev(o[:n]), dev(d[:n]), s, K, S)
        check_fwd(host(out), oracle.render_diff(o[:n].astype(np.float64), d[:n].astype(np.float64), sc, S, K))


def test_split_automatic_choice(rm, monkeypatch):
    """2048 spheres on a 32x32 view: the split march is taken automatically (the same bits as
    RM_SPLIT=1); RM_MARCH_NO_SPLIT gives the unsplit bits."""
    render, model, native = rm
    M, S, K = 2048, 16, 32.0
    s = model.scene_tensors(model.synthetic_scene(M, 16, radius_range=(0.01, 0.04)))
    cams = model.ring_cameras(10)[:1]
    tg = render.render_diff_camera(cams, 32, 32, model.scene_tensors(model.synthetic_scene(M, 17)), K, S)
    monkeypatch.delenv("RM_SPLIT", raising=False)
    auto = _train(render, native, cams, 32, 32, tg, s, K, S)
    no = _train(render, native, cams, 32, 32, tg, s, K, S, flags=native.RM_MARCH_NO_SPLIT)
    monkeypatch.setenv("RM_SPLIT", "1")
    forced = _train(render, native, cams, 32, 32, tg, s, K, S)
    monkeypatch.setenv("RM_SPLIT", "0")
    off = _train(render, native, cams, 32, 32, tg, s, K, S)
    _equal(auto, forced)
    _equal(no, off)
    assert not np.array_equal(auto[2], off[2])


@pytest.mark.parametrize("m,views,size,split", [(256, 1, 64, True), (512, 4, 96, True), (256, 10, 512, False),
                                                (128, 1, 64, False)])
def test_split_threshold(rm, monkeypatch, m, views, size, split):
    """The automatic choice at the thresholds: 256 spheres split up to 262,144 rays per launch,
    512 spheres up to 1,048,576; 10 views of 512x512 at 256 spheres (the bench metric) and fewer
    than 256 spheres stay unsplit. The automatic run equals (==) the forced one it picks."""
    render, model, native = rm
    S, K = 16, 32.0
    s = model.scene_tensors(model.synthetic_scene(m, 21, radius_range=(0.02, 0.08)))
    cams = model.ring_cameras(10)[:views]
    tg = render.render_diff_camera(cams, size, size, model.scene_tensors(model.synthetic_scene(m, 22)), K, S)
    monkeypatch.delenv("RM_SPLIT", raising=False)
    auto = _train(render, native, cams, size, size, tg, s, K, S)
    forced = _train(render, native, cams, size, size, tg, s, K, S,
                    flags=native.RM_MARCH_SPLIT if split else native.RM_MARCH_NO_SPLIT)
    _equal(auto, forced)


def test_split_continuation(rm, oracle, monkeypatch):
    """Continuation launches (split train / backward launches with S >= 64; ray mode): at step
    max(32, 3S/8) the groups still marching stop, their still-marching RAYS go on in a launch that
    marches 32 listed rays per block (from S >= 128 once more from 3S/4), and a resume launch runs
    the groups' post-march forward and backward from the rays' final states: bit-identical to one
    launch (RM_SPLIT_CONT_STEPS=0), to other continuation steps and to the march with the early exit
    off; the timed launches show first + continuations + resume; the image is within the oracle's
    tolerance."""
    render, model, native = rm
    W = H = 64
    M, S, K = 300, 64, 32.0
    sc = model.synthetic_scene(M, 23, radius_range=(0.02, 0.08))
    s = model.scene_tensors(sc)
    cams = model.ring_cameras(10, offset=3)[:2]
    tg = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(M, 24)), K, S)
    monkeypatch.setenv("RM_SPLIT", "1")
    monkeypatch.delenv("RM_SPLIT_CONT_STEPS", raising=False)
    monkeypatch.delenv("RM_SPLIT_CONT2_STEPS", raising=False)
    ctx = render.context()
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    base = _train(render, native, cams, W, H, tg, s, K, S)
    ctx.timing(False)
    _, launches = ctx.collect_timing(reset=True)
    assert launches == 3
    for steps in ("0", "8", "31", "40"):
        monkeypatch.setenv("RM_SPLIT_CONT_STEPS", steps)
        _equal(base, _train(render, native, cams, W, H, tg, s, K, S))
    monkeypatch.delenv("RM_SPLIT_CONT_STEPS")
    # a second continuation (three launches)
    monkeypatch.setenv("RM_SPLIT_CONT2_STEPS", "48")
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    _equal(base, _train(render, native, cams, W, H, tg, s, K, S))
    ctx.timing(False)
    assert ctx.collect_timing(reset=True)[1] == 4
    monkeypatch.delenv("RM_SPLIT_CONT2_STEPS")
    _equal(base, _train(render, native, cams, W, H, tg, s, K, S, flags=native.RM_MARCH_NO_EARLY_EXIT))
    # from S = 128 the default continues at 3S/16, 3S/8 and 3S/4: five launches, the one launch's bits
    tg2 = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(M, 24)), K, 128)
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    b128 = _train(render, native, cams, W, H, tg2, s, K, 128)
    ctx.timing(False)
    assert ctx.collect_timing(reset=True)[1] == 5
    monkeypatch.setenv("RM_SPLIT_CONT_STEPS", "0")
    _equal(b128, _train(render, native, cams, W, H, tg2, s, K, 128))
    monkeypatch.delenv("RM_SPLIT_CONT_STEPS")
    # four continuations (RM_SPLIT_CONT_LIST: the deferred lists alternate, each cleared ahead)
    monkeypatch.setenv("RM_SPLIT_CONT_LIST", "40,72,96,112")
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    _equal(b128, _train(render, native, cams, W, H, tg2, s, K, 128))
    ctx.timing(False)
    assert ctx.collect_timing(reset=True)[1] == 6
    monkeypatch.delenv("RM_SPLIT_CONT_LIST")
    o, d = cam_rays(oracle, cams, W, H)
    check_fwd(base[2].reshape(-1, 3), oracle.render_diff(o.astype(np.float64), d.astype(np.float64), sc, S, K))
    # the backward mode continues the same way (ragged: 3 views of 40x24 = 90 blocks of 32 rays)
    import torch
    cams3 = model.ring_cameras(10, offset=5)[:3]
    g = torch.randn((3 * 40 * 24, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(7))
    b0 = {k: host(v) for k, v in render.render_diff_backward_camera(cams3, 40, 24, s, K, g, S).items()}
    monkeypatch.setenv("RM_SPLIT_CONT_STEPS", "0")
    b1 = {k: host(v) for k, v in render.render_diff_backward_camera(cams3, 40, 24, s, K, g, S).items()}
    for key in KEYS:
        assert np.array_equal(b0[key], b1[key]), key


@pytest.mark.parametrize("m", [256, 300, 1100])
def test_split_costs_no_accuracy(rm, oracle, monkeypatch, m):
    """The split march's gradient error against the fp64 oracle is of the unsplit kernel's order and
    both sit below the fp32 reference order's own relative-L2 error at these cases. The two march
    with different soft-min shifts (ray mode: a fixed shift per ray against the unsplit kernel's
    per-wave choice), so they no longer agree to a fraction of their error; tools/split_margin.py over
    8 seeds (profiles/r07j_split_margin.jsonl): relL2 split <= 3.7e-4, unsplit <= 3.4e-4, fp32
    reference order <= 9.4e-4; split / unsplit relL2 <= 1.36, worst element at |g| >= 1e-2 4.2e-2
    against 4.3e-2."""
    from conftest import PER_SPHERE, grad_errors
    render, model, _ = rm
    W = H = 48
    S, K = 32, 32.0
    sc = model.synthetic_scene(m, 11, radius_range=(0.02, 0.08))
    cams = model.ring_cameras(10, offset=4)[:2]
    o, d = cam_rays(oracle, cams, W, H)
    g = np.random.default_rng(3).normal(size=o.shape).astype(np.float32)
    g64 = oracle.render_diff_backward(o.astype(np.float64), d.astype(np.float64), sc, S, K, g.astype(np.float64))
    g32 = oracle.render_diff_backward(o, d, sc, S, K, g, precision="f32")
    s = model.scene_tensors(sc)
    got = {}
    for env in ("1", "0"):
        monkeypatch.setenv("RM_SPLIT", env)
        got[env] = {k: host(v) for k, v in render.render_diff_backward_camera(cams, W, H, s, K, dev(g), S).items()}
    for key in PER_SPHERE:
        ref = np.asarray(g64[key], np.float64).reshape(-1)
        a, b = got["1"][key].reshape(-1).astype(np.float64), got["0"][key].reshape(-1).astype(np.float64)
        ea, eb = grad_errors(a, ref)[1], grad_errors(b, ref)[1]
        assert ea <= 1.5 * eb + 1e-6, key
        for e in (ea, eb):
            assert e <= grad_errors(g32[key], ref)[1], key


@pytest.mark.parametrize("k,flag", [(5.0, None), (32.0, "FORCE_MAX_SHIFT"), (32.0, "VALU_ONLY")])
def test_split_ray_mode_forms(rm, monkeypatch, k, flag):
    """Ray mode under the other soft-min paths: at k = 5 (the reference loop's first stage: the
    forms differ between rays more often), with the running maximum forced for every step
    (RM_MARCH_FORCE_MAX_SHIFT) and on the vector-only march (RM_MARCH_VALU_ONLY). The default
    continuation at S = 128 (five launches) equals one launch and the march with the exit off, bit
    for bit."""
    render, model, native = rm
    W = H = 48
    M, S = 300, 128
    s = model.scene_tensors(model.synthetic_scene(M, 31, radius_range=(0.02, 0.08)))
    cams = model.ring_cameras(10, offset=7)[:1]
    tg = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(M, 32)), k, S)
    f = getattr(native, "RM_MARCH_" + flag) if flag else 0
    monkeypatch.setenv("RM_SPLIT", "1")
    monkeypatch.delenv("RM_SPLIT_CONT_STEPS", raising=False)
    monkeypatch.delenv("RM_SPLIT_CONT_LIST", raising=False)
    ctx = render.context()
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    base = _train(render, native, cams, W, H, tg, s, k, S, flags=f)
    ctx.timing(False)
    assert ctx.collect_timing(reset=True)[1] == 5
    _equal(base, _train(render, native, cams, W, H, tg, s, k, S, flags=f | native.RM_MARCH_NO_EARLY_EXIT))
    monkeypatch.setenv("RM_SPLIT_CONT_STEPS", "0")
    _equal(base, _train(render, native, cams, W, H, tg, s, k, S, flags=f))


def test_split_ray_mode_array_ragged(rm, oracle, monkeypatch):
    """Array-mode train steps continue at the caps like camera mode, with a ragged last block
    (777 rays: 24 blocks of 32 and one of 9) and rays listed from any block: the same loss,
    gradients and image as one launch, bit for bit."""
    render, model, native = rm
    M, S, K = 300, 128, 32.0
    sc = model.synthetic_scene(M, 33, radius_range=(0.02, 0.08))
    s = model.scene_tensors(sc)
    cams = model.ring_cameras(10, offset=1)[:1]
    o, d = cam_rays(oracle, cams, 48, 48)
    sel = np.random.default_rng(5).permutation(o.shape[0])[:777]  # scattered rays: ragged, mixed tiles
    o, d = o[sel], d[sel]
    tg = np.random.default_rng(6).uniform(0.0, 1.0, size=o.shape).astype(np.float32)
    monkeypatch.setenv("RM_SPLIT", "1")
    monkeypatch.delenv("RM_SPLIT_CONT_LIST", raising=False)
    got = []
    for env in (None, "0"):
        if env is None:
            monkeypatch.delenv("RM_SPLIT_CONT_STEPS", raising=False)
        else:
            monkeypatch.setenv("RM_SPLIT_CONT_STEPS", env)
        ctx = render.context()
        ctx.collect_timing(reset=True)
        ctx.timing(True)
        loss, g, out = render.train_step(dev(o), dev(d), dev(tg), s, K, 0.3, S, with_out=True)
        ctx.timing(False)
        got.append((host(loss), {key: host(v) for key, v in g.items()}, host(out),
                    ctx.collect_timing(reset=True)[1]))
    assert got[0][3] == 5 and got[1][3] == 1
    _equal(got[0][:3], got[1][:3])


def test_split_ray_mode_sub_launches(rm, oracle, monkeypatch):
    """A call split into sub-launches (RM_MAX_BLOCKS_PER_LAUNCH=40: 90 groups of 32 rays in three
    sub-launches, gradients accumulated) continues each sub-launch at the caps with the buffers of
    the one before reused: the same bits as one launch per sub-launch, and within the oracle's
    tolerance of the whole-call result."""
    render, model, native = rm
    M, S, K = 300, 128, 32.0
    sc = model.synthetic_scene(M, 35, radius_range=(0.02, 0.08))
    s = model.scene_tensors(sc)
    cams = model.ring_cameras(10, offset=8)[:3]
    tg = render.render_diff_camera(cams, 40, 24, model.scene_tensors(model.synthetic_scene(M, 36)), K, S)
    monkeypatch.setenv("RM_SPLIT", "1")
    monkeypatch.delenv("RM_SPLIT_CONT_LIST", raising=False)
    monkeypatch.delenv("RM_SPLIT_CONT_STEPS", raising=False)
    whole = _train(render, native, cams, 40, 24, tg, s, K, S)
    monkeypatch.setenv("RM_MAX_BLOCKS_PER_LAUNCH", "40")
    ctx = render.context()
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    sub = _train(render, native, cams, 40, 24, tg, s, K, S)
    ctx.timing(False)
    assert ctx.collect_timing(reset=True)[1] == 3 * 5
    monkeypatch.setenv("RM_SPLIT_CONT_STEPS", "0")
    _equal(sub, _train(render, native, cams, 40, 24, tg, s, K, S))
    np.testing.assert_array_equal(sub[2], whole[2])  # the image does not depend on the grouping
    for key in KEYS:
        a, b = sub[1][key], whole[1][key]
        assert np.abs(a - b).max() <= 1e-5 * max(np.abs(b).max(), 1e-12), key


def test_split_ray_mode_saved_t(rm, oracle, monkeypatch):
    """The split backward from the forward's saved march t (t_march: no march, no continuation)
    equals the backward that marches again through the ray-mode continuations, bit for bit; the
    forward's t is the same whether its march ran in one launch or not (forward calls never
    continue), and retired and gone rays hand over their final t."""
    render, model, _ = rm
    M, S, K = 300, 128, 32.0
    sc = model.synthetic_scene(M, 37, radius_range=(0.02, 0.08))
    s = model.scene_tensors(sc)
    cams = model.ring_cameras(10, offset=9)[:1]
    o, d = cam_rays(oracle, cams, 48, 48)
    monkeypatch.setenv("RM_SPLIT", "1")
    monkeypatch.delenv("RM_SPLIT_CONT_LIST", raising=False)
    monkeypatch.delenv("RM_SPLIT_CONT_STEPS", raising=False)
    _, t = render.render_diff_forward(dev(o), dev(d), s, K, S, return_t=True)
    g = dev(np.random.default_rng(8).normal(size=o.shape).astype(np.float32))
    a = render.render_diff_backward(dev(o), dev(d), s, K, g, S)
    b = render.render_diff_backward(dev(o), dev(d), s, K, g, S, t_march=t)
    for key in a:
        assert np.array_equal(host(a[key]), host(b[key])), key
