"""Launch fusions that must not change a bit:
  * the reduction's second pass inside rm_reduce_partials (the last-arriving segment block of each
    column block, RM_REDUCE_FUSED) against its own launch (rm_finalize_grads);
  * the one-block optimizer of small models (rm_optimizer_small) against the oracle-free
    reference of test_gpu_parity.py (covered there); here: repeated steps are deterministic."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]
KEYS = ("centers", "colors", "radius", "light_dir", "ambient")


@pytest.fixture(scope="module")
def mods():
    import torch
    from burn_raymarching_amd import model, native, render
    torch.cuda.init()
    return torch, model, native, render


def _train(torch, model, render, m, views, w, steps):
    sc = model.scene_tensors(model.synthetic_scene(m, 3), "cuda")
    cams = model.ring_cameras(10)[:views]
    tgt = render.render_diff_camera(cams, w, w, model.scene_tensors(model.synthetic_scene(m, 4), "cuda"), 32.0, steps)
    out = torch.empty_like(tgt)
    loss, g, _ = render.train_step_camera(cams, w, w, tgt, sc, 32.0, 0.4, steps, out=out)
    torch.cuda.synchronize()
    return loss.clone(), {k: v.clone() for k, v in g.items()}, out


@pytest.mark.parametrize("env,m,views,w", [("RM_REDUCE_FUSED", 64, 3, 128), ("RM_REDUCE_FUSED", 256, 2, 256),
                                           ("RM_REDUCE_FUSED", 1100, 1, 64), ("RM_REDUCE_FUSED", 40, 16, 32)])
def test_fused_launch_is_bitwise_equal(mods, monkeypatch, env, m, views, w):
    torch, model, _, render = mods
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setenv(env, flag)
        res[flag] = [_train(torch, model, render, m, views, w, 24) for _ in range(2)]
    for r in res["0"] + res["1"][1:]:
        assert torch.equal(r[0], res["1"][0][0]) and torch.equal(r[2], res["1"][0][2])
        for k in KEYS:
            assert torch.equal(r[1][k], res["1"][0][1][k]), (env, k)


def test_small_optimizer_deterministic(mods):
    torch, model, _, _ = mods
    outs = []
    for _ in range(2):
        sc = model.synthetic_scene(48, 2)
        sm = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
        opt = model.Adam(sm, weight_decay=1e-5, with_penalties=True)
        g = torch.randn(model.packed_size(48), device="cuda", generator=torch.Generator("cuda").manual_seed(4))
        pen = torch.zeros(1, device="cuda")
        for _ in range(3):
            opt.step(g, 0.05, penalty_out=pen)
        outs.append((sm.raw.clone(), pen.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("m", [9, 64])
def test_small_optimizer_matches_two_kernel_path(mods, monkeypatch, m):
    """rm_optimizer_small (one block) against rm_penalty_pairs + rm_optimizer_kernel (RM_OPT_SMALL=0):
    the same update; the repulsion sums are added in another order (fp32 rounding)."""
    torch, model, _, _ = mods
    res = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("RM_OPT_SMALL", flag)
        sc = model.synthetic_scene(m, 5)
        sm = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
        opt = model.Adam(sm, weight_decay=1e-5, with_penalties=True)
        g = torch.randn(model.packed_size(m), device="cuda", generator=torch.Generator("cuda").manual_seed(6))
        pen = torch.zeros(1, device="cuda")
        for _ in range(3):
            opt.step(g, 0.05, penalty_out=pen)
        res[flag] = (sm.raw.clone(), pen.clone(), sm.activated_packed().clone())
    for a, b in zip(res["1"], res["0"]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()


@pytest.mark.timeout(240)
def test_reduce_handoff_stress_under_uneven_load(mods, monkeypatch):
    """The in-launch hand-offs (rm_reduce_partials' last-arriving segment block, the small kernel's
    last block): write-through (sc1) record stores drained by every storing wave before the block
    barrier, one lane's relaxed agent-scope arrival, an agent-scope acquire in the last block
    (MI355X_MICROARCH.md, inter-workgroup visibility: the write-through form that needs no release
    fence). Stressed where stale data would show: many column blocks and segments (4096 spheres:
    129 column blocks x 128 segments), repeated, while another stream keeps the CUs unevenly busy
    and the consumers' L1 warm; every result bitwise equal to the two-launch reduction
    (RM_REDUCE_FUSED=0), whose pass 2 reads after a kernel boundary."""
    torch, model, _, render = mods
    cases = ((4096, 2, 64), (1100, 1, 96), (24, 4, 64))  # the last: the small kernel's hand-off
    monkeypatch.setenv("RM_REDUCE_FUSED", "0")
    ref = {c: _train(torch, model, render, *c, 24) for c in cases}  # idle chip, two-launch reduction
    monkeypatch.setenv("RM_REDUCE_FUSED", "1")
    side = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda")
    for it in range(6):
        with torch.cuda.stream(side):  # uneven load: a GEMM stream competing for the CUs
            for _ in range(1 + it % 3):
                a = torch.tanh(a @ a * 1e-3)
        for c in cases:
            got = _train(torch, model, render, *c, 24)
            assert torch.equal(got[0], ref[c][0]), (it, c)
            for k in KEYS:
                assert torch.equal(got[1][k], ref[c][1][k]), (it, c, k)
    torch.cuda.synchronize()
