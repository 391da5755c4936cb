"""rm_train_step_camera_adam (train.rs:182-198 in one call): the camera-mode train step and the
optimizer step, the optimizer inside the gradient reduction for <= 64 spheres -- bit for bit the
two calls rm_train_step_camera -> rm_optimizer_step[_f16], over several steps (parameters,
moments, activated parameters, fp16 colours, gradient, loss, penalty), on the fused path (64 / 48
spheres, fp32 and fp16 colours, RM_FUSED_ADAM on and off) and on the fallbacks (the small-scene
kernel at 20 spheres, the multi-block optimizer at 100)."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

W = H = 64
S, K, LR = 32, 32.0, 0.02


def _models(model, m, f16):
    sc = model.synthetic_scene(m, 3)
    out = []
    for _ in range(2):
        mdl = model.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"],
                                              sc["ambient"], color_dtype="f16" if f16 else "f32")
        out.append((mdl, model.Adam(mdl, weight_decay=1e-5, with_penalties=True)))
    return out


def _state(torch, mdl, opt, g, loss, pen):
    t = [mdl.raw, mdl._act, opt.m, opt.v, g, loss, pen]
    if mdl._col_h is not None:
        t.append(mdl._col_h)
    return [x.clone() for x in t]


@pytest.mark.parametrize("m,f16", [(64, False), (48, True), (20, False), (100, False)])
def test_fused_adam_equals_two_calls(monkeypatch, m, f16):
    import torch
    from burn_raymarching_amd import model, render
    cams = model.ring_cameras(10)[:3]
    tg = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(m, 4)), K, S)
    results = []
    for fused_env in ("1", "0"):
        monkeypatch.setenv("RM_FUSED_ADAM", fused_env)
        (ma, oa), (mb, ob) = _models(model, m, f16)
        ga, la, pa = torch.zeros(model.packed_size(m), device="cuda"), torch.zeros(1, device="cuda"), \
            torch.zeros(1, device="cuda")
        gb, lb, pb = torch.zeros_like(ga), torch.zeros_like(la), torch.zeros_like(pa)
        for i in range(3):
            render.train_step_camera(cams, W, H, tg, ma.scene(), K, 0.3 + 0.1 * i, S, grads_packed=ga, loss=la)
            oa.step(ga, LR, penalty_out=pa)
            ob.train_step_camera(cams, W, H, tg, K, 0.3 + 0.1 * i, LR, S, grads_packed=gb, loss=lb, penalty_out=pb)
        torch.cuda.synchronize()
        sa, sb = _state(torch, ma, oa, ga, la, pa), _state(torch, mb, ob, gb, lb, pb)
        for k, (x, y) in enumerate(zip(sa, sb)):
            assert torch.equal(x, y), (fused_env, k)
        assert all(bool(torch.isfinite(x.float()).all()) for x in sb)
        results.append(sb)
    for x, y in zip(*results):  # the fused and unfused paths agree too
        assert torch.equal(x, y)


def test_fused_adam_with_step_scalars():
    """With a bound rm_step_scalars record (hipGraph mode) the fused call takes progress and Adam's
    step from the record and advances it, as the two calls do."""
    import torch
    from burn_raymarching_amd import model, render
    m = 64
    cams = model.ring_cameras(10)[:2]
    tg = render.render_diff_camera(cams, W, H, model.scene_tensors(model.synthetic_scene(m, 4)), K, S)
    ctx = render.context()
    (ma, oa), (mb, ob) = _models(model, m, False)
    out = []
    for mdl, opt, fused in ((ma, oa, False), (mb, ob, True)):
        rec = torch.tensor([1, 0, 10, 0], dtype=torch.int32, device="cuda")
        ctx.bind_step_scalars(rec.data_ptr())
        g, loss = torch.zeros(model.packed_size(m), device="cuda"), torch.zeros(1, device="cuda")
        for _ in range(3):
            if fused:
                opt.train_step_camera(cams, W, H, tg, K, 0.0, LR, S, grads_packed=g, loss=loss)
            else:
                render.train_step_camera(cams, W, H, tg, mdl.scene(), K, 0.0, S, grads_packed=g, loss=loss)
                opt.step(g, LR)
        torch.cuda.synchronize()
        ctx.bind_step_scalars(0)
        out.append((rec.clone(), mdl.raw.clone(), opt.m.clone(), g.clone(), loss.clone()))
    assert out[0][0].tolist() == [4, 3, 10, 0]
    for x, y in zip(*out):
        assert torch.equal(x, y)
