"""hipGraph capture of a training step (raymarch.h, "hipGraph capture of a training step"): a step
of bench.py's shape -- rm_train_step_camera (records, origin steps, train kernel, reduction) then
rm_optimizer_step -- captured once with torch.cuda.CUDAGraph over the rm_* calls and replayed,
gives the eager steps' results bit for bit (also for a call of more than 16 views, whose camera
bases the captured call reads from the context's device table): the per-step scalars (compute_loss's progress, Adam's
step) come from a device record the optimizer advances (rm_bind_step_scalars), and the cost-ordered
dispatch rotates its list sets on the device (the replayed launches keep using the previous step's
cost order)."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _setup(torch, rmm, rmr, native, m, w, views, steps, order):
    sc0, sc1 = rmm.synthetic_scene(m, 0), rmm.synthetic_scene(m, 1)
    cams = rmm.ring_cameras(views)
    tg = rmr.render_diff_camera(cams, w, w, rmm.scene_tensors(sc1), 32.0, steps).view(-1, 3).contiguous()
    model = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"],
                                          sc0["ambient"])
    opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
    march = native.march_params(steps, 32.0, flags=0 if order == "cost" else native.RM_MARCH_STATIC_ORDER)
    buf = torch.zeros(rmm.packed_size(m) + 1, device="cuda")
    inv = 1.0 / (3.0 * views * w * w)

    def step():
        rmr.train_step_camera(cams, w, w, tg, model.scene(), 32.0, 0.0, steps, inv_count=inv,
                              grads_packed=buf[:-1], loss=buf[-1:], march=march)
        opt.step(buf[:-1], 0.05)
    return model, opt, buf, step


@pytest.mark.parametrize("order", ["cost", "static"])
@pytest.mark.parametrize("m,w,views,steps", [(64, 128, 4, 24), (300, 64, 2, 64), (40, 32, 20, 16)])
def test_graph_replay_equals_eager(order, m, w, views, steps):
    import torch
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr
    total, warm, n = 40, 3, 6
    s = torch.cuda.Stream()
    runs = {}
    with torch.cuda.stream(s):
        ctx = rmr.context()
        for mode in ("eager", "graph"):
            sdev = torch.tensor([1, 0, total, 0], dtype=torch.int32, device="cuda")
            ctx.bind_step_scalars(sdev.data_ptr())
            try:
                model, opt, buf, step = _setup(torch, rmm, rmr, native, m, w, views, steps, order)
                for _ in range(warm):
                    step()
                torch.cuda.synchronize()
                seq = []
                if mode == "eager":
                    for _ in range(n):
                        step()
                        seq.append((model.raw.clone(), buf.clone()))
                else:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        step()
                    assert sdev.tolist()[:2] == [warm + 1, warm]  # captured, not run
                    for _ in range(n):
                        g.replay()
                        seq.append((model.raw.clone(), buf.clone()))
                torch.cuda.synchronize()
                assert sdev.tolist()[:2] == [warm + n + 1, warm + n]  # the optimizer advanced the record
                if order == "cost":
                    counts, nxt = ctx.order_counts()
                    assert sum(counts[(nxt + 2) % 3]) > 0  # the last replayed launch appended its lists
                runs[mode] = seq
            finally:
                ctx.bind_step_scalars(None)
    for k, ((ra, ba), (rb, bb)) in enumerate(zip(runs["eager"], runs["graph"])):
        assert torch.equal(ba, bb), k  # gradient + loss of the step
        assert torch.equal(ra, rb), k  # parameters after the optimizer


def test_bound_scalars_match_by_value_arguments():
    """A bound record gives the same step as the by-value arguments (progress = index / total in
    fp32, Adam's step): bound and unbound eager runs agree bit for bit."""
    import torch
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr
    m, w, views, steps, total = 48, 64, 2, 24, 10
    ctx = rmr.context()
    out = []
    for bound in (False, True):
        sdev = torch.tensor([1, 0, total, 0], dtype=torch.int32, device="cuda")
        if bound:
            ctx.bind_step_scalars(sdev.data_ptr())
        try:
            sc0, sc1 = rmm.synthetic_scene(m, 2), rmm.synthetic_scene(m, 3)
            cams = rmm.ring_cameras(views)
            tg = rmr.render_diff_camera(cams, w, w, rmm.scene_tensors(sc1), 32.0, steps).view(-1, 3).contiguous()
            model = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"],
                                                  sc0["ambient"])
            opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
            buf = torch.zeros(rmm.packed_size(m) + 1, device="cuda")
            for i in range(4):
                prog = float(np.float32(i) / np.float32(total))
                rmr.train_step_camera(cams, w, w, tg, model.scene(), 32.0, prog, steps,
                                      inv_count=1.0 / (3.0 * views * w * w), grads_packed=buf[:-1], loss=buf[-1:])
                opt.step(buf[:-1], 0.05)
            torch.cuda.synchronize()
            out.append((model.raw.clone(), buf.clone()))
        finally:
            ctx.bind_step_scalars(None)
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
