import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from burn_raymarching_amd import model, render
from oracle import oracle as orc
orc.build()
def dev(x): return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()
for m, n in ((1, 257), (4, 257), (8, 4096), (9, 16384)):
    sc = model.synthetic_scene(m, m + n)
    cams = model.ring_cameras(3, offset=0)
    rays = [orc.camera_rays(48, 48, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays]); d = np.concatenate([r[1] for r in rays])
    idx = np.random.default_rng(n).integers(0, o.shape[0], n); o, d = o[idx], d[idx]
    g = np.random.default_rng(n).normal(size=o.shape)
    ref = orc.render_diff_backward(o.astype(np.float64), d.astype(np.float64), sc, 20, 24.0, g)
    s = model.scene_tensors(sc)
    for env in (("1", "1"), ("1", "0"), ("0", "1")):
        os.environ["RM_SMALL"], os.environ["RM_SMALL_FINAL"] = env
        got = render.render_diff_backward(dev(o), dev(d), s, 24.0, dev(g), 20)
        torch.cuda.synchronize()
        print(m, n, env, {k: float(np.abs(got[k].cpu().numpy().reshape(-1) - ref[k].reshape(-1)).max() / max(np.abs(ref[k]).max(), 1e-30)) for k in ref}, flush=True)
    print("ref centers", ref["centers"].reshape(-1)[:6], "got", got["centers"].cpu().numpy().reshape(-1)[:6])
