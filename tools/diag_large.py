"""Finiteness probe at large M / S (BASELINE configs[4] shape): one camera-mode train step, then a
few Adam steps, reporting where non-finite values first appear."""
import sys

import torch

sys.path.insert(0, ".")
from burn_raymarching_amd import model as rmm, native, render as rmr  # noqa: E402


def finite(name, t):
    ok = bool(torch.isfinite(t).all().item())
    if not ok:
        bad = (~torch.isfinite(t)).nonzero()
        print(f"  {name}: {bad.shape[0]} non-finite, first at {bad[:3].tolist()}", flush=True)
    return ok


def main():
    M, S, W = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    rr = (0.01, 0.04) if M > 1024 else (0.03, 0.12)
    sc0 = rmm.synthetic_scene(M, seed=0, radius_range=rr)
    sc1 = rmm.synthetic_scene(M, seed=1, radius_range=rr)
    cams = rmm.ring_cameras(10)[:1]
    tgt = rmr.render_diff_camera(cams, W, W, rmm.scene_tensors(sc1), 32.0, S)
    print("target finite", finite("target", tgt), flush=True)
    model = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"], sc0["ambient"])
    opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
    for it in range(6):
        out = torch.empty_like(tgt)
        loss, g, _ = rmr.train_step_camera(cams, W, W, tgt, model.scene(), 32.0, 0.5, S, out=out)
        torch.cuda.synchronize()
        ok = finite("out", out) & finite("loss", loss)
        for k, v in g.items():
            ok &= finite("grad " + k, v)
        print(f"step {it}: loss {loss.item():.6g} finite {ok}", flush=True)
        if not ok:
            break
        packed = torch.cat([g[k].reshape(-1) for k in ("centers", "colors", "radius", "light_dir", "ambient")])
        opt.step(packed, 0.05)
        print("  raw finite", finite("raw", model.raw), flush=True)


if __name__ == "__main__":
    main()
