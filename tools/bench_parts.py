"""Stage timing of the fused kernels at the metric workload (512x512, 256 spheres, 32 steps),
via the C ABI's hipEvent kernel timing. Prints one JSON line per variant.

  fwd_S32      forward-only, full march                      (rm_render_diff_camera)
  fwd_S0       forward-only, no march (reconnect+normal+shade)
  bwd_t        backward given the saved march t              (march skipped)
  train        fused train step (what bench.py times)
Differences isolate the march, the post-march forward and the backward sweeps.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from burn_raymarching_amd import model, render  # noqa: E402


def timed(ctx, fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ctx.collect_timing(reset=True)
    ctx.timing(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    ctx.timing(False)
    ms, n = ctx.collect_timing(reset=True)
    return ms / max(n, 1)


def main():
    W = int(os.environ.get("RM_W", "512"))
    M = int(os.environ.get("RM_M", "256"))
    S = int(os.environ.get("RM_S", "32"))
    V = int(os.environ.get("RM_V", "2"))
    sc = model.scene_tensors(model.synthetic_scene(M, 0))
    cams = model.ring_cameras(10)[:V]
    ctx = render.context()
    tgt = render.render_diff_camera(cams, W, W, model.scene_tensors(model.synthetic_scene(M, 1)), 32.0, S)
    _, t = render.render_diff_camera(cams, W, W, sc, 32.0, S, return_t=True)
    g = torch.randn((V * W * W, 3), device="cuda")
    res = {
        "fwd_S32": timed(ctx, lambda: render.render_diff_camera(cams, W, W, sc, 32.0, S)),
        "fwd_S0": timed(ctx, lambda: render.render_diff_camera(cams, W, W, sc, 32.0, 0)),
        "bwd_t": timed(ctx, lambda: render.render_diff_backward_camera(cams, W, W, sc, 32.0, g, S, t_march=t)),
        "train": timed(ctx, lambda: render.train_step_camera(cams, W, W, tgt, sc, 32.0, 0.5, S)),
    }
    res["march_only"] = res["fwd_S32"] - res["fwd_S0"]
    res["backward_sweeps"] = res["bwd_t"] - res["fwd_S0"]
    res["config"] = {"W": W, "M": M, "S": S, "V": V}
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
