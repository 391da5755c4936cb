"""How much of a small config's step is launch overhead a hipGraph removes?

The C2-shaped step (256x256 / 64 spheres / 32 steps / 10 views, synthetic scene and targets, camera
mode; static dispatch order, since a captured launch keeps the cost-order list set it was captured
with) as bench.py runs it -- rm_train_step_camera (records, origin steps, train kernel, reduction)
then rm_optimizer_step -- timed eagerly and as a torch.cuda.CUDAGraph of one step replayed. The
graph freezes the step's by-value scalars (progress, Adam's step), so this is a timing probe, not a
training run: both legs run the same kernels on the same data.

    python tools/graph_probe.py [--width 256 --spheres 64 --march-steps 32 --views 10 --steps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--spheres", type=int, default=64)
    ap.add_argument("--march-steps", type=int, default=32)
    ap.add_argument("--views", type=int, default=10)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--order", choices=["static", "cost"], default="static")
    args = ap.parse_args()
    import torch
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr
    W = H = args.width
    M, S, K, V = args.spheres, args.march_steps, 32.0, args.views
    s = torch.cuda.Stream()
    res = {}
    with torch.cuda.stream(s):
        sc0, sc1 = rmm.synthetic_scene(M, 0), rmm.synthetic_scene(M, 1)
        cams = rmm.ring_cameras(V)
        tg = rmr.render_diff_camera(cams, W, H, rmm.scene_tensors(sc1), K, S).view(-1, 3).contiguous()
        m = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"], sc0["ambient"])
        opt = rmm.Adam(m, weight_decay=1e-5, with_penalties=True)
        flags = native.RM_MARCH_STATIC_ORDER if args.order == "static" else 0
        march = native.march_params(S, K, flags=flags)
        buf = torch.zeros(rmm.packed_size(M) + 1, device="cuda")
        inv = 1.0 / (3.0 * V * W * H)

        def step():
            rmr.train_step_camera(cams, W, H, tg, m.scene(), K, 0.5, S, inv_count=inv,
                                  grads_packed=buf[:-1], loss=buf[-1:], march=march)
            opt.step(buf[:-1], 0.05)

        for _ in range(5):
            step()
        torch.cuda.synchronize()

        def timed(fn, n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / n * 1e3

        res["eager_ms"] = timed(step, args.steps)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            step()
        g.replay()
        res["graph_ms"] = timed(g.replay, args.steps)
        res["eager_ms_again"] = timed(step, args.steps)
    res.update(vars(args))
    res["saved_us_per_step"] = round((min(res["eager_ms"], res["eager_ms_again"]) - res["graph_ms"]) * 1e3, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
