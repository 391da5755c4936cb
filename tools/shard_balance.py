#!/usr/bin/env python3
"""How evenly the strong-scaling default's 80 views split over 2 / 4 / 8 ranks (one GPU).

bench.py's strong mode gives rank r of N a contiguous slice of the 80-camera ring; the step
time of an N-GPU run is the slowest rank's. This replays each rank's slice on one GPU (the same
scene, targets and optimizer state as bench.py after --warm steps of the 80-view step), each
slice on its own rm_context (so its cost-ordered dispatch comes from its own previous call, as
on a rank), and reports per-slice train-call times: max / mean per N is the load imbalance a
SCALE run pays. Two assignments of camera angles to ring positions are compared:
  contiguous  -- ring position j looks from angle j (bench.py's ring before --ring-order)
  spread      -- ring position j looks from angle (j * 49) mod 80 (bench.py --ring-order spread):
                 any contiguous slice of the ring covers the circle evenly

    python tools/shard_balance.py [--warm 5] [--reps 5]      (prints one JSON object)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--views", type=int, default=80)
    ap.add_argument("--ranks", type=int, nargs="+", default=[2, 4, 8])
    args = ap.parse_args()
    import torch
    from bench import ring_order
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr
    from burn_raymarching_amd.parallel import Shard

    W = H = 512
    M, S, K, V = 256, 32, 32.0, args.views
    npix = W * H
    sc0 = rmm.synthetic_scene(M, seed=0, radius_range=(0.03, 0.12))
    sc1 = rmm.synthetic_scene(M, seed=1, radius_range=(0.03, 0.12))
    tgt_scene = rmm.scene_tensors(sc1)
    out = {"views": V, "warm": args.warm, "reps": args.reps}
    for order in ("contiguous", "spread"):
        cams = [rmm.ring_cameras(V)[a] for a in ring_order(V, order)]
        targets = torch.empty((V, npix, 3), device="cuda")
        for v0 in range(0, V, native.RM_MAX_VIEWS_PER_CALL):
            ch = cams[v0:v0 + native.RM_MAX_VIEWS_PER_CALL]
            targets[v0:v0 + len(ch)] = rmr.render_diff_camera(ch, W, H, tgt_scene, K, S).view(len(ch), npix, 3)
        model = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"],
                                              sc0["ambient"])
        opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
        march = native.march_params(S, K)
        g = torch.zeros(rmm.packed_size(M), device="cuda")
        loss = torch.zeros(1, device="cuda")
        inv = 1.0 / (3.0 * V * npix)
        for i in range(args.warm):  # the N = 1 step over all views, as bench.py's warm-up
            rmr.train_step_camera(cams, W, H, targets.view(-1, 3), model.scene(), K, progress=i / 35, steps=S,
                                  inv_count=inv, grads_packed=g, loss=loss, march=march)
            opt.step(g, 0.05)
        torch.cuda.synchronize()
        res = {}
        for n in args.ranks:
            times = []
            for r in range(n):
                sh = Shard(r, n, 0, V, V)
                vs = sh.views(0)
                tg = targets[vs[0]:vs[0] + len(vs)].reshape(-1, 3)
                ctx = native.Context(torch.cuda.current_device())
                kw = dict(progress=0.2, steps=S, inv_count=inv, grads_packed=g, loss=loss, march=march, ctx=ctx)
                for _ in range(2):  # seeds this context's cost order (its own previous call)
                    rmr.train_step_camera([cams[j] for j in vs], W, H, tg, model.scene(), K, **kw)
                torch.cuda.synchronize()
                ms = []
                for _ in range(args.reps):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    rmr.train_step_camera([cams[j] for j in vs], W, H, tg, model.scene(), K, **kw)
                    e1.record()
                    torch.cuda.synchronize()
                    ms.append(e0.elapsed_time(e1))
                ms.sort()
                times.append(ms[len(ms) // 2])
            mean = sum(times) / len(times)
            res[str(n)] = {"slice_ms": [round(t, 4) for t in times], "max_over_mean": round(max(times) / mean, 4),
                           "min_over_mean": round(min(times) / mean, 4)}
        out[order] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
