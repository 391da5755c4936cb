"""Does every train launch of a repeated call use the cost order? C2's step (256x256, 64 spheres,
32 steps, 10 views, rm_train_step_camera + rm_optimizer_step) for --steps steps: per launch the
train kernel's hipEvent time, the device turn (the list set the next launch appends to) and the
per-set block totals after the launch (the next launch reads set (turn + 2) % 3 and takes the cost
order only when its total equals the launch's block count); then the same steps with the static
order for comparison.

    python tools/order_probe.py [--steps 15]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=15)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--spheres", type=int, default=64)
    ap.add_argument("--views", type=int, default=10)
    args = ap.parse_args()
    import torch
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr
    W, M, S, V = args.width, args.spheres, 32, args.views
    blocks = V * (W // 16) * (W // 16)
    out = {"blocks_per_launch": blocks}
    for mode in ("cost", "static"):
        sc0, sc1 = rmm.synthetic_scene(M, 0), rmm.synthetic_scene(M, 1)
        cams = rmm.ring_cameras(V)
        tg = rmr.render_diff_camera(cams, W, W, rmm.scene_tensors(sc1), 32.0, S).view(-1, 3).contiguous()
        model = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"],
                                              sc0["ambient"])
        opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
        march = native.march_params(S, 32.0, flags=0 if mode == "cost" else native.RM_MARCH_STATIC_ORDER)
        buf = torch.zeros(rmm.packed_size(M) + 1, device="cuda")
        ctx = native.Context(torch.cuda.current_device(), torch.cuda.current_stream().cuda_stream)
        rows = []
        for i in range(args.steps):
            ctx.timing(True)
            rmr.train_step_camera(cams, W, W, tg, model.scene(), 32.0, 0.5, S, inv_count=1.0 / (3 * V * W * W),
                                  grads_packed=buf[:-1], loss=buf[-1:], march=march, ctx=ctx)
            ms, n = ctx.collect_timing(reset=True)
            ctx.timing(False)
            opt.step(buf[:-1], 0.05)
            counts, nxt = ctx.order_counts()
            rows.append({"step": i, "kernel_ms": round(ms, 4), "turn": nxt,
                         "set_totals": [sum(c) for c in counts],
                         "next_reads_total": sum(counts[(nxt + 2) % 3])})
        out[mode] = rows
        ctx.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
