"""Where does the split march's gradient error sit against the fp32 reference order?

For the cases of tests/test_gpu_split.py::test_split_against_oracle (48x48, two ring views, radii
U[0.02, 0.08], 32 steps, k = 32, a seeded N(0,1) dL/dout) over several scene seeds: the backward
through the split march (RM_SPLIT=1), the unsplit general kernel (RM_SPLIT=0) and the oracle's
fp32 reference-order restatement, each against the fp64 oracle -- relative L2 and the per-element
tiers of tests/conftest.py::check_grads. One JSON object per line, then a summary.

    python tools/split_margin.py [--seeds 11 12 ...] [--spheres 256 300 1100] > out.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=list(range(11, 19)))
    ap.add_argument("--spheres", type=int, nargs="+", default=[256, 300, 1100])
    args = ap.parse_args()
    import torch
    from burn_raymarching_amd import model, render
    from conftest import grad_errors
    from oracle import oracle
    W = H = 48
    S, K = 32, 32.0
    cams = model.ring_cameras(10, offset=4)[:2]
    rays = [oracle.camera_rays(W, H, *c, precision="f32") for c in cams]
    o = np.concatenate([r[0] for r in rays])
    d = np.concatenate([r[1] for r in rays])
    g = np.random.default_rng(3).normal(size=o.shape).astype(np.float32)
    summary = {}
    for m in args.spheres:
        for seed in args.seeds:
            sc = model.synthetic_scene(m, seed, radius_range=(0.02, 0.08))
            g64 = oracle.render_diff_backward(o.astype(np.float64), d.astype(np.float64), sc, S, K,
                                              g.astype(np.float64), precision="f64")
            res = {"fp32_ref": oracle.render_diff_backward(o, d, sc, S, K, g, precision="f32")}
            s = model.scene_tensors(sc)
            gt = torch.from_numpy(g).cuda()
            for name, env in (("gpu_split", "1"), ("gpu_unsplit", "0")):
                os.environ["RM_SPLIT"] = env
                got = render.render_diff_backward_camera(cams, W, H, s, K, gt, S)
                res[name] = {k: v.detach().cpu().numpy() for k, v in got.items()}
            os.environ.pop("RM_SPLIT", None)
            line = {"spheres": m, "seed": seed}
            for key in ("centers", "colors", "radius"):
                ref = np.asarray(g64[key], np.float64).reshape(-1)
                a = res["gpu_split"][key].reshape(-1).astype(np.float64)
                b = res["gpu_unsplit"][key].reshape(-1).astype(np.float64)
                # the split / unsplit disagreement as a fraction of the split march's own worst error
                r = float(np.abs(a - b).max() / max(np.abs(a - ref).max(), 1e-30))
                line[f"split_vs_unsplit.{key}"] = r
                summary.setdefault("split_vs_unsplit", []).append(r)
            for name, gr in res.items():
                for key in ("centers", "colors", "radius"):
                    _, rl2, tiers = grad_errors(gr[key], g64[key])
                    line[f"{name}.{key}"] = {"relL2": rl2, "elem1e-2": tiers[0][1], "elem1e-3": tiers[1][1]}
                    for q, v in (("relL2", rl2), ("elem1e-2", tiers[0][1]), ("elem1e-3", tiers[1][1])):
                        summary.setdefault(f"{name}.{q}", []).append(v)
            print(json.dumps(line), flush=True)
    print(json.dumps({"summary": {k: {"max": float(np.max(v)), "median": float(np.median(v)), "n": len(v)}
                                  for k, v in sorted(summary.items())}}), flush=True)


if __name__ == "__main__":
    main()
