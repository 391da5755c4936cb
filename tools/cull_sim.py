"""Study (numpy, float64; not product code): how many (wave, march step, 16-sphere row block)
triples of the bench workload contribute nothing to the soft-min sum -- every term of the row
block below 2^-THR of the ray's largest term, for all 64 rays of the wave -- with the spheres in
their given order and sorted along a Morton curve. A row block no ray of a wave needs could be
skipped by the march sweep (lse_mfma) of that wave; this sizes the opportunity.

    python tools/cull_sim.py [--tiles 256] [--thr 30]
"""
from __future__ import annotations

import argparse
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from burn_raymarching_amd import model as rmm  # noqa: E402


def morton_order(c):
    q = np.clip(((c - c.min(0)) / (np.ptp(c, 0) + 1e-9) * 1023).astype(np.int64), 0, 1023)
    code = np.zeros(len(c), np.int64)
    for b in range(10):
        for ax in range(3):
            code |= ((q[:, ax] >> b) & 1) << (3 * b + ax)
    return np.argsort(code, kind="stable")


def camera_rays(W, H, eye, target, fov):
    eye, target = np.asarray(eye, float), np.asarray(target, float)
    fwd = target - eye
    fwd /= np.linalg.norm(fwd)
    right = np.cross(fwd, [0.0, 1.0, 0.0])
    right /= np.linalg.norm(right)
    up = np.cross(right, fwd)
    th = math.tan(math.radians(fov) / 2)
    ys, xs = np.mgrid[0:H, 0:W]
    u = ((xs + 0.5) / W * 2 - 1) * th * W / H
    v = (1 - (ys + 0.5) / H * 2) * th
    d = fwd + u[..., None] * right + v[..., None] * up
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    return eye, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=256)
    ap.add_argument("--thr", type=float, default=30.0)
    ap.add_argument("--spheres", type=int, default=256)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--k", type=float, default=32.0)
    ap.add_argument("--radius-range", type=float, nargs=2, default=(0.03, 0.12))
    ap.add_argument("--scene-json", default="", help="a scene.json (e.g. the grown configs[4] model) instead "
                                                     "of the synthetic ball; --spheres from the file")
    ap.add_argument("--cameras", default="", help="cameras.json poses instead of the ring")
    args = ap.parse_args()
    if args.scene_json:
        from bench import load_scene_json
        sc = load_scene_json(args.scene_json)
        args.spheres = int(sc["centers"].shape[0])
    else:
        sc = rmm.synthetic_scene(args.spheres, seed=0, radius_range=tuple(args.radius_range))
    c, r = np.asarray(sc["centers"], float), np.asarray(sc["radius"], float)
    orders = {"given": np.arange(len(c)), "morton": morton_order(c)}
    W = H = 512
    rng = np.random.default_rng(0)
    if args.cameras:
        import json
        cams = [(q["origin"], q["target"], q["fov"]) for q in json.load(open(args.cameras))]
    else:
        cams = rmm.ring_cameras(10)
    kl2 = args.k / math.log(2.0)  # base-2 exponent scale
    res = {name: [0, 0] for name in orders}
    # the conservative test a kernel can run: per row block a bounding sphere (c_b, R_b), per ray
    # an upper bound D_up = 2 D_prev + ln(M)/k of the hard min (no bound at the first step)
    bounds = {}
    for name, o in orders.items():
        cb = c[o].reshape(-1, 16, 3)
        ctr = 0.5 * (cb.max(1) + cb.min(1))
        rb = (np.linalg.norm(cb - ctr[:, None], axis=-1) + r[o].reshape(-1, 16)).max(1)
        bounds[name] = (ctr, rb)
    test = {name: [0, 0, 0] for name in orders}  # wave-level, 16-ray-group level, count
    slack = math.log(args.spheres) / args.k
    alive_steps = 0
    for ti in range(args.tiles):
        eye, tgt, fov = cams[ti % len(cams)]
        eye, d = camera_rays(W, H, eye, tgt, fov)
        ty, tx = rng.integers(0, H // 8), rng.integers(0, W // 8)
        dw = d[8 * ty:8 * ty + 8, 8 * tx:8 * tx + 8].reshape(64, 3)
        t = np.zeros(64)
        Dprev = None
        for st in range(args.steps):
            p = eye + t[:, None] * dw
            dist = np.linalg.norm(p[:, None, :] - c[None], axis=-1) - r[None]  # [64, M]
            e = -kl2 * dist
            emax = e.max(1, keepdims=True)
            D = -(emax[:, 0] + np.log2(np.exp2(e - emax).sum(1))) / kl2
            if np.all(D > 3.0):  # the wave left the scene (early exit)
                break
            alive_steps += 1
            rel = e - emax  # log2 of each term relative to the ray's largest
            for name, o in orders.items():
                blk = rel[:, o].reshape(64, -1, 16).max(2)  # [64, blocks]
                skip = np.all(blk < -args.thr, axis=0)
                res[name][0] += int(skip.sum())
                res[name][1] += skip.size
            if Dprev is not None:
                dup = 2 * np.maximum(Dprev, 0) + slack
                for name, (ctr, rb) in bounds.items():
                    dist = np.linalg.norm(p[:, None, :] - ctr[None], axis=-1)  # [64, blocks]
                    ok = dist - rb[None] - dup[:, None] > args.thr / kl2
                    test[name][0] += int(np.all(ok, axis=0).sum())
                    test[name][1] += int(np.all(ok.reshape(4, 16, -1), axis=1).sum()) / 4
                    test[name][2] += ok.shape[1]
            Dprev = D
            t = t + D
    print(f"tiles {args.tiles}, wave-steps alive {alive_steps}, threshold 2^-{args.thr:g}")
    for name, (s, n) in res.items():
        print(f"  {name:7s} row blocks skippable: {s / max(n, 1):.3f}; by the bound test: per wave "
              f"{test[name][0] / max(test[name][2], 1):.3f}, per 16-ray group {test[name][1] / max(test[name][2], 1):.3f}")


if __name__ == "__main__":
    main()
