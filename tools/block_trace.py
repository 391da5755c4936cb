#!/usr/bin/env python3
"""Per-wave timeline of one train-kernel launch (measurement build, -DRM_BLOCK_TRACE).

Runs the bench workload's training loop (same scene, cameras, targets and optimizer as bench.py)
for --warm steps, then records one more step's rm_ray_kernel<train> launch: every wave's start and
end (s_memrealtime, 100 MHz), hardware slot (XCC, SE, SH, CU, SIMD) and logical block / launch
position. Prints how busy the SIMDs are over the launch (live waves per SIMD over time, SIMDs with
at least one live wave), the tail, and how the dispatcher placed consecutive launch positions.

A split launch with a continuation (S >= 64) runs the train kernel twice per step; the records
then hold the second launch (every block writes one; the ones with nothing to continue end at
once), unless RM_SPLIT_CONT_STEPS=0.

    bash tools/build_variant.sh HEAD trace -DRM_BLOCK_TRACE
    RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so python tools/block_trace.py --spheres 4096 \
        --march-steps 128 --views 1 --out gpurun_out/trace_c5.npz
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    import torch
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr

    import json
    import numpy as np
    sys.path.insert(0, ROOT)
    from bench import DANGO, load_scene_json
    if args.scene_json:
        sc0 = load_scene_json(args.scene_json)
        args.spheres = sc0["centers"].shape[0]
    W, H, M, S, K, V = args.width, args.height, args.spheres, args.march_steps, args.smooth_k, args.views
    rr = (0.03, 0.12) if M <= 256 else ((0.02, 0.06) if M <= 1024 else (0.01, 0.04))
    if not args.scene_json:
        sc0 = rmm.synthetic_scene(M, seed=0, radius_range=rr)
    sc1 = rmm.synthetic_scene(M, seed=1, radius_range=rr)
    if args.cameras:  # the generate.rs scene through the renderer.rs kernel, as bench.py --targets dango
        cams = [(c["origin"], c["target"], c["fov"]) for c in json.load(open(args.cameras))][:V]
        t = [torch.tensor(DANGO[k], device="cuda") for k in ("centers", "colors", "radius")]
        tg = rmr.render_camera(cams, W, H, *t).view(-1, 3)
    else:
        cams = rmm.ring_cameras(max(10, V))[:V]
        tg = rmr.render_diff_camera(cams, W, H, rmm.scene_tensors(sc1), K, S).view(-1, 3)
    mdl = rmm.SceneModel.from_activated(sc0["centers"], np.clip(sc0["colors"], 1e-6, 1 - 1e-6), sc0["radius"],
                                        sc0["light_dir"], sc0["ambient"],
                                        color_dtype="f16" if args.color_f16 else "f32")
    opt = rmm.Adam(mdl, weight_decay=1e-5, with_penalties=True)
    march = native.march_params(S, K)
    g = torch.zeros(rmm.packed_size(M), device="cuda")
    loss = torch.zeros(1, device="cuda")
    for i in range(args.warm + 1):
        rmr.train_step_camera(cams, W, H, tg, mdl.scene(), K, progress=0.5, steps=S, grads_packed=g, loss=loss,
                              march=march)
        if i < args.warm:
            opt.step(g, 0.05)
    ctx = rmr.context()
    lib = native.lib()
    fn = lib.rm_debug_block_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    cap = 16384 * 4
    buf = np.zeros((cap, 12), np.uint64)
    n = ctypes.c_int64()
    ctx.check(fn(ctx.handle, buf.ctypes.data, cap, ctypes.byref(n)), "rm_debug_block_trace")
    tr = buf[:n.value]
    return tr[tr[:, 0] != 0]  # split blocks of two waves leave the records of waves 2-3 empty


def analyse(tr, bins=40, steps=0):
    t0, t1 = tr[:, 0].astype(np.int64), tr[:, 1].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / 100.0, (t1 - base) / 100.0  # microseconds (100 MHz)
    hw = tr[:, 2]
    xcc = (hw >> np.uint64(32)).astype(np.int64) & 0xF
    lo = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
    simd = (lo >> 4) & 3
    cu = (lo >> 8) & 0xF
    sh = (lo >> 12) & 1
    se = (lo >> 13) & 7
    blk = (tr[:, 3] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    pos = (tr[:, 3] >> np.uint64(32)).astype(np.int64)
    span = e.max()
    dur = e - s
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    simd_key = cu_key * 4 + simd
    ncu, nsimd = len(np.unique(cu_key)), len(np.unique(simd_key))
    print(f"waves {len(tr)}, launch span {span:.1f} us, CUs seen {ncu}, SIMDs seen {nsimd}")
    q = np.percentile(dur, [0, 25, 50, 75, 90, 99, 100])
    print("wave duration us  min/25/50/75/90/99/max: " + " ".join(f"{v:.1f}" for v in q))
    print(f"sum of wave durations / (SIMDs x span) = mean live waves per SIMD: {dur.sum() / (nsimd * span):.2f}")
    edges = np.linspace(0, span, bins + 1)
    print(" time(us)  live/SIMD  SIMDs>=1  waves started")
    for i in range(bins):
        a, b = edges[i], edges[i + 1]
        ov = np.clip(np.minimum(e, b) - np.maximum(s, a), 0, None)
        live = ov.sum() / (b - a) / nsimd
        busy = len(np.unique(simd_key[ov > 0])) / nsimd
        st = int(((s >= a) & (s < b)).sum())
        print(f" {a:8.1f}  {live:9.2f}  {busy:8.2f}  {st:6d}")
    # dispatcher placement of the first launch positions (first wave of each block)
    first = np.argsort(pos * 4 + (np.arange(len(pos)) % 4), kind="stable")
    bpos = pos[first][::4][:48]
    bcu = cu_key[first][::4][:48]
    print("launch position -> (xcc, se, sh, cu) for the first 48 blocks:")
    print(" ".join(f"{p}:{c // 256}.{(c // 32) % 8}.{(c // 16) % 2}.{c % 16}" for p, c in zip(bpos, bcu)))
    # per-CU finish time spread
    cu_end = {}
    for k, v in zip(cu_key, e):
        cu_end[k] = max(cu_end.get(k, 0.0), v)
    ce = np.array(sorted(cu_end.values()))
    print("CU last-wave end us  min/10/50/90/max: " + " ".join(f"{np.percentile(ce, p):.1f}" for p in (0, 10, 50, 90, 100)))
    if tr.shape[1] >= 8 and steps:
        tm = (tr[:, 4].astype(np.int64) - base) / 100.0
        tp = (tr[:, 5].astype(np.int64) - base) / 100.0
        run_steps = steps - tr[:, 6].astype(np.int64)
        live = tp > tm  # waves that ran the post-march forward (and the backward)
        print(f"live waves {int(live.sum())} of {len(tr)}; march steps run: mean {run_steps.mean():.1f}, "
              f"live mean {run_steps[live].mean() if live.any() else 0:.1f}")
        # where the waves' time goes, summed over all waves (wall time of each wave, so a phase's
        # share includes its SIMD sharing: a proxy for its share of the launch's issue)
        # (stamps outside the wave's own [start, end] are stale: a wave that ended before writing
        # them, e.g. an empty block of a continuation launch, counts as march time only)
        ok = live & (tm >= s) & (tp >= tm) & (e >= tp)
        m_all = np.where(ok, tm - s, e - s)
        p_all = np.where(ok, tp - tm, 0.0)
        b_all = np.where(ok, e - tp, 0.0)
        tot = m_all.sum() + p_all.sum() + b_all.sum()
        print(f"summed wave time: march {m_all.sum() / tot:.3f}, post-march forward {p_all.sum() / tot:.3f}, "
              f"backward {b_all.sum() / tot:.3f} (of {tot / 1e3:.1f} wave-ms)")
        if tr.shape[1] >= 12:  # march steps per path over every wave (which share takes the clamped sweep)
            pw = tr[:, 7].astype(np.uint64)
            tot_paths = [int(((pw >> np.uint64(16 * k)) & np.uint64(0xFFFF)).sum()) for k in range(4)]
            tot_paths.append(int(tr[:, 9].astype(np.int64).sum()))
            n = max(sum(tot_paths), 1)
            print("march steps by path (none fast, none clamped, fixed fast, fixed clamped, vector): "
                  + " ".join(f"{v} ({v / n:.3f})" for v in tot_paths))
        order = np.argsort(-dur)[:12]
        print(" slowest waves: total  march  post  bwd (us)  steps  us/step  SIMD-sharing"
              + ("  paths(none f/c, fixed f/c, vector)  lse-cycles/step  march-cycles/step" if tr.shape[1] >= 12 else ""))
        for i in order:
            m_us, p_us, b_us = tm[i] - s[i], tp[i] - tm[i], e[i] - tp[i]
            share = ((s < e[i]) & (e > s[i]) & (simd_key == simd_key[i])).sum()
            extra = ""
            if tr.shape[1] >= 12:
                pw = int(tr[i, 7])
                paths = [(pw >> (16 * k)) & 0xFFFF for k in range(4)] + [int(tr[i, 9])]
                extra = (f"  {paths}  {int(tr[i, 8]) / max(run_steps[i], 1):10.0f}"
                         f"  {int(tr[i, 10]) / max(run_steps[i], 1):10.0f}")
            print(f"  {dur[i]:9.1f} {m_us:8.1f} {p_us:6.1f} {b_us:6.1f}  {run_steps[i]:5d}  "
                  f"{m_us / max(run_steps[i], 1):7.2f}  {share}{extra}")
    return {"span_us": float(span), "mean_live_per_simd": float(dur.sum() / (nsimd * span))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--spheres", type=int, default=256)
    ap.add_argument("--march-steps", type=int, default=32)
    ap.add_argument("--smooth-k", type=float, default=32.0)
    ap.add_argument("--views", type=int, default=10)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--bins", type=int, default=40)
    ap.add_argument("--out", default="")
    ap.add_argument("--load", default="", help="analyse a saved .npz instead of running")
    ap.add_argument("--scene-json", default="", help="start scene (bench.py --scene-json; --spheres from the file)")
    ap.add_argument("--cameras", default="", help="cameras.json poses instead of the ring (bench.py --cameras)")
    ap.add_argument("--color-f16", action="store_true")
    args = ap.parse_args()
    tr = np.load(args.load)["trace"] if args.load else run(args)
    if args.out:
        np.savez_compressed(args.out, trace=tr)
    analyse(tr, args.bins, args.march_steps)


if __name__ == "__main__":
    main()
