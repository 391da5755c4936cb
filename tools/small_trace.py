#!/usr/bin/env python3
"""Phase timeline of the small-scene kernel (measurement build, -DRM_BLOCK_TRACE): one fused
training iteration (rm_train_iteration: the reference loop's step, train.rs:169-198) of a random
batch drawn from a few 64x64 views, then per wave the s_memrealtime stamps (100 MHz) of its phases
(rm_small.h): sphere data + ray, march, post-march forward, backward sweeps, record + arrival, and
for the last block the final reduction and the optimizer.

    bash tools/build_variant.sh WT trace -DRM_BLOCK_TRACE
    RM_LIB_PATH=burn_raymarching_amd/lib/var/trace.so python tools/small_trace.py [--spheres 9] [--rays 16384]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spheres", type=int, default=9)
    ap.add_argument("--rays", type=int, default=16384)
    ap.add_argument("--march-steps", type=int, default=40)
    ap.add_argument("--warm", type=int, default=5)
    args = ap.parse_args()
    import torch
    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr

    M, n, S = args.spheres, args.rays, args.march_steps
    cams = rmm.ring_cameras(4)
    sc = rmm.synthetic_scene(M, seed=3, radius_range=(0.08, 0.3))
    o, d = [], []
    for c in cams:  # camera.rs rays of four 64x64 views, the dataset's pixel arrays
        ro, rd = rmr.create_camera_rays(64, 64, *c)
        o.append(ro.reshape(-1, 3))
        d.append(rd.reshape(-1, 3))
    o = torch.cat(o).contiguous()
    d = torch.cat(d).contiguous()
    tg = rmr.render_diff_forward(o, d, rmm.scene_tensors(rmm.synthetic_scene(5, seed=7, radius_range=(0.08, 0.3))),
                                 32.0, S).contiguous()
    fg = torch.nonzero(tg.sum(1) > 0.01).flatten().to(torch.int32).contiguous()
    sm = rmm.SceneModel.from_activated(sc["centers"], sc["colors"], sc["radius"], sc["light_dir"], sc["ambient"])
    raw = sm.raw.clone()
    act = sm.activated_packed().clone()
    npk = rmm.packed_size(M)
    grad = torch.zeros(npk, device="cuda")
    m1, m2 = torch.zeros(npk, device="cuda"), torch.zeros(npk, device="cuda")
    loss = torch.zeros(2, device="cuda")
    ctx = rmr.context()
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    nu = int(0.8 * n)
    for it in range(1, args.warm + 2):
        march = native.march_params(S, 20.0)
        ctx.check(ctx._lib.rm_train_iteration(ctx.handle, p(o), p(d), p(tg), o.shape[0], p(fg), fg.numel(), nu,
                                              n - nu, 1, 1, it, 0.5, 1.0 / (3 * n), ctypes.byref(march), p(act),
                                              p(grad), p(raw), p(m1), p(m2), M, it, 0.01, 1e-5, 1, p(loss), None),
                  "rm_train_iteration")
    torch.cuda.synchronize()
    fn = native.lib().rm_debug_block_trace
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    cap = 4096
    buf = np.zeros((cap, 12), np.uint64)
    cnt = ctypes.c_int64()
    ctx.check(fn(ctx.handle, buf.ctypes.data, cap, ctypes.byref(cnt)), "rm_debug_block_trace")
    tr = buf[:cnt.value].astype(np.int64)
    tr = tr[tr[:, 0] != 0]
    base = tr[:, 0].min()
    us = lambda c: (tr[:, c] - base) / 100.0  # noqa: E731
    # the fused launch's extra block (the optimizer's gradient-independent part) has no ray phases
    extra = tr[:, 4] == 0
    last_arrival = float(us(8).max())
    span = float(us(1).max())
    pre = {"optimizer_part_us": float((us(8)[extra] - us(0)[extra]).max()),
           "optimizer_part_arrival_us": float(us(8)[extra].max())} if extra.any() else {}
    tr_all, tr = tr, tr[~extra]
    t0, t4, t5, t6, t7, t8 = us(0), us(4), us(5), us(6), us(7), us(8)
    res = {"waves": int(len(tr)), "span_us": span, **pre,
           "start_spread_us": float(t0.max()),
           "phase_us_mean": {"setup": float((t4 - t0).mean()), "march": float((t5 - t4).mean()),
                             "post_march": float((t6 - t5).mean()), "backward": float((t7 - t6).mean()),
                             "record_arrival": float((t8 - t7).mean())},
           "phase_us_max": {"setup": float((t4 - t0).max()), "march": float((t5 - t4).max()),
                            "post_march": float((t6 - t5).max()), "backward": float((t7 - t6).max()),
                            "record_arrival": float((t8 - t7).max())},
           "last_arrival_us": last_arrival}
    tr = tr_all
    last = tr[:, 9] != 0
    if last.any():
        t9, t10 = us(9)[last], us(10)[last]
        res["final_reduction_us"] = float((t9 - us(8)[last]).max())
        res["final_acquire_us"] = float((us(11)[last] - us(8)[last]).max())
        res["final_record_sums_us"] = float((us(2)[last] - us(11)[last]).max())
        res["final_scatter_us"] = float((t9 - us(2)[last]).max())
        res["optimizer_us"] = float((t10 - t9).max()) if (tr[last, 10] != 0).any() else None
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
