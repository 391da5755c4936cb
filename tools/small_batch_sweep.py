#!/usr/bin/env python3
"""Time of the training driver's call -- rm_train_step in ray-array mode (train.rs:169-190 with
the dataset.rs batch) -- over batch size x march steps at the driver's sphere count, to tell
per-step latency from work. The call goes straight through the C ABI on
preallocated device buffers (no per-call tensor allocation, loss overwritten, accumulate = 0), so
the loop measures the library's call, not the Python wrapper. torch events around 50 calls each,
after 10 warm-up calls; rays from the eye at (0, 0, -2.5) through a 50-degree cone, uniform
targets. Both kernels: the small-scene kernel (default for M <= 32 in ray-array mode) and the
general kernel (RM_SMALL=0).

    python tools/small_batch_sweep.py [--spheres 9] > gpurun_out/small_batch.json
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spheres", type=int, default=9)
    ap.add_argument("--k", type=float, default=20.0)
    ap.add_argument("--kernels", default="small,general")
    args = ap.parse_args()
    import torch
    from burn_raymarching_amd import model, native, render
    sc = model.scene_tensors(model.synthetic_scene(args.spheres, 5, radius_range=(0.1, 0.3)))
    ctx = render.context()
    m = args.spheres
    keys = ("centers", "colors", "radius", "light_dir", "ambient")
    g = {k: torch.empty(s, device="cuda") for k, s in zip(keys, ((m, 3), (m, 3), (m,), (3,), (1,)))}
    cg = native.RmGrads(*(g[k].data_ptr() for k in keys))
    loss = torch.zeros(1, device="cuda")
    rows = []
    for kern in args.kernels.split(","):
        os.environ["RM_SMALL"] = "1" if kern == "small" else "0"
        for n in (4096, 16384, 65536, 262144):
            rng = np.random.default_rng(n)
            o = np.tile(np.array([[0.0, 0.0, -2.5]], np.float32), (n, 1))
            d = rng.normal(size=(n, 3)).astype(np.float32) * np.float32(0.2) + np.array([0, 0, 1], np.float32)
            d /= np.linalg.norm(d, axis=1, keepdims=True)
            t = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()  # noqa: E731
            o_, d_, tg = t(o), t(d), t(rng.uniform(size=(n, 3)))
            ptrs = [ctypes.c_void_p(x.data_ptr()) for x in (o_, d_, tg)]
            for steps in (10, 20, 40):
                march = sc.march_for(native.march_params(steps, args.k))
                scs = sc.c_struct()

                def call():
                    ctx.check(ctx._lib.rm_train_step(ctx.handle, ptrs[0], ptrs[1], ptrs[2], n, 0.5, 1.0 / (3 * n),
                                                     ctypes.byref(scs), ctypes.byref(march), ctypes.byref(cg),
                                                     ctypes.c_void_p(loss.data_ptr()), None, 0), "rm_train_step")

                for _ in range(10):
                    call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    call()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 50 * 1e3
                rows.append({"kernel": kern, "rays": n, "march_steps": steps, "us_per_call": round(us, 2),
                             "Mrays_s": round(n / us, 1)})
                print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    # camera mode (rm_train_step_camera): BASELINE configs[0] (64x64, 1 view, 16 steps) and the
    # preview / driver image size (256x256, 40 steps), one view, both kernels
    cams = model.ring_cameras(10)[:1]
    mc = native.cameras(cams)
    for kern in args.kernels.split(","):
        os.environ["RM_SMALL"] = "1" if kern == "small" else "0"
        for size, steps in ((64, 16), (256, 40)):
            n = size * size
            tg = torch.rand((n, 3), device="cuda", generator=torch.Generator("cuda").manual_seed(size))
            march = sc.march_for(native.march_params(steps, args.k))
            scs = sc.c_struct()

            def call():
                ctx.check(ctx._lib.rm_train_step_camera(ctx.handle, mc, 1, size, size, ctypes.c_void_p(tg.data_ptr()),
                                                        0.5, 1.0 / (3 * n), ctypes.byref(scs), ctypes.byref(march),
                                                        ctypes.byref(cg), ctypes.c_void_p(loss.data_ptr()), None, 0),
                          "rm_train_step_camera")

            for _ in range(10):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 50 * 1e3
            rows.append({"kernel": kern, "camera": f"{size}x{size}", "rays": n, "march_steps": steps,
                         "us_per_call": round(us, 2), "Mrays_s": round(n / us, 1)})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"spheres": args.spheres, "k": args.k, "rows": rows}))


if __name__ == "__main__":
    main()
