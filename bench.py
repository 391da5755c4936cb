#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: Mrays/s of the differentiable render's forward+backward
train step at 512x512 / 256 spheres / 32 march steps, on 1..8 MI355X (one process per GPU).

One timed step = one full training step of the reference loop (train.rs:169-198) on the
HIP path, per rank:
  rm_scene_activate          (scene.rs:41-45)
  rm_train_step_camera       (10 512x512 views: in-kernel rays, fused forward + compute_loss
                              seed + analytic backward, fixed-order gradient reduction)
  all_reduce(grads) [N > 1]  (RCCL over xGMI; 7M+4 floats)
  rm_optimizer_step          (activation chain rule + training.rs penalties + Burn Adam)
Views shard across ranks (weak scaling: every rank renders its own 10 views of 512x512 per step).
value = rays of all ranks / max-over-ranks wall time of the K timed steps.

--skip-escaped on (off by default, like the library): ray blocks whose rays provably leave the
scene with a silhouette mask of exactly 0 get out = 0 and zero gradients without marching --
bit-identical results (tests/test_gpu_escape.py); `escape_skip` reports the skipped share.

Synthetic data (no datasets offline): scene seed 0 (BASELINE.md "Synthetic inputs"), targets
= the seed-1 scene rendered by the forward kernel from a ring of cameras at radius 2.5, y 0.5.

Extra objects on the JSON line:
  roofline      -- the dominant kernel (rm_ray_kernel<train>) timed with hipEvents on its own
                   stream inside the timed region (on every 5th step, --timing-every: the
                   events cost ~0.6 % of a timed step); algorithmic FLOP = 16*(S+10)*M per ray
                    counted only for sphere sweeps that actually ran (waves
                   whose rays all escaped stop early, see early_exit, and the normal is one
                   sweep instead of six; achieved_all_rays counts the full 16*(S+10)*M for
                   every ray); bound "valu" (fp32 vector);
                   traffic = HBM bytes per launch from the committed rocprofv3 PMC summary
                   (profiles/r01_pmc_traffic.json) when present, else null.
  cpu_baseline  -- the oracle's fp32 reference-order C restatement (OpenMP) on a bounded
                   strided sample of the same view, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "Mrays/s fwd+bwd, 512x512 / 256 spheres / 32 steps, at 1/2/4/8 MI355X"
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md chip table (vector fp32, spec)
PEAK_HBM_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FLOP_PER_EVAL = 16         # SURVEY.md §8d canonical count (sqrt and exp counted as 1)


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--spheres", type=int, default=256)
    ap.add_argument("--march-steps", type=int, default=32)
    ap.add_argument("--smooth-k", type=float, default=32.0)
    ap.add_argument("--views-per-gpu", type=int, default=10,
                    help="512x512 views per GPU per step: 10 = the whole 10-camera ring of BASELINE configs[1-2] "
                         "= 2,621,440 rays = 10240 ray blocks in one launch (the once-per-launch ramp-down and "
                         "the per-step O(M) kernels are amortised); at 8 GPUs a step covers 80 views")
    ap.add_argument("--ring", type=int, default=10, help="cameras on the target ring")
    ap.add_argument("--radius-range", type=float, nargs=2, default=None,
                    help="activated radii U[lo, hi] of the synthetic scenes (default per SURVEY.md 8d: "
                         "0.03-0.12 up to 256 spheres, 0.02-0.06 up to 1024, 0.01-0.04 beyond)")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--kernel-timing", choices=["on", "off"], default="on",
                    help="hipEvents on the train kernel's dispatch packets (off: no roofline; A/B of their cost)")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="time the train kernel on every n-th timed step (the events cost ~0.6 %% per timed step)")
    ap.add_argument("--cpu-sample", type=int, default=262144, help="rays of the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: repeat the sample this long")
    ap.add_argument("--skip-escaped", choices=["on", "off"], default="off",
                    help="RM_MARCH_SKIP_ESCAPED: skip ray blocks that provably leave the scene (exact)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if rank == 0:
            print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    import torch
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import render as rmr
    from burn_raymarching_amd import native
    from burn_raymarching_amd.parallel import Shard, ViewShardedStep

    W, H, M, S, K = args.width, args.height, args.spheres, args.march_steps, args.smooth_k
    vpg = args.views_per_gpu
    if not 1 <= vpg <= native.RM_MAX_VIEWS_PER_CALL:
        raise SystemExit("--views-per-gpu must be in 1..16")
    npix = W * H
    rays_per_rank = vpg * npix
    rays_global = rays_per_rank * world

    # ---- synthetic scene, targets, optimizer --------------------------------------------
    rr = tuple(args.radius_range) if args.radius_range else (
        (0.03, 0.12) if M <= 256 else ((0.02, 0.06) if M <= 1024 else (0.01, 0.04)))
    sc0 = rmm.synthetic_scene(M, seed=0, radius_range=rr)
    sc1 = rmm.synthetic_scene(M, seed=1, radius_range=rr)
    ring = max(args.ring, world * vpg)
    cams = rmm.ring_cameras(ring)
    tgt_scene = rmm.scene_tensors(sc1)
    targets = torch.empty((ring, npix, 3), device="cuda")
    for v0 in range(0, ring, native.RM_MAX_VIEWS_PER_CALL):
        chunk = cams[v0:v0 + native.RM_MAX_VIEWS_PER_CALL]
        targets[v0:v0 + len(chunk)] = rmr.render_diff_camera(chunk, W, H, tgt_scene, K, S).view(len(chunk), npix, 3)
    model = rmm.SceneModel.from_activated(sc0["centers"], sc0["colors"], sc0["radius"], sc0["light_dir"],
                                          sc0["ambient"])
    opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
    march = native.march_params(S, K, skip_escaped=args.skip_escaped == "on")
    ctx = rmr.context()
    total_steps = args.warmup + args.steps
    progress = {"i": 0}

    # the ring twice over: a rank's views are consecutive mod ring, so its targets are always one
    # contiguous slice (no gather kernel, no host-built index tensor inside the timed loop)
    targets2 = torch.cat([targets, targets])

    def step_fn(views, inv_count, grads_out, loss_out):
        # rm_train_step_camera over this rank's views (fused forward + loss seed + backward)
        first = views[0]
        assert views == [(first + j) % ring for j in range(len(views))]
        tg = targets2[first:first + len(views)]
        rmr.train_step_camera([cams[j] for j in views], W, H, tg.view(-1, 3), model.scene(), K,
                              progress=progress["i"] / total_steps, steps=S, inv_count=inv_count,
                              grads_packed=grads_out, loss=loss_out, march=march)

    dp = ViewShardedStep(Shard(rank, world, vpg, ring), npix, rmm.packed_size(M), "cuda", step_fn,
                         optim_fn=lambda g: opt.step(g, args.lr))
    loss = dp.loss

    def step(i):
        progress["i"] = i
        dp(i)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    ctx.collect_timing(reset=True)
    ctx.stats(True)
    ctx.collect_stats(reset=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # every n-th step when there are enough to sample (short runs: every step)
    every = max(args.timing_every, 1) if args.steps >= 4 * max(args.timing_every, 1) else 1
    timed_steps = 0
    for i in range(args.warmup, total_steps):
        timed = args.kernel_timing == "on" and (i - args.warmup) % every == 0
        ctx.timing(timed)
        timed_steps += timed
        step(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.timing(False)
    kern_ms, launches = ctx.collect_timing(reset=True)
    st = ctx.collect_stats(reset=True)
    ctx.stats(False)
    blocks_run, blocks_skipped = st["blocks"], st["blocks_skipped"]
    skipped_frac = blocks_skipped / max(blocks_run, 1)
    # march steps not run: whole skipped blocks plus waves that left the march early
    waves_total = max(st["waves"], 1)
    march_saved_frac = (blocks_skipped * 4 * S + st["steps_saved"]) / (waves_total * S)
    if dist is not None:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        kt = torch.tensor([kern_ms], device="cuda", dtype=torch.float64)
        dist.all_reduce(kt, op=dist.ReduceOp.MAX)
        kern_ms = float(kt.item())
    kern_avg_ms = kern_ms / max(launches, 1)  # per launch (one per step unless the step splits)
    kern_step_ms = kern_ms / max(timed_steps, 1)  # per step: the roofline's time base

    value = rays_global * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    finite = bool(torch.isfinite(model.raw).all().item()) and bool(torch.isfinite(loss).all().item())

    # ---- roofline of the dominant kernel -------------------------------------------------
    # algorithmic work actually executed: skipped blocks run no sphere evaluation at all, and a
    # wave that left the march early skips its remaining march steps and the 10 post-march /
    # backward sweeps (its outputs and gradient terms are exactly 0)
    flop_per_ray = FLOP_PER_EVAL * (S + 10) * M
    # sweeps a wave runs: S march + reconnect + normal + shade + 2 backward = S + 5 (the kernel
    # takes the normal's six central-difference sweeps as one gradient sweep)
    sweeps_total = waves_total * (S + 10)
    waves_post = max(waves_total - blocks_skipped * 4 - st["waves_exited"], 0)
    sweeps_run = (waves_total - blocks_skipped * 4) * S - st["steps_saved"] + waves_post * 5
    executed_frac = max(0.0, sweeps_run / sweeps_total)
    flops_launch = flop_per_ray * rays_per_rank * executed_frac
    kern_step_ms = kern_step_ms or float("nan")  # no timed launches (--kernel-timing off)
    achieved_tf = flops_launch / (kern_step_ms * 1e-3) / 1e12
    mpad = (M + 31) // 32 * 32
    blocks = (rays_per_rank + 255) // 256
    alg_bytes = rays_per_rank * 12 + blocks * (mpad * 12 + 8) * 4  # target read + partial-gradient slabs
    traffic = None
    traffic_src = None
    pmc_path = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")  # committed rocprofv3 PMC summary
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            key = f"{W}x{H}_M{M}_S{S}_V{vpg}"
            if key in pmc.get("train_kernel_bytes_per_launch", {}):
                traffic = float(pmc["train_kernel_bytes_per_launch"][key])
                traffic_src = os.path.relpath(pmc_path, ROOT)
        except Exception:
            traffic = None
    roofline = None if launches == 0 else {
        "bound": "valu",
        "kernel": "rm_ray_kernel<train,camera>",
        "achieved": round(achieved_tf, 3),
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 4),
        "traffic": traffic,
        "traffic_source": traffic_src,
        "kernel_ms": round(kern_avg_ms, 4),
        "kernel_ms_per_step": round(kern_step_ms, 4),
        "launches_timed": launches,
        "flop_per_ray": flop_per_ray,
        "rays_per_launch": rays_per_rank,
        "executed_frac": round(executed_frac, 4),
        "achieved_all_rays": round(flop_per_ray * rays_per_rank / (kern_step_ms * 1e-3) / 1e12, 3),
        "hbm": {"algorithmic_bytes_per_launch": alg_bytes,
                "achieved_GBs": round(alg_bytes / (kern_step_ms * 1e-3) / 1e9, 2),
                "peak_GBs": PEAK_HBM_GBS,
                "frac": round(alg_bytes / (kern_step_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 6)},
    }

    # ---- CPU baseline (rank 0, N = 1 only) -----------------------------------------------
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(args, sc0, sc1, cams[0], W, H, M, S, K)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded scene + targets rendered by the forward kernel)",
            "config": {"workload": f"train step fwd+bwd, {W}x{H} view(s) per GPU, {M} spheres, {S} march steps, "
                                   f"k={K:g}, camera mode, Adam",
                       "width": W, "height": H, "spheres": M, "march_steps": S, "smooth_k": K,
                       "views_per_gpu": vpg, "rays_per_step": rays_global, "radius_range": list(rr),
                       "parallelism": f"views-dp{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "escape_skip": {"enabled": args.skip_escaped == "on", "blocks": blocks_run,
                            "blocks_skipped": blocks_skipped, "skipped_frac": round(skipped_frac, 4)},
            "early_exit": {"enabled": os.environ.get("RM_NO_EARLY_EXIT") != "1", "waves": st["waves"],
                           "waves_exited": st["waves_exited"],
                           "exited_frac": round(st["waves_exited"] / waves_total, 4),
                           "march_steps_saved_frac": round(march_saved_frac, 4)},
            "finite": finite,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(args, sc0, sc1, cam, W, H, M, S, K):
    """Oracle fp32 reference-order restatement (OpenMP) on a strided sample of the view."""
    from oracle import oracle as orc
    o, d = orc.camera_rays(W, H, *cam, precision="f32")
    stride = max(1, (W * H) // max(args.cpu_sample, 1))
    idx = np.arange(0, W * H, stride)
    o, d = o[idx], d[idx]
    tg = orc.render_diff(o, d, sc1, S, K, precision="f32")
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    reps = 0
    t0 = time.perf_counter()
    while True:  # repeat the sample until ~10 s of CPU work (bounded: at most 30 repetitions)
        orc.train_step(o, d, tg, sc0, S, K, 0.5, precision="f32")
        reps += 1
        sec = time.perf_counter() - t0
        if sec >= args.cpu_seconds or reps >= 30:
            break
    return {"value": round(reps * len(idx) / sec / 1e6, 6), "unit": "Mrays/s", "cores": threads,
            "hardware_threads": os.cpu_count(), "kind": "port",
            "sample": f"{reps} x {len(idx)} rays (every {stride}th pixel of one {W}x{H} view), fwd+bwd train "
                      f"step, {M} spheres, {S} steps, fp32 reference op order, OpenMP; {sec:.2f} s"}


if __name__ == "__main__":
    main()
