#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: Mrays/s of the differentiable render's forward+backward
train step at 512x512 / 256 spheres / 32 march steps, on 1..8 MI355X (one process per GPU).

One timed step = one full training step of the reference loop (train.rs:169-198) on the
HIP path, per rank:
  rm_train_step_camera       (10 512x512 views: in-kernel rays, fused forward + compute_loss
                              seed + analytic backward, fixed-order gradient reduction)
  all_reduce(grads) [N > 1]  (RCCL over xGMI; 7M+5 floats: gradient + loss)
  rm_optimizer_step          (activation chain rule + training.rs penalties + Burn Adam, which
                              also writes the activated parameters of the next step)
With --fused-adam on (one GPU, one call per step) the two calls are one (rm_train_step_camera_adam:
for <= 64 spheres the optimizer runs in the gradient reduction's last block).
Views shard across ranks. Default: STRONG scaling -- a step covers --global-views 80 views of
512x512 (a ring of 80 cameras) in all, split into contiguous parts over the N ranks (80 on one
GPU, 10 per GPU on 8), so the total work per step is fixed as N grows; a rank issues its views in
calls of up to 16 (one launch each), every call slot on its own rm_context so that its
cost-ordered dispatch comes from the same views' previous step. `--views-per-gpu V` alone selects
weak scaling (V views per rank per step). value = rays of all ranks * K / max-over-ranks wall time
of the K timed steps (barrier + synchronize on both sides). `value_median` / `ms_per_step_median` use the median of the per-step
hipEvent times of every --timing-every-th timed step (max over ranks per step).

`--gpus N` without WORLD_SIZE in the environment launches N rank processes itself (one per
GPU, before anything touches a GPU) and exits with the first failing rank's status; under
torch.distributed.run the ranks come from the environment, and a WORLD_SIZE that differs from
--gpus is an error.

Synthetic data (no datasets offline): scene seed 0 (BASELINE.md "Synthetic inputs"), targets
= the seed-1 scene rendered by the forward kernel from a ring of cameras at radius 2.5, y 0.5.
Ring position j looks from angle (49 j mod 80) / 80 of the circle (--ring-order spread), so each
rank's contiguous slice samples the whole circle: per-slice train-call times at N = 8 differ by
0.5 % instead of 3.5 % with angle j (tools/shard_balance.py, profiles/r04b_shard_balance.json).

Extra objects on the JSON line:
  roofline      -- the dominant kernel (rm_ray_kernel<train>) timed with hipEvents from its own
                   dispatch packet inside the timed region (every 5th step, --timing-every);
                   algorithmic FLOP = 16*(S+10)*M per ray. `achieved`/`frac`
                   count the sweeps that ran (executed_frac, from the kernel's work counters in an
                   untimed replay of the timed steps from a snapshot of the training state:
                   waves whose rays all escaped stop early, the normal is one sweep instead of
                   six, and the two backward sweeps run only for rays with non-zero seeds);
                   `canonical` is the work of a second replay with the early exit off (every ray's
                   S+3 sweeps, the seeded rays' backward sweeps) over its kernel time; `pmc` quotes the committed rocprofv3 SQ summary
                   (profiles/r*_pmc_sq.json) for this workload; traffic = HBM bytes per launch from
                   the committed FETCH_SIZE / WRITE_SIZE summary (profiles/r*_pmc_traffic.json).
  cpu_baseline  -- the oracle's fp32 reference-order C restatement (OpenMP) on a bounded strided
                   sample of the same view, rank 0 at N=1 only: at the box's CPU share (value)
                   and on one core.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
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
BYTES_PER_RAY_CAMERA = 24  # SURVEY.md §8d algorithmic HBM bytes per ray, camera mode
DEFAULT_GLOBAL_VIEWS = 80  # strong scaling: 80 views per step = 10 per GPU at N = 8
MAX_RAYS_PER_CALL = 128 * 512 * 512  # one launch of 256-ray blocks (kMaxBlocksPerLaunch)


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
    ap.add_argument("--anneal-k", type=float, default=None, metavar="K0",
                    help="anneal the soft-min sharpness as train.rs:174 does (k = K0 + (K - K0) * progress), "
                         "over the timed steps: the warmup runs at K0, timed step j of K at "
                         "K0 + (K - K0) * j / (K - 1)")
    ap.add_argument("--global-views", type=int, default=None,
                    help="strong scaling (the default, %d views): views per step over ALL ranks, split into "
                         "contiguous parts over the ranks" % DEFAULT_GLOBAL_VIEWS)
    ap.add_argument("--views-per-gpu", type=int, default=None,
                    help="weak scaling: views per GPU per step (e.g. 10 = the 10-camera ring of BASELINE "
                         "configs[1-2] = 2,621,440 rays in one launch); exclusive with --global-views")
    ap.add_argument("--ring", type=int, default=10, help="cameras on the target ring (at least the views of a step)")
    ap.add_argument("--ring-order", choices=["contiguous", "spread"], default=None,
                    help="camera angle of ring position j: angle j (contiguous) or angle (j * s) mod ring with s the "
                         "coprime stride nearest 0.618 ring (spread: a rank's contiguous slice covers the circle); "
                         "default spread for strong scaling, contiguous for weak (whose per-step view rotation, and "
                         "so the training trajectory of the BASELINE configs, stays that of earlier rounds)")
    ap.add_argument("--views-per-call", type=int, default=0,
                    help="views per train call (0: as many as one launch takes, up to 128 = the strong default's "
                         "80 views in one call)")
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the calls of a step are spread over (>1: the calls run concurrently, each "
                         "into its own gradient row, summed in call order before the all-reduce)")
    ap.add_argument("--dump-grad", default=None,
                    help="rank 0 saves the all-reduced [gradient | loss] of step 0 here (.npy; rehearsal tests)")
    ap.add_argument("--radius-range", type=float, nargs=2, default=None,
                    help="activated radii U[lo, hi] of the synthetic scenes (default per SURVEY.md 8d: "
                         "0.03-0.12 up to 256 spheres, 0.02-0.06 up to 1024, 0.01-0.04 beyond)")
    ap.add_argument("--color-dtype", choices=["f32", "f16"], default="f32",
                    help="f16: fp16 colour / fp32 SDF (BASELINE configs[4], RM_MARCH_COLOR_F16)")
    ap.add_argument("--cameras", default=None,
                    help="cameras.json (the reference's data/cameras.json schema): its poses replace the synthetic "
                         "ring (BASELINE configs[1]: '10 views (data/cameras.json)')")
    ap.add_argument("--targets", choices=["synthetic", "dango", "files"], default="synthetic",
                    help="synthetic: the seed-1 scene rendered by the forward kernel; dango: the generate.rs scene "
                         "rendered by the renderer.rs kernel at WxH (what generate.rs writes at that size); files: "
                         "the PNGs cameras.json names (their size must be WxH)")
    ap.add_argument("--scene-json", default=None,
                    help="start from this scene.json (train.rs:238-262 layout, radius + 0.01 re-added as scene.rs:43) "
                         "instead of the synthetic seed-0 scene; --spheres is taken from the file (e.g. a model grown "
                         "by `rm_train train --split-all --max-spheres 4096`, BASELINE configs[4])")
    ap.add_argument("--fused-adam", choices=["on", "off"], default="off",
                    help="on (one GPU, one call per step): the train step and the optimizer as ONE call "
                         "(rm_train_step_camera_adam: for <= 64 spheres the optimizer runs in the gradient "
                         "reduction's last block; bit-identical to the two calls). Off by default: no measured "
                         "gain at C2 (profiles/r06_ab.txt)")
    ap.add_argument("--graph", choices=["on", "off"], default="off",
                    help="on (one GPU): capture one training step in a hipGraph (torch.cuda.CUDAGraph over the rm_* "
                         "calls, per-step scalars on the device: rm_bind_step_scalars) and replay it for the timed "
                         "steps; the train-kernel time then comes from the statistics replay (eager, timed)")
    ap.add_argument("--as-rank", default=None, metavar="R/N",
                    help="one GPU runs rank R's share of an N-rank strong-scaling step alone: its fixed views of "
                         "the global ones, the global ray count, no all-reduce (what that rank's GPU does per step "
                         "at N ranks, for tools/predict_scaling.py); value = this rank's rays per second")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--kernel-timing", choices=["on", "off"], default="on",
                    help="hipEvents on the train kernel's dispatch packets (off: no roofline; A/B of their cost)")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="time the train kernel on every n-th timed step (the events cost ~0.6 %% per timed step)")
    ap.add_argument("--aux-steps", type=int, default=1,
                    help="1: replay the timed steps untimed twice after the timed region (work statistics; early "
                         "exit off for the canonical kernel time); 0: no replays (PMC passes)")
    ap.add_argument("--cpu-sample", type=int, default=262144, help="rays of the CPU baseline sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: repeat the sample this long")
    ap.add_argument("--skip-escaped", choices=["on", "off"], default="off",
                    help="RM_MARCH_SKIP_ESCAPED: skip ray blocks that provably leave the scene (exact)")
    args = ap.parse_args()
    if args.global_views is not None and args.views_per_gpu is not None:
        ap.error("--global-views (strong scaling) and --views-per-gpu (weak scaling) are exclusive")
    if args.global_views is None and args.views_per_gpu is None:
        args.global_views = DEFAULT_GLOBAL_VIEWS
    if args.ring_order is None:
        args.ring_order = "spread" if args.global_views is not None else "contiguous"
    if args.global_views is not None and args.global_views < args.gpus:
        ap.error(f"--global-views {args.global_views} < --gpus {args.gpus}: every rank needs a view")
    if args.graph == "on" and args.anneal_k is not None:
        ap.error("--graph on freezes the march parameters of the captured step: no --anneal-k")
    if args.as_rank is not None:
        try:
            r, n = (int(x) for x in args.as_rank.split("/"))
        except ValueError:
            ap.error("--as-rank takes R/N")
        if args.global_views is None or args.gpus != 1 or not 0 <= r < n or n > args.global_views:
            ap.error("--as-rank R/N: strong scaling on one GPU, 0 <= R < N <= --global-views")
        args.as_rank = (r, n)
    return args


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """One child process per GPU (this process never touches a GPU). Returns the first nonzero
    exit status, terminating the other ranks when one fails."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


def ring_order(n: int, order: str) -> list[int]:
    """Camera angle index of each ring position. 'spread': position j looks from angle (j * s) mod n,
    s the stride coprime with n nearest 0.618 n (a golden-ratio sequence), so any contiguous slice
    of positions -- a rank's views in strong scaling -- samples the whole circle."""
    if order == "contiguous" or n <= 2:
        return list(range(n))
    import math
    base = max(1, round(0.618 * n))
    s = min((c for c in range(1, n) if math.gcd(c, n) == 1), key=lambda c: (abs(c - base), c))
    return [(j * s) % n for j in range(n)]


def _latest_profile(pattern: str, key: str, field: str):
    """(value, relative path) of `field`[key] in the newest committed profile matching pattern."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), reverse=True):
        try:
            data = json.load(open(path))
        except (OSError, ValueError):
            continue
        if key in data.get(field, {}):
            return data[field][key], os.path.relpath(path, ROOT)
    return None, None


# generate.rs:29-40: the target scene of the reference's data/ ("dango")
DANGO = {"centers": [[-0.3, 0.0, 0.0], [0.0, 0.0, 0.0], [0.3, 0.0, 0.0]],
         "colors": [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]], "radius": [0.2, 0.15, 0.2]}


def load_scene_json(path):
    """scene.json (train.rs:238-262: activated colours / ambient, softplus radii without the +0.01,
    raw light_dir) as the activated scene the renderer sees (radius + 0.01, scene.rs:43)."""
    d = json.load(open(path))
    c = np.asarray(d["centers"], np.float32).reshape(-1, 3)
    return {"centers": c, "colors": np.asarray(d["colors"], np.float32).reshape(-1, 3),
            "radius": (np.asarray(d["radii"], np.float32) + np.float32(0.01)).astype(np.float32),
            "light_dir": np.asarray(d["light_dir"], np.float32).reshape(3),
            "ambient": np.asarray(d["ambient_intensity"], np.float32).reshape(1)}


def load_target_files(cameras_json, entries, W, H):
    """The target PNGs cameras.json names (util.rs:21-33 linear RGB), resolved as rm_train does:
    as given, next to the json, or by file name next to the json."""
    from burn_raymarching_amd import host
    base = os.path.dirname(os.path.abspath(cameras_json))
    out = []
    for e in entries:
        f = e["file"]
        for cand in (f, os.path.join(base, f), os.path.join(base, os.path.basename(f))):
            if os.path.exists(cand):
                break
        img = host.image_load(cand)
        if img.shape[0] != W * H:
            raise SystemExit(f"{cand} has {img.shape[0]} pixels, expected {W}x{H}")
        out.append(img)
    return np.stack(out)


def _json_stdout():
    """The stream for the one JSON line: the process's stdout, while fd 1 itself points at stderr
    for the rest of the run, so that what libraries write there (gloo's connection banner, HIP or
    RCCL diagnostics) cannot interleave the line the driver parses."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w", buffering=1)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if os.environ.get("RM_BENCH_RANK_PROBE") == "1":  # launcher test (CPU): report the rank layout, no GPU
        print(json.dumps({"rank": rank, "local_rank": local, "world": world,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return
    json_out = _json_stdout()

    import torch
    # RM_BENCH_BACKEND=gloo: rehearsal of the N-rank path on fewer GPUs than ranks (ranks share
    # the devices round-robin; RCCL refuses two ranks on one device). Never a measurement.
    backend = os.environ.get("RM_BENCH_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"RM_BENCH_BACKEND={backend}: nccl or gloo")
    if backend == "gloo":
        if torch.cuda.device_count() == 0:
            raise SystemExit("bench.py needs a HIP device")
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    use_graph = args.graph == "on"
    if use_graph:
        if world > 1:
            raise SystemExit("--graph on is for one GPU (the N-rank step keeps its all-reduce eager)")
        torch.cuda.set_stream(torch.cuda.Stream())  # a capturable stream for every call of the run
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            # the measured run must be what it claims: --gpus ranks, each on its own device
            props = torch.cuda.get_device_properties(local)
            me = (socket.gethostname(), str(props.uuid), f"{props.pci_domain_id}:{props.pci_bus_id}:{props.pci_device_id}")
            devices = [None] * world
            dist.all_gather_object(devices, me)
            if dist.get_world_size() != args.gpus or len(set(devices)) != world:
                print(f"error: rank {rank}: world {dist.get_world_size()} for --gpus {args.gpus}, devices {devices}",
                      file=sys.stderr, flush=True)
                sys.exit(3)
        else:
            dist.init_process_group("gloo")

    from burn_raymarching_amd import model as rmm
    from burn_raymarching_amd import native
    from burn_raymarching_amd import render as rmr
    from burn_raymarching_amd.parallel import Shard, ViewShardedStep

    start_scene = load_scene_json(args.scene_json) if args.scene_json else None
    if start_scene is not None:
        args.spheres = int(start_scene["centers"].shape[0])
    W, H, M, S, K = args.width, args.height, args.spheres, args.march_steps, args.smooth_k
    strong = args.global_views is not None
    if not strong and not 1 <= args.views_per_gpu <= native.RM_MAX_VIEWS_PER_CALL:
        raise SystemExit(f"--views-per-gpu must be in 1..{native.RM_MAX_VIEWS_PER_CALL}")
    npix = W * H
    shard = (Shard(args.as_rank[0], args.as_rank[1], 0, 1, args.global_views) if args.as_rank is not None else
             Shard(rank, world, 0 if strong else args.views_per_gpu, 1, args.global_views or 0))
    vpg = shard.count()  # this rank's views per step
    rays_per_rank = vpg * npix
    rays_global = shard.views_total * npix if args.as_rank is None else rays_per_rank
    # views per train call (one launch of up to 128 views / 33.5M rays each)
    views_per_call = max(1, min(native.RM_MAX_VIEWS_PER_CALL, MAX_RAYS_PER_CALL // npix))
    if args.views_per_call > 0:
        views_per_call = min(views_per_call, args.views_per_call)
    ncalls = (vpg + views_per_call - 1) // views_per_call

    # ---- synthetic scene, targets, optimizer --------------------------------------------
    rr = tuple(args.radius_range) if args.radius_range else (
        (0.03, 0.12) if M <= 256 else ((0.02, 0.06) if M <= 1024 else (0.01, 0.04)))
    sc0 = start_scene if start_scene is not None else rmm.synthetic_scene(M, seed=0, radius_range=rr)
    sc1 = rmm.synthetic_scene(M, seed=1, radius_range=rr)
    if args.cameras:  # the reference's poses (data/cameras.json) instead of the synthetic ring
        cam_entries = json.load(open(args.cameras))
        cams = [(c["origin"], c["target"], c["fov"]) for c in cam_entries]
        ring = len(cams)
        if shard.count() > ring:
            raise SystemExit(f"{shard.count()} views per rank per step but {args.cameras} holds {ring} cameras")
    else:
        cam_entries = None
        ring = max(args.ring, shard.views_total)
        cams = [rmm.ring_cameras(ring)[a] for a in ring_order(ring, args.ring_order)]
    shard.ring = ring
    if use_graph and shard.views_total != ring:
        # a captured step freezes its views, target slice and camera bases: replays would train the
        # captured views while eager steps rotate through the ring -- not the same run
        raise SystemExit(f"--graph on needs the same views every step: {shard.views_total} views per step "
                         f"on a ring of {ring} rotate (use --ring {shard.views_total})")
    targets = torch.empty((ring, npix, 3), device="cuda")
    if args.targets == "files":
        targets.copy_(torch.from_numpy(load_target_files(args.cameras, cam_entries, W, H)).view(ring, npix, 3))
    else:
        for v0 in range(0, ring, native.RM_MAX_VIEWS_PER_CALL):
            chunk = cams[v0:v0 + native.RM_MAX_VIEWS_PER_CALL]
            if args.targets == "dango":  # generate.rs:29-40 through the renderer.rs kernel
                t = [torch.tensor(DANGO[k], device="cuda") for k in ("centers", "colors", "radius")]
                img = rmr.render_camera(chunk, W, H, *t)
            else:
                img = rmr.render_diff_camera(chunk, W, H, rmm.scene_tensors(sc1), K, S)
            targets[v0:v0 + len(chunk)] = img.view(len(chunk), npix, 3)
    model = rmm.SceneModel.from_activated(sc0["centers"], np.clip(sc0["colors"], 1e-6, 1 - 1e-6), sc0["radius"],
                                          sc0["light_dir"],
                                          sc0["ambient"], color_dtype=args.color_dtype)
    opt = rmm.Adam(model, weight_decay=1e-5, with_penalties=True)
    march = native.march_params(S, K, skip_escaped=args.skip_escaped == "on")
    # one rm_context per call slot of a step (same stream): each keeps the cost-ordered dispatch
    # state of the views it trains every step
    # one rm_context per call slot of a step: each keeps the cost-ordered dispatch state of the views
    # it trains every step; with --streams K the slots are spread over K streams
    nstreams = max(1, min(args.streams, ncalls))
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(1, nstreams)]
    ctxs = [rmr.context()] + [native.Context(torch.cuda.current_device(), streams[c % nstreams].cuda_stream)
                              for c in range(1, ncalls)]
    ctx = Contexts(ctxs)
    slot_buf = torch.zeros((ncalls, rmm.packed_size(M) + 1), device="cuda") if nstreams > 1 else None
    total_steps = args.warmup + args.steps
    progress = {"i": 0}

    # the ring twice over: a rank's views are consecutive mod ring, so its targets are always one
    # contiguous slice (no gather kernel, no host-built index tensor inside the timed loop)
    targets2 = torch.cat([targets, targets])

    # one GPU, one call per step: the train step and the optimizer as one call (no gradient exchange
    # between them)
    fused_adam = args.fused_adam == "on" and world == 1 and slot_buf is None and ncalls == 1

    def step_fn(views, inv_count, grads_out, loss_out):
        # rm_train_step_camera over this rank's views (fused forward + loss seed + backward), in
        # calls of up to views_per_call views; the later calls add into the gradient and loss
        first = views[0]
        assert views == [(first + j) % ring for j in range(len(views))]
        main = torch.cuda.current_stream()
        if slot_buf is not None:
            start = torch.cuda.Event()
            start.record(main)
        nm = rmm.packed_size(M)
        for c, c0 in enumerate(range(0, len(views), views_per_call)):
            part = views[c0:c0 + views_per_call]
            tg = targets2[part[0]:part[0] + len(part)]
            kw = dict(progress=min(progress["i"] / total_steps, 1.0), steps=S, inv_count=inv_count, march=march,
                      ctx=ctxs[c])
            if fused_adam:  # the optimizer step in the same call (rm_train_step_camera_adam)
                opt.train_step_camera([cams[j] for j in part], W, H, tg.view(-1, 3), K, kw["progress"], args.lr, S,
                                      inv_count=inv_count, grads_packed=grads_out, loss=loss_out, march=march,
                                      ctx=ctxs[c])
                continue
            if slot_buf is None:  # one stream: the later calls add into the gradient and loss
                rmr.train_step_camera([cams[j] for j in part], W, H, tg.view(-1, 3), model.scene(), K,
                                      grads_packed=grads_out, loss=loss_out, accumulate=c > 0, **kw)
                continue
            st = streams[c % nstreams]
            st.wait_event(start)
            with torch.cuda.stream(st):
                rmr.train_step_camera([cams[j] for j in part], W, H, tg.view(-1, 3), model.scene(), K,
                                      grads_packed=slot_buf[c, :nm], loss=slot_buf[c, nm:], **kw)
        if slot_buf is not None:
            for st in streams[1:]:
                main.wait_stream(st)
            tot = slot_buf.sum(0)  # the calls' rows in a fixed order
            grads_out.copy_(tot[:nm])
            loss_out.copy_(tot[nm:])

    dp = ViewShardedStep(shard, npix, rmm.packed_size(M), "cuda", step_fn,
                         optim_fn=None if fused_adam else (lambda g: opt.step(g, args.lr)),
                         collective=args.as_rank is None)
    # graph mode: progress and Adam's step from a device record the optimizer advances (the
    # eager steps of the run read it too, so eager and replayed steps compute the same thing)
    sdev = None
    if use_graph:
        sdev = torch.tensor([1, 0, total_steps, 0], dtype=torch.int32, device="cuda")
        for cx in ctxs:
            cx.bind_step_scalars(sdev.data_ptr())
    loss = dp.loss
    grad0 = []

    def step(i):
        progress["i"] = i
        if args.anneal_k is not None:  # train.rs:174 over the timed steps
            f = min(max((i - args.warmup) / max(args.steps - 1, 1), 0.0), 1.0)
            march.smooth_k = float(args.anneal_k + (K - args.anneal_k) * f)
        dp(i)
        if i == 0 and args.dump_grad and not grad0:
            grad0.append(dp.buf.detach().clone())

    for i in range(args.warmup):
        step(i)
    # snapshot of the training state at the start of the timed region (for the untimed replays)
    snap = (model.raw.clone(), model._act.clone(), opt.m.clone(), opt.v.clone(), opt.t,
            None if model._col_h is None else model._col_h.clone(), None if sdev is None else sdev.clone())

    def restore():
        model.raw.copy_(snap[0])
        model._act.copy_(snap[1])
        opt.m.copy_(snap[2])
        opt.v.copy_(snap[3])
        opt.t = snap[4]
        if snap[5] is not None:
            model._col_h.copy_(snap[5])
        if snap[6] is not None:
            sdev.copy_(snap[6])
        model._act_valid = True

    graph = None
    if use_graph:  # one step captured (not run: the record is not advanced), replayed per timed step
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=torch.cuda.current_stream()):
            step(args.warmup)
        torch.cuda.synchronize()

    torch.cuda.synchronize()
    ctx.collect_timing(reset=True)
    # every n-th step when there are enough to sample (short runs: every step)
    every = max(args.timing_every, 1) if args.steps >= 4 * max(args.timing_every, 1) else 1
    # per-step events on the sampled steps only: an event record is a barrier packet on the stream
    # (~5 us of GPU idle each), which would inflate short steps (C2) if every step had two
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) if j % every == 0 else None
          for j in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timed_steps = 0
    for j, i in enumerate(range(args.warmup, total_steps)):
        timed = args.kernel_timing == "on" and j % every == 0 and graph is None
        ctx.timing(timed)
        dp.time_allreduce = timed
        timed_steps += timed
        if ev[j] is not None:
            ev[j][0].record()
        if graph is None:
            step(i)
        else:
            graph.replay()
        if ev[j] is not None:
            ev[j][1].record()
    host_s = time.perf_counter() - t0  # host time to submit the K steps (before the final sync)
    dp.time_allreduce = False
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.timing(False)
    kern_ms, launches = ctx.collect_timing(reset=True)
    step_ms = torch.tensor([e[0].elapsed_time(e[1]) for e in ev if e is not None], dtype=torch.float64,
                           device="cuda")

    # ---- untimed replays of the timed steps: work statistics, then the canonical kernel time.
    # The training state was snapshotted before the timed region; every step is deterministic,
    # so a replay repeats the timed steps' work exactly (same scenes, same rays).
    def replay(fn_before):
        restore()
        for j, i in enumerate(range(args.warmup, total_steps)):
            fn_before(j)
            step(i)
        torch.cuda.synchronize()

    st = {"blocks": 0, "blocks_skipped": 0, "waves": 0, "waves_exited": 0, "steps_saved": 0}
    canon_ms = None
    exit_off_s = None
    if args.aux_steps > 0:
        ctx.stats(True)
        ctx.collect_stats(reset=True)
        if graph is not None and args.kernel_timing == "on":
            # graph mode: the train kernel timed on this eager replay of the same steps
            ctx.collect_timing(reset=True)
            replay(lambda j: ctx.timing(j % every == 0))
            ctx.timing(False)
            kern_ms, launches = ctx.collect_timing(reset=True)
            timed_steps = sum(1 for j in range(args.steps) if j % every == 0)
        else:
            replay(lambda j: None)
        st = ctx.collect_stats(reset=True)
        ctx.stats(False)
        if args.kernel_timing == "on":  # the same steps with the early exit off (full work per ray)
            march.flags |= native.RM_MARCH_NO_EARLY_EXIT
            ctx.collect_timing(reset=True)
            replay(lambda j: ctx.timing(j % every == 0 and j > 0))
            ctx.timing(False)
            cms, cl = ctx.collect_timing(reset=True)
            canon_steps = sum(1 for j in range(args.steps) if j % every == 0 and j > 0)
            canon_ms = cms / canon_steps if cl and canon_steps else None  # per step (a step may be several launches)
            # the whole step with the exit off (full work per ray), no events inside: value_exit_off
            restore()
            if dist is not None:
                dist.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for i in range(args.warmup, total_steps):
                step(i)
            torch.cuda.synchronize()
            if dist is not None:
                dist.barrier()
            exit_off_s = time.perf_counter() - t1
            march.flags &= ~native.RM_MARCH_NO_EARLY_EXIT

    ranks_info = None
    kern_rank_ms = kern_ms / max(timed_steps, 1)  # this rank's train-kernel time per step
    if dist is not None:
        # per-rank train-kernel and all-reduce times (sampled steps), before the max over ranks
        ar_ms = dp.collect_allreduce_ms()
        # (RCCL gathers device tensors; the gloo rehearsal host tensors)
        mine = torch.tensor([kern_rank_ms, ar_ms if ar_ms is not None else -1.0], dtype=torch.float64,
                            device="cuda" if backend == "nccl" else "cpu")
        every_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every_rank, mine)
        per = torch.stack(every_rank).cpu().numpy()
        ranks_info = {"train_kernel_ms_per_step": [round(float(x), 4) for x in per[:, 0]],
                      "train_kernel_ms_min_max": [round(float(per[:, 0].min()), 4), round(float(per[:, 0].max()), 4)],
                      "allreduce_ms_per_step": [round(float(x), 4) for x in per[:, 1]],
                      "allreduce_ms_min_max": [round(float(per[:, 1].min()), 4), round(float(per[:, 1].max()), 4)],
                      "allreduce_note": "hipEvents on the compute stream around dist.all_reduce of the 7M+5-float "
                                        "[gradient | loss] on every timed step the kernel is timed on: the collective "
                                        "plus the wait for the slowest rank's train step",
                      "allreduce_bytes": 4 * (rmm.packed_size(M) + 1)}
        t = torch.tensor([elapsed, kern_ms, canon_ms or 0.0, exit_off_s or 0.0], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, canon_ms, exit_off_s = float(t[0]), float(t[1]), (float(t[2]) or None), (float(t[3]) or None)
        dist.all_reduce(step_ms, op=dist.ReduceOp.MAX)
    step_ms = step_ms.cpu().numpy()
    med_ms = float(np.median(step_ms))

    blocks_run, blocks_skipped = st["blocks"], st["blocks_skipped"]
    skipped_frac = blocks_skipped / max(blocks_run, 1)
    # march steps not run: whole skipped blocks plus waves that left the march early
    waves_total = max(st["waves"], 1)
    march_saved_frac = (blocks_skipped * 4 * S + st["steps_saved"]) / (waves_total * S)
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
    # the two backward sweeps run only for the rays with non-zero seeds (the kernel's counters;
    # in wave units: rays per counted wave, 64, or a split block's rays)
    rays_replayed = rays_per_rank * args.steps
    rays_per_wave = rays_replayed / waves_total
    seeded = st.get("seeded_rays", 0) + st.get("seeded_rays_a", 0)
    bwd_counted = seeded > 0 or waves_post == 0  # (the small kernel, M <= 32, does not count them)
    bwd_sweeps = seeded / rays_per_wave if bwd_counted else waves_post * 2
    sweeps_run = (waves_total - blocks_skipped * 4) * S - st["steps_saved"] + waves_post * 3 + bwd_sweeps
    have_stats = st["waves"] > 0  # --aux-steps 0 (PMC passes): no statistics, no executed-work figure
    executed_frac = max(0.0, sweeps_run / sweeps_total) if have_stats else None
    kern_step_ms = kern_step_ms or float("nan")  # no timed launches (--kernel-timing off)
    achieved_tf = (flop_per_ray * rays_per_rank * executed_frac / (kern_step_ms * 1e-3) / 1e12
                   if have_stats else None)
    key = (f"{W}x{H}_M{M}_S{S}_V{vpg}" + ("_c16" if args.color_dtype == "f16" else "")
           + (f"_k{K:g}" if K != 32.0 else "") + (f"_ka{args.anneal_k:g}" if args.anneal_k is not None else "")
           + ("_cj" if args.cameras else "")
           + ("_grown" if args.scene_json else ""))
    # per step (the step's launches together), like `achieved`; per launch where no per-step
    # summary exists for this workload
    traffic, traffic_src = _latest_profile("r*_pmc_traffic.json", key, "train_kernel_bytes_per_step")
    traffic_basis = "per step"
    if traffic is None:
        traffic, traffic_src = _latest_profile("r*_pmc_traffic.json", key, "train_kernel_bytes_per_launch")
        traffic_basis = "per launch"
    # the same profile's uncalibrated sum and calibration, so that the line states which figure it quotes
    tdetail, _ = _latest_profile(os.path.basename(traffic_src) if traffic_src else "none", key, "detail")
    traffic_raw = None
    if tdetail and tdetail.get("raw_bytes_per_launch") is not None:
        per_step = tdetail["launches"] / max(tdetail.get("steps") or tdetail["launches"], 1)
        traffic_raw = tdetail["raw_bytes_per_launch"] * (per_step if traffic_basis == "per step" else 1.0)
    pmc, pmc_src = _latest_profile("r*_pmc_sq.json", key, "train_kernel")
    alg_bytes = rays_per_rank * BYTES_PER_RAY_CAMERA  # per step (all of this rank's rays)
    mpad = (M + 31) // 32 * 32
    slab_bytes = (rays_per_rank + 255) // 256 * (mpad * 8 + 8) * 4  # partial-gradient slabs, if all written
    canonical = None
    if canon_ms:
        # with the exit off every ray runs S march + 5 post-march sweeps (reconnect, shade, the normal
        # as the one gradient sweep the kernel runs, 2 backward): 16*(S+5)*M FLOP; the reference's
        # 16*(S+10)*M credits its six normal taps, which this kernel does not run
        # the backward sweeps of the seeded rays only (the same rays with the exit on and off)
        bwd_per_step = (seeded / args.steps) if (bwd_counted and have_stats) else 2 * rays_per_rank
        flop_canon = FLOP_PER_EVAL * M * ((S + 3) * rays_per_rank + bwd_per_step)
        ach = flop_canon / (canon_ms * 1e-3) / 1e12
        ach_all = FLOP_PER_EVAL * (S + 5) * M * rays_per_rank / (canon_ms * 1e-3) / 1e12
        ach_ref = flop_per_ray * rays_per_rank / (canon_ms * 1e-3) / 1e12
        canonical = {"kernel_ms": round(canon_ms, 4), "achieved": round(ach, 3),
                     "frac": round(ach / PEAK_FP32_TFLOPS, 4),
                     "flop_per_ray": round(flop_canon / rays_per_rank),
                     "frac_backward_all_rays": round(ach_all / PEAK_FP32_TFLOPS, 4),
                     "frac_reference_taps": round(ach_ref / PEAK_FP32_TFLOPS, 4),
                     "note": "exit off: 16*M*(S+3) FLOP per ray (march, reconnect, normal, shade) + 16*M per backward "
                             "sweep of a ray with non-zero seeds (rm_stats seeded_rays + seeded_rays_a) over the kernel "
                             "time of the timed steps replayed untimed with the early exit off; "
                             "frac_backward_all_rays credits both backward sweeps to every ray (16*(S+5)*M), "
                             "frac_reference_taps the reference's 16*(S+10)*M (six normal taps)"}
    roofline = None if launches == 0 else {
        "bound": "valu",
        "kernel": "rm_ray_kernel<train,camera>",
        "achieved": round(achieved_tf, 3) if have_stats else None,
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved_tf / PEAK_FP32_TFLOPS, 4) if have_stats else None,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "traffic_basis": traffic_basis,
        "traffic_kind": None if traffic is None else (
            "FETCH_SIZE x read factor + WRITE_SIZE x write factor, factors measured on known byte counts "
            "(tools/fetch_calib)" if tdetail and tdetail.get("calibration") else "raw FETCH_SIZE + WRITE_SIZE"),
        "traffic_raw": None if traffic_raw is None else round(traffic_raw),
        "traffic_calibration": None if not tdetail else tdetail.get("calibration"),
        "kernel_ms": round(kern_avg_ms, 4),
        "kernel_ms_per_step": round(kern_step_ms, 4),
        "launches_timed": launches,
        "flop_per_ray": flop_per_ray,
        "rays_per_launch": rays_per_rank,
        "executed_frac": round(executed_frac, 4) if have_stats else None,
        "executed_frac_source": "rm_stats counters, untimed replay of the timed steps",
        "backward_rays_frac": (None if not (have_stats and bwd_counted) else
                               [round(st.get("seeded_rays", 0) / rays_replayed, 4),
                                round(st.get("seeded_rays_a", 0) / rays_replayed, 4)]),
        "backward_rays_note": "fraction of the rays the two backward sweeps ran for (non-zero seeds; the "
                              "others contribute exact zeros and are not swept): counted as executed work",
        "achieved_all_rays": round(flop_per_ray * rays_per_rank / (kern_step_ms * 1e-3) / 1e12, 3),
        "canonical": canonical,
        "pmc": None if pmc is None else dict(pmc, source=pmc_src),
        "hbm": {"algorithmic_bytes_per_step": alg_bytes,
                "bytes_per_ray": BYTES_PER_RAY_CAMERA,
                "achieved_GBs": round(alg_bytes / (kern_step_ms * 1e-3) / 1e9, 2),
                "peak_GBs": PEAK_HBM_GBS,
                "frac": round(alg_bytes / (kern_step_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 6),
                "partial_slab_bytes_max": slab_bytes},
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
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (seeded scene + targets rendered by the forward kernel)" if args.targets == "synthetic"
                     and not args.scene_json and not args.cameras else
                     f"start scene {'file ' + os.path.basename(args.scene_json) if args.scene_json else 'synthetic seed 0'}"
                     f", targets {args.targets}, poses {'cameras.json' if args.cameras else 'synthetic ring'}"),
            "config": {"workload": (f"train step fwd+bwd, {shard.views_total} {W}x{H} views per step over all GPUs"
                                    if strong else f"train step fwd+bwd, {vpg} {W}x{H} view(s) per GPU")
                                   + f", {M} spheres, {S} march steps, "
                                   + (f"k={K:g}" if args.anneal_k is None else f"k annealed {args.anneal_k:g}->{K:g}")
                                   + ", camera mode, Adam"
                                   + (", fp16 colour / fp32 SDF" if args.color_dtype == "f16" else ""),
                       "width": W, "height": H, "spheres": M, "march_steps": S, "smooth_k": K, "anneal_k_from": args.anneal_k,
                       "views_per_gpu": vpg, "global_views": shard.views_total, "views_per_call": views_per_call,
                       "streams": nstreams, "graph": use_graph, "fused_adam": fused_adam,
                       "ring": ring, "ring_order": args.ring_order, "rays_per_step": rays_global, "radius_range": list(rr),
                       "color_storage": args.color_dtype, "sdf_dtype": "f32",
                       "cameras": args.cameras and os.path.relpath(os.path.abspath(args.cameras), ROOT),
                       "targets": args.targets,
                       "start_scene": args.scene_json and os.path.relpath(os.path.abspath(args.scene_json), ROOT),
                       "parallelism": (f"views-dp{world}" + ("" if backend == "nccl" else f" ({backend} rehearsal)")
                                       if args.as_rank is None else
                                       f"rank {args.as_rank[0]} of views-dp{args.as_rank[1]}, alone on one GPU "
                                       f"(no all-reduce)")},
            "value_median": round(rays_global / (med_ms * 1e-3) / 1e6, 3),
            "value_exit_off": None if not exit_off_s else round(rays_global * args.steps / exit_off_s / 1e6, 3),
            "value_exit_off_note": "the same steps replayed untimed-by-events with the exact early exit off (every "
                                   "ray does the full march): whole-step Mrays/s independent of how many rays escape",
            "ms_per_step_median": round(med_ms, 4),
            "host_submit_ms_per_step": round(host_s / args.steps * 1e3, 4),
            "ms_per_step_min_max": [round(float(step_ms.min()), 4), round(float(step_ms.max()), 4)],
            "roofline": roofline,
            "ranks": ranks_info,
            "cpu_baseline": cpu,
            "escape_skip": {"enabled": args.skip_escaped == "on", "blocks": blocks_run,
                            "blocks_skipped": blocks_skipped, "skipped_frac": round(skipped_frac, 4)},
            "early_exit": {"enabled": os.environ.get("RM_NO_EARLY_EXIT") != "1", "waves": st["waves"],
                           "waves_exited": st["waves_exited"],
                           "exited_frac": round(st["waves_exited"] / waves_total, 4),
                           "march_steps_saved_frac": round(march_saved_frac, 4)},
            "finite": finite,
        }
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
        if args.dump_grad and grad0:
            np.save(args.dump_grad, grad0[0].cpu().numpy())
    if dist is not None:
        dist.destroy_process_group()


class Contexts:
    """The rm_contexts of a step's call slots, timed and counted together."""

    def __init__(self, ctxs):
        self.ctxs = ctxs

    def timing(self, enable=True):
        for c in self.ctxs:
            c.timing(enable)

    def collect_timing(self, reset=True):
        ms, n = 0.0, 0
        for c in self.ctxs:
            a, b = c.collect_timing(reset=reset)
            ms += a
            n += b
        return ms, n

    def stats(self, enable=True):
        for c in self.ctxs:
            c.stats(enable)

    def collect_stats(self, reset=True):
        tot = {}
        for c in self.ctxs:
            for k, v in c.collect_stats(reset=reset).items():
                tot[k] = tot.get(k, 0) + v
        return tot


def cpu_baseline(args, sc0, sc1, cam, W, H, M, S, K):
    """Oracle fp32 reference-order restatement (OpenMP) on a strided sample of the view: at the
    CPU share of this box (OMP_NUM_THREADS, else the affinity mask) and on one core."""
    from oracle import oracle as orc
    o, d = orc.camera_rays(W, H, *cam, precision="f32")
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    threads = int(os.environ.get("OMP_NUM_THREADS") or share)

    def rate(n_rays, seconds, nthreads):
        orc.set_threads(nthreads)
        stride = max(1, (W * H) // max(n_rays, 1))
        idx = np.arange(0, W * H, stride)
        oo, dd = o[idx], d[idx]
        tg = orc.render_diff(oo, dd, sc1, S, K, precision="f32")
        reps = 0
        t0 = time.perf_counter()
        while True:  # repeat the sample for ~`seconds` of CPU work (bounded: at most 30 repetitions)
            orc.train_step(oo, dd, tg, sc0, S, K, 0.5, precision="f32")
            reps += 1
            sec = time.perf_counter() - t0
            if sec >= seconds or reps >= 30:
                break
        return reps * len(idx) / sec / 1e6, reps, len(idx), stride, sec

    v1, r1, n1, s1, t1 = rate(max(args.cpu_sample // 16, 1), max(args.cpu_seconds / 4, 0.05), 1)
    vn, rn, nn, sn, tn = rate(args.cpu_sample, args.cpu_seconds, threads)
    return {"value": round(vn, 6), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "single_core_value": round(v1, 6), "hardware_threads": os.cpu_count(), "affinity_cpus": share,
            "all_hw_threads_linear_estimate": round(v1 * (os.cpu_count() or 1), 4),
            "sample": f"{rn} x {nn} rays (every {sn}th pixel of one {W}x{H} view) on {threads} threads "
                      f"({tn:.2f} s) and {r1} x {n1} rays on 1 thread ({t1:.2f} s); fwd+bwd train step, {M} spheres, "
                      f"{S} steps, fp32 reference op order, OpenMP. The box's CPU share is {threads} threads; "
                      f"the all-thread figure is a linear estimate, not measured"}


if __name__ == "__main__":
    main()
