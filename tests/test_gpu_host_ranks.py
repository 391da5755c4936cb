"""Data-parallel training in the C++ host driver (rmh_train with an rmh_collective, SURVEY.md
§8(e); the reference's schedule train.rs:138-330 with prune_and_split training.rs:87-238
between stages).

  * `rm_train train --ranks 1`: the CLI's rank launcher (fork before any GPU use) and the real
    RCCL communicator (one rank: its all-reduce and broadcasts run on the device);
  * two rank processes on the test box's one GPU with a gloo collective plugged in through the
    C ABI (RCCL refuses two ranks on one device; the driver's collective calls are the same):
    the collective sequence (one all-reduce of 7M+5 floats per step, then per stage transition a
    broadcast of the size and of the 7M'+4 raw parameters), every reduced buffer = the sum of
    the ranks' local buffers, broadcasts deliver rank 0's data, and both ranks end with
    bit-identical parameters;
  * an identity collective on one rank changes no bit of the single-process run.
"""
import ctypes
import json
import os
import socket
import subprocess
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

STAGES, STEPS, BATCH = 2, 40, 4096


def _hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    return h


def _cfg(H, seed=3):
    return H.train_config(cameras_json=os.path.join(GOLDEN, "cameras.json"), out_dir=None, log_every=0, previews=0,
                          stages=STAGES, steps_per_stage=STEPS, batch=BATCH, seed=seed)


def _gloo_collective(H, rank, world, log):
    """rmh_collective over torch.distributed (gloo) on host copies of the device buffers."""
    import torch
    import torch.distributed as dist
    hip = _hip()

    def fetch(buf, count, stream):
        assert hip.hipStreamSynchronize(stream) == 0
        a = np.empty(count, np.float32)
        assert hip.hipMemcpy(a.ctypes.data, buf, 4 * count, 2) == 0  # device -> host
        return a

    def store(buf, a):
        assert hip.hipMemcpy(buf, a.ctypes.data, 4 * a.size, 1) == 0  # host -> device

    def all_reduce(buf, count, stream):
        a = fetch(buf, count, stream)
        t = torch.from_numpy(a.copy())
        dist.all_reduce(t)
        store(buf, t.numpy())
        log.append(("ar", count, a, t.numpy().copy()))

    def broadcast(buf, count, root, stream):
        a = fetch(buf, count, stream)
        t = torch.from_numpy(a.copy())
        dist.broadcast(t, root)
        store(buf, t.numpy())
        log.append(("bc", count, a, t.numpy().copy()))

    return H.collective(rank, world, all_reduce, broadcast)


def _worker(rank, world, port, out_dir, grow=False):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from burn_raymarching_amd import host as H
    log = []
    comm = _gloo_collective(H, rank, world, log)
    cfg = _cfg(H)
    if grow:  # configs[4]-style growth: every surviving sphere splits, 128 march steps, fp16 colours
        cfg.stages, cfg.steps_per_stage, cfg.march_steps = 8, 6, 128
        cfg.split_scale, cfg.split_move, cfg.color_f16 = -1.0, -1.0, 1
    cfg.comm = ctypes.pointer(comm)
    res, raw = H.train(cfg)
    np.save(os.path.join(out_dir, f"raw{rank}.npy"), raw)
    seq = [(k, c) for k, c, _, _ in log]
    json.dump({"seq": seq, "M": res.num_spheres, "steps": res.steps}, open(os.path.join(out_dir, f"r{rank}.json"), "w"))
    # first and last all-reduce and every broadcast: local (pre) and reduced (post) buffers
    keep = [i for i, e in enumerate(log) if e[0] == "bc"] + [0, len(log) - 1]
    np.savez(os.path.join(out_dir, f"bufs{rank}.npz"),
             **{f"pre{i}": log[i][2] for i in keep}, **{f"post{i}": log[i][3] for i in keep})
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_two_rank_growth_broadcasts_large_generations():
    """The rank-0 broadcast of the next generation at configs[4]-style growth (7 -> ~900 spheres,
    128 march steps, fp16 colours): every stage transition broadcasts the size, then 7M'+4 raw
    parameters; both ranks end bit-identical, past 512 spheres."""
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, _free_port(), tmp, True), nprocs=world, join=True,
                           start_method="spawn")
        r = [json.load(open(os.path.join(tmp, f"r{q}.json"))) for q in range(world)]
        raw = [np.load(os.path.join(tmp, f"raw{q}.npy")) for q in range(world)]
        assert np.array_equal(raw[0], raw[1]) and np.isfinite(raw[0]).all()
        assert r[0]["M"] == r[1]["M"] and r[0]["M"] > 512, r[0]["M"]
        sizes = [c for k, c in r[0]["seq"] if k == "bc" and c != 1]
        assert len(sizes) == 7 and sizes[-1] == 7 * r[0]["M"] + 4


@pytest.mark.timeout(300)
def test_two_rank_driver_over_plugged_collective():
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_worker, args=(world, _free_port(), tmp), nprocs=world, join=True, start_method="spawn")
        r = [json.load(open(os.path.join(tmp, f"r{q}.json"))) for q in range(world)]
        raw = [np.load(os.path.join(tmp, f"raw{q}.npy")) for q in range(world)]
        bufs = [np.load(os.path.join(tmp, f"bufs{q}.npz")) for q in range(world)]
        assert np.array_equal(raw[0], raw[1])  # replicated parameters stay identical
        assert r[0]["seq"] == r[1]["seq"] and r[0]["steps"] == STAGES * STEPS
        seq = r[0]["seq"]
        # the collective schedule: STEPS all-reduces per stage, a size + params broadcast between
        kinds = [k for k, _ in seq]
        assert kinds == (["ar"] * STEPS + ["bc", "bc"]) * (STAGES - 1) + ["ar"] * STEPS
        assert seq[0][1] == 7 * 7 + 5  # the 7-sphere initial model: gradient + loss sum
        m_next = None
        for i, (k, c) in enumerate(seq):
            if k == "bc" and c == 1:
                m_next = int(bufs[0][f"post{i}"][0])
            elif k == "bc":
                assert c == 7 * m_next + 4
        assert seq[-1][1] == 7 * r[0]["M"] + 5
        for key in bufs[0].files:
            i = int(key[4:]) if key.startswith("post") else None
            if i is None:
                continue
            pre0, pre1 = bufs[0][f"pre{i}"], bufs[1][f"pre{i}"]
            post0, post1 = bufs[0][f"post{i}"], bufs[1][f"post{i}"]
            assert np.array_equal(post0, post1), i
            if seq[i][0] == "ar":
                assert np.array_equal(post0, pre0 + pre1), i  # sum of the two ranks' local buffers
                assert not np.array_equal(pre0, pre1)          # rank-distinct batches
            else:
                assert np.array_equal(post0, pre0), i          # rank 0's data everywhere


def test_identity_collective_changes_nothing():
    from burn_raymarching_amd import host as H
    res_a, raw_a = H.train(_cfg(H, seed=5))
    calls = []
    comm = H.collective(0, 1, lambda b, c, s: calls.append(c), lambda b, c, r, s: calls.append(-c))
    cfg = _cfg(H, seed=5)
    cfg.comm = ctypes.pointer(comm)
    res_b, raw_b = H.train(cfg)
    assert np.array_equal(raw_a, raw_b) and res_a.num_spheres == res_b.num_spheres
    assert len(calls) == STAGES * STEPS + 2 * (STAGES - 1)


def test_cli_ranks_1_over_rccl(tmp_path):
    exe = os.path.join(ROOT, "burn_raymarching_amd", "lib", "rm_train")
    out = subprocess.run([exe, "train", "--ranks", "1", "--cameras", os.path.join(GOLDEN, "cameras.json"),
                          "--out", str(tmp_path), "--stages", str(STAGES), "--steps", str(STEPS), "--batch",
                          str(BATCH), "--log-every", "0", "--no-previews"], capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["ranks"] == 1 and line["steps"] == STAGES * STEPS
    assert os.path.exists(tmp_path / "scene.json")


def _failing_worker(rank, world, port, out_dir):
    """Rank 0's all-reduce fails at its 5th step (an injected fault); both ranks must leave
    rmh_train with an error -- rank 0 from the fault, rank 1 because its peer is gone -- instead of
    rank 1 waiting in the collective forever."""
    import sys
    import datetime
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    from burn_raymarching_amd import host as H
    hip = _hip()
    calls = {"n": 0}

    def all_reduce(buf, count, stream):
        calls["n"] += 1
        if rank == 0 and calls["n"] == 5:
            raise RuntimeError("injected fault")
        assert hip.hipStreamSynchronize(stream) == 0
        a = np.empty(count, np.float32)
        assert hip.hipMemcpy(a.ctypes.data, buf, 4 * count, 2) == 0
        t = torch.from_numpy(a)
        dist.all_reduce(t)
        assert hip.hipMemcpy(buf, t.numpy().ctypes.data, 4 * count, 1) == 0

    def broadcast(buf, count, root, stream):
        raise RuntimeError("no stage transition in this test")

    def abort():  # the failing rank releases its side: its peer's pending collective then fails
        dist.destroy_process_group()

    comm = H.collective(rank, world, all_reduce, broadcast, abort=abort)
    cfg = _cfg(H)
    cfg.stages = 1
    cfg.comm = ctypes.pointer(comm)
    err = None
    try:
        H.train(cfg)
    except H.HostError as e:
        err = str(e)
    json.dump({"rank": rank, "error": err, "calls": calls["n"]}, open(os.path.join(out_dir, f"f{rank}.json"), "w"))


@pytest.mark.timeout(200)
def test_failing_rank_does_not_hang_its_peer():
    world = 2
    with tempfile.TemporaryDirectory() as tmp:
        mp.start_processes(_failing_worker, args=(world, _free_port(), tmp), nprocs=world, join=True,
                           start_method="spawn")
        r = [json.load(open(os.path.join(tmp, f"f{q}.json"))) for q in range(world)]
        assert r[0]["error"] and "all-reduce of the gradient" in r[0]["error"] and r[0]["calls"] == 5
        assert r[1]["error"] and "all-reduce of the gradient" in r[1]["error"], r[1]


def test_rccl_watchdog_aborts_a_stalled_stream():
    """The RCCL collective's watchdog (rmh_collective.wait, csrc/host/comm.cpp) on one GPU: a
    one-rank communicator does one real all-reduce, then its stream is held by a kernel that spins
    on a host-mapped flag (rm_debug_stall, standing for a collective whose peer died). wait() must
    notice that the stream has not drained within the collective's timeout, abort the communicator
    and return an error; the aborted communicator refuses further collectives (VERDICT r05 item 6;
    the reference panics instead, train.rs:66-68). ncclCommAbort itself waits for the device's
    in-flight work (measured: with the stall left to its own 60 s end the abort returned with it),
    which a stuck RCCL kernel leaves at once -- the abort makes it exit -- but this stand-in kernel
    does not, so a timer releases it one second after the timeout."""
    import threading
    import time
    import torch
    from burn_raymarching_amd import host as H, native
    s = torch.cuda.Stream()
    ctx = native.Context(0, s.cuda_stream)
    c = H.RmhCollective()
    timeout = 2.0
    assert H.lib().rmh_collective_rccl_create(0, 1, 0, None, b"watchdog-test", timeout, ctypes.byref(c)) == 0, \
        H.lib().rmh_last_error()
    try:
        buf = torch.arange(64, dtype=torch.float32, device="cuda")
        ref = buf.clone()
        torch.cuda.synchronize()
        assert c.all_reduce_sum(c.state, buf.data_ptr(), 64, s.cuda_stream) == 0
        assert c.wait(c.state, s.cuda_stream) == 0  # drains at once
        assert torch.equal(buf, ref)  # one rank: the sum is the buffer
        ctx.check(ctx._lib.rm_debug_stall(ctx.handle, 60000), "rm_debug_stall")
        t0 = time.monotonic()
        release = threading.Timer(timeout + 1.0, lambda: ctx._lib.rm_debug_stall_release(ctx.handle))
        release.start()
        rc = c.wait(c.state, s.cuda_stream)
        waited = time.monotonic() - t0
        release.join()
        msg = H.lib().rmh_last_error().decode()
        print(f"wait returned {rc} after {waited:.2f} s: {msg}")
        assert rc == H.RMH_ERR_GPU, (rc, msg)
        assert "did not drain" in msg and "communicator aborted" in msg, msg
        assert timeout <= waited < timeout + 10, waited  # the timeout, the release, the abort
        assert c.all_reduce_sum(c.state, buf.data_ptr(), 64, s.cuda_stream) != 0  # aborted
        assert "aborted" in H.lib().rmh_last_error().decode()
    finally:
        ctx._lib.rm_debug_stall_release(ctx.handle)
        s.synchronize()
        H.lib().rmh_collective_rccl_destroy(ctypes.byref(c))
    ctx.close()
