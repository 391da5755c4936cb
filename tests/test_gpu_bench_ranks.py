"""bench.py's N-rank path end to end on the one-GPU test box: `--gpus 2` without WORLD_SIZE
starts two rank processes itself, each runs the real HIP train step on its own views, the
gradient all-reduce and the max-over-ranks timing go through torch.distributed -- over gloo
(RM_BENCH_BACKEND=gloo, both ranks on the one device), since RCCL refuses two ranks on one
device. The 8-GPU run uses the same code with RCCL. Checked: one JSON line (rank 0), n_gpus 2,
the rays of both ranks in `value`, finite parameters after the steps."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.mark.timeout(300)
def test_bench_two_ranks_gloo_rehearsal():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RM_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
                        "--views-per-gpu", "2", "--cpu-baseline", "off", "--aux-steps", "0"],
                       env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["warmup"] == 1
    assert d["config"]["rays_per_step"] == 2 * 2 * 512 * 512
    assert d["config"]["parallelism"].startswith("views-dp2")
    assert d["value"] > 0 and d["finite"]
    assert abs(d["value"] - d["config"]["rays_per_step"] / (d["ms_per_step"] * 1e-3) / 1e6) <= 0.01 * d["value"]
    # where a multi-rank step's time goes: per-rank train-kernel and all-reduce times
    rk = d["ranks"]
    assert len(rk["train_kernel_ms_per_step"]) == 2 and len(rk["allreduce_ms_per_step"]) == 2
    assert 0 < rk["train_kernel_ms_min_max"][0] <= rk["train_kernel_ms_min_max"][1]
    assert all(x >= 0 for x in rk["allreduce_ms_per_step"]) and rk["allreduce_bytes"] == 4 * (7 * 256 + 5)


@pytest.mark.timeout(400)
def test_strong_scaling_two_ranks_equal_one(tmp_path):
    """--global-views 4 (strong scaling): two ranks (gloo rehearsal on the one GPU) each train
    two of the four views; the all-reduced gradient of step 0 equals the one-rank run's over all
    four views up to the summation order (fp32 rounding), and the line says "strong"."""
    import numpy as np
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RM_BENCH_BACKEND"] = "gloo"
    common = ["--steps", "2", "--warmup", "1", "--global-views", "4", "--cpu-baseline", "off", "--aux-steps", "0",
              "--width", "256", "--height", "256"]
    lines = {}
    for n in (1, 2):
        dump = str(tmp_path / f"g{n}.npy")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dump-grad", dump]
                           + common, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-2000:]
        out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(out) == 1, r.stdout
        lines[n] = json.loads(out[0])
        assert lines[n]["scaling"] == "strong" and lines[n]["n_gpus"] == n
        assert lines[n]["config"]["global_views"] == 4 and lines[n]["config"]["views_per_gpu"] == 4 // n
        assert lines[n]["config"]["rays_per_step"] == 4 * 256 * 256
    a, b = np.load(tmp_path / "g1.npy"), np.load(tmp_path / "g2.npy")
    assert np.isfinite(a).all() and np.isfinite(b).all()
    assert np.abs(a - b).max() <= 1e-5 * np.abs(a).max(), np.abs(a - b).max() / np.abs(a).max()
