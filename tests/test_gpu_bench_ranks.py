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
