"""bench.py's JSON line (the driver's contract): one small run on the GPU in a child process --
every contract key present, the throughput positive and consistent with ms_per_step, the
roofline and cpu_baseline objects filled, and the early-exit / work statistics in range."""
import json
import os
import subprocess
import sys

import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                         text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


def test_bench_json_contract():
    d = _bench("--steps", "4", "--warmup", "1", "--width", "128", "--height", "128", "--views-per-gpu", "2",
               "--cpu-sample", "2048", "--cpu-seconds", "0.2")
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1
    assert d["unit"] == "Mrays/s" and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["value"] > 0 and d["finite"]
    rays = d["config"]["rays_per_step"]
    assert rays == 2 * 128 * 128
    assert abs(d["value"] - rays / (d["ms_per_step"] * 1e-3) / 1e6) <= 0.01 * d["value"]
    assert "workload" in d["config"]
    r = d["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in r, key
    assert r["launches_timed"] == 4  # short runs time every step
    assert 0 < r["frac"] < 1 and abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    assert 0 < r["executed_frac"] <= 1
    assert r["kernel_ms"] > 0 and r["kernel_ms"] <= d["ms_per_step"] * 1.05
    c = d["cpu_baseline"]
    assert c["value"] > 0 and c["kind"] in ("port", "reference") and c["cores"] >= 1 and c["sample"]
    ee = d["early_exit"]
    assert 0 <= ee["exited_frac"] <= 1 and 0 <= ee["march_steps_saved_frac"] <= 1


def test_bench_without_kernel_timing():
    d = _bench("--steps", "2", "--warmup", "1", "--width", "64", "--height", "64", "--views-per-gpu", "1",
               "--cpu-baseline", "off", "--kernel-timing", "off")
    assert d["value"] > 0 and d["roofline"] is None and d["cpu_baseline"] is None


def test_graph_refuses_rotating_views():
    """--graph captures one step: its views are frozen into the graph, so a run whose views rotate
    over a larger ring is refused rather than timed on other work than its eager steps."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--graph", "on", "--views-per-gpu", "2",
                          "--ring", "10", "--width", "64", "--height", "64", "--steps", "2", "--cpu-baseline", "off"],
                         cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode != 0 and "--graph on needs the same views every step" in out.stderr, out.stderr[-2000:]


def test_bench_annealed_k_and_rank_share():
    """--anneal-k K0 (train.rs:174's schedule over the timed steps) is named in the workload and the
    config; --as-rank R/N runs rank R's fixed share of an N-rank strong step alone (its views, its
    rays in value); the backward sweeps' ray shares are reported and bounded."""
    d = _bench("--steps", "3", "--warmup", "1", "--width", "64", "--height", "64", "--global-views", "4",
               "--ring", "4", "--anneal-k", "5", "--cpu-baseline", "off")
    assert d["config"]["anneal_k_from"] == 5.0 and "k annealed 5->32" in d["config"]["workload"]
    bw = d["roofline"]["backward_rays_frac"]
    assert bw is not None and 0 < bw[1] <= bw[0] <= 1
    d = _bench("--steps", "3", "--warmup", "1", "--width", "64", "--height", "64", "--global-views", "8",
               "--ring", "8", "--as-rank", "1/4", "--cpu-baseline", "off")
    assert d["config"]["rays_per_step"] == 2 * 64 * 64 and "rank 1 of views-dp4" in d["config"]["parallelism"]
    assert abs(d["value"] - 2 * 64 * 64 / (d["ms_per_step"] * 1e-3) / 1e6) <= 0.01 * d["value"]
