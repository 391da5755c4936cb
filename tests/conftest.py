import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: larger cases")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.build()
    return orc


def load_png(path):
    from PIL import Image
    return np.asarray(Image.open(path).convert("RGB"))


def final1_scene():
    """scene.json (reference, N=6) with the +0.01 radius offset render_diff saw (scene.rs:43 vs
    train.rs:216): colours and ambient are stored post-sigmoid, light_dir raw."""
    sc = json.load(open(os.path.join(GOLDEN, "scene.json")))
    return {
        "centers": np.array(sc["centers"], np.float32).reshape(-1, 3),
        "colors": np.array(sc["colors"], np.float32).reshape(-1, 3),
        "radius": (np.array(sc["radii"], np.float32) + np.float32(0.01)).astype(np.float32),
        "light_dir": np.array(sc["light_dir"], np.float32),
        "ambient": np.array(sc["ambient_intensity"], np.float32),
    }


# train.rs:37-44: the preview camera that produced steps/final_1.png
FINAL1_CAMERA = ([0.0, 0.0, -2.5], [0.0, 0.0, 0.0], 50.0)

# generate.rs:29-40: the target "dango" scene
DANGO = {
    "centers": np.array([[-0.3, 0.0, 0.0], [0.0, 0.0, 0.0], [0.3, 0.0, 0.0]], np.float32),
    "colors": np.eye(3, dtype=np.float32),
    "radius": np.array([0.2, 0.15, 0.2], np.float32),
}


# Parity margins: every GPU-vs-oracle comparison records its measured error next to its bound,
# and the session writes them to gpurun_out/parity_margins.json (copied into profiles/ per
# round), so the committed evidence states how close each case sits to its tolerance.
_MARGINS = []


def record_margin(quantity, err, bound):
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    _MARGINS.append({"test": test, "quantity": quantity, "err": float(err), "bound": float(bound),
                     "ratio": float(err) / float(bound) if bound > 0 else None})


def pytest_sessionfinish(session, exitstatus):
    if not _MARGINS:
        return
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    worst = {}
    for m in _MARGINS:
        q = m["quantity"]
        if m["ratio"] is not None and (q not in worst or m["ratio"] > worst[q]["ratio"]):
            worst[q] = m
    with open(os.path.join(out, "parity_margins.json"), "w") as f:
        json.dump({"worst_by_quantity": worst, "cases": _MARGINS}, f, indent=1)


# ---- gradient parity (every -m gpu comparison of a gradient against the fp64 oracle) ----------
# Three bounds per parameter group:
#  1. normwise: max |a - b| <= GRAD_TOL * max |b| (all five groups);
#  2. relative L2: ||a - b||_2 / ||b||_2 <= REL_L2[mode] (the per-sphere groups);
#  3. per element: |a - b| <= rel * |b| for every element with |b| >= floor * max |b| (the
#     per-sphere groups), tiers REL_ELEM[mode] = ((floor, rel), ...): a sphere whose gradient is
#     wrong (dropped, sign-flipped) fails here even when it is small next to the group's largest.
# Bounds 2 and 3 are set from the fp32 reference-order oracle's own error against the fp64 oracle
# at the same cases (tests/test_oracle.py::test_fp32_gradient_error_within_gpu_bounds pins that
# it stays inside them; worst fp32 values measured at the -m gpu cases, incl. the 2 x 512^2 bench
# workload: backward relL2 4.2e-4, element >= 1e-2 max 2.6e-2, >= 1e-3 max 3.5e-2; train step
# 1.8e-3, 8.3e-2, 1.7e-1 -- the L1 seed sign(out - target) flips where out ~ target).
# light_dir (3 values, a sum that cancels across rays) and ambient (1 value) keep bound 1, which
# over so few elements is already a per-element bound.
GRAD_TOL = 3e-3
GRAD_KEYS = ("centers", "colors", "radius", "light_dir", "ambient")
PER_SPHERE = ("centers", "colors", "radius")
REL_L2 = {"bwd": 1e-3, "train": 3e-3}
REL_ELEM = {"bwd": ((1e-2, 5e-2), (1e-3, 1e-1)), "train": ((1e-2, 0.15), (1e-3, 0.3))}


def grad_errors(a, b):
    """(normwise, relative L2, [(floor, worst element relative error)]) of a against b."""
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    bmax = max(np.abs(b).max(), 1e-12)
    norm = np.abs(a - b).max() / bmax
    if np.abs(b).max() < 1e-12:  # a group the rays do not reach (fp32 underflow): bound 1 only
        return norm, 0.0, [(floor, 0.0) for floor, _ in REL_ELEM["bwd"]]
    rl2 = np.linalg.norm(a - b) / np.linalg.norm(b)
    tiers = []
    for floor, _ in REL_ELEM["bwd"]:
        big = np.abs(b) >= floor * bmax
        tiers.append((floor, float((np.abs(a - b)[big] / np.abs(b)[big]).max()) if big.any() else 0.0))
    return norm, rl2, tiers


def check_grads(got, ref, scale=1.0, mode="bwd", tol=GRAD_TOL):
    """got: dict of device tensors / arrays; ref: dict of fp64 arrays. mode: "bwd" (smooth
    upstream gradient) or "train" (the L1 seed). scale loosens every bound (documented cases)."""
    for key in GRAD_KEYS:
        a = got[key]
        if hasattr(a, "detach"):
            a = a.detach().float().cpu().numpy()
        b = np.asarray(ref[key], np.float64)
        norm, rl2, tiers = grad_errors(a, b)
        record_margin("grad_" + key, norm, tol * scale)
        assert norm <= tol * scale, (key, "normwise", norm, tol * scale)
        if key not in PER_SPHERE:
            continue
        record_margin("grad_relL2_" + key, rl2, REL_L2[mode] * scale)
        assert rl2 <= REL_L2[mode] * scale, (key, "relL2", rl2, REL_L2[mode] * scale)
        for (floor, err), (_, bound) in zip(tiers, REL_ELEM[mode]):
            record_margin(f"grad_elem{floor:g}_{key}", err, bound * scale)
            assert err <= bound * scale, (key, f"element (|g| >= {floor:g} max)", err, bound * scale)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
