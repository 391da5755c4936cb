"""The build's C1 golden vectors (made by tools/make_golden.py from the
oracle): the oracle still reproduces them (CPU), and the GPU path matches the fp64 values
(GPU, same tolerances as tests/test_gpu_parity.py)."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, gpu_available

FILES = sorted(glob.glob(os.path.join(GOLDEN, "c1_S*_k*.npz")))
KEYS = ("centers", "radius", "colors", "light_dir", "ambient")


def _scene(z):
    return {k: z["scene_" + k] for k in KEYS}


def test_golden_files_present():
    assert len(FILES) == 4


@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_oracle_reproduces_golden(oracle, path):
    z = np.load(path)
    steps, k = int(z["steps"]), float(z["smooth_k"])
    o, d = z["ray_org"], z["ray_dir"]
    for prec, dt, rtol in (("f64", np.float64, 1e-10), ("f32", np.float32, 2e-4)):
        out = oracle.render_diff(o, d, _scene(z), steps, k, precision=prec)
        assert np.array_equal(out, z[f"out_{prec}"])  # per-ray work is deterministic
        gr = oracle.render_diff_backward(o, d, _scene(z), steps, k, z["grad_out"].astype(dt), precision=prec)
        for key in KEYS:
            ref = z[f"grad_{key}_{prec}"]
            assert np.allclose(gr[key], ref, rtol=rtol, atol=rtol * np.abs(ref).max()), (prec, key)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")
@pytest.mark.parametrize("path", FILES, ids=os.path.basename)
def test_gpu_matches_golden(path):
    import torch
    from burn_raymarching_amd import render
    from test_gpu_parity import FWD_MAX, FWD_MEAN
    from conftest import GRAD_KEYS, GRAD_TOL, PER_SPHERE, REL_ELEM, REL_L2, grad_errors, record_margin
    z = np.load(path)
    steps, k = int(z["steps"]), float(z["smooth_k"])
    dv = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()
    sc = render.Scene(*(dv(z["scene_" + key]) for key in ("centers", "colors", "radius", "light_dir", "ambient")))
    out = render.render_diff_forward(dv(z["ray_org"]), dv(z["ray_dir"]), sc, k, steps).cpu().numpy()
    e = np.abs(out - z["out_f64"])
    assert e.max() <= FWD_MAX and e.mean() <= FWD_MEAN, (e.max(), e.mean())
    gr = render.render_diff_backward(dv(z["ray_org"]), dv(z["ray_dir"]), sc, k, dv(z["grad_out"]), steps)
    for key in GRAD_KEYS:
        tol = GRAD_TOL
        ref = z[f"grad_{key}_f64"].reshape(-1)
        err = np.abs(gr[key].cpu().numpy().reshape(-1) - ref).max()
        # the bar is the stated tolerance, or twice the error of the reference's own f32 op order
        # where that is larger (light_dir with a random upstream gradient sums n over rays with
        # cancelling signs: the f32 restatement is 8e-2 off at S=16, k=5)
        f32_err = np.abs(z[f"grad_{key}_f32"].astype(np.float64).reshape(-1) - ref).max()
        assert err <= max(tol * np.abs(ref).max(), 2.0 * f32_err), (key, err, f32_err)
        if key not in PER_SPHERE:
            continue
        # check_grads' relative bounds per sphere group: relative L2 and per element (tiers of
        # |g| >= 1e-2 / 1e-3 of the largest), each at least twice the reference f32 op order's own
        # error at this vector (c1_S16_k32: the f32 restatement's centres are 0.112 off at the
        # 1e-3 tier, over the 0.1 of tests/conftest.py)
        _, rl2, tiers = grad_errors(gr[key].cpu().numpy(), ref)
        _, rl2_32, tiers_32 = grad_errors(z[f"grad_{key}_f32"], ref)
        bound = max(REL_L2["bwd"], 2.0 * rl2_32)
        record_margin("golden_relL2_" + key, rl2, bound)
        assert rl2 <= bound, (key, "relL2", rl2, bound)
        for (floor, e_gpu), (_, e_32), (_, rel) in zip(tiers, tiers_32, REL_ELEM["bwd"]):
            bound = max(rel, 2.0 * e_32)
            record_margin(f"golden_elem{floor:g}_{key}", e_gpu, bound)
            assert e_gpu <= bound, (key, floor, e_gpu, bound)
