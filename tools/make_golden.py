"""Generate the build's C1 golden vectors with the CPU oracle.

C1 = 64x64 rays of one view, M = 8 spheres (synthetic_scene(8, seed=0)), S in {16, 40},
k in {5, 32}: the forward image and the five gradient arrays of render_diff for a fixed
seeded upstream gradient g ~ N(0, 1) (numpy PCG64 seed 1), in fp64 and fp32.

    python tools/make_golden.py     ->  tests/golden/c1_S{S}_k{k}.npz

The fp64 values are the parity anchor for the GPU (tests/test_gpu_parity.py); the fp32
values record the oracle in the reference's f32 op order. Re-running reproduces the files
up to the summation order of the OpenMP gradient reduction.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from burn_raymarching_amd.model import synthetic_scene  # noqa: E402
from oracle import oracle as orc  # noqa: E402

W = H = 64
EYE, TARGET, FOV = [2.5, 0.5, 0.0], [0.0, 0.0, 0.0], 50.0  # ring camera 0 (generate.rs:44-63)
CASES = [(16, 5.0), (16, 32.0), (40, 5.0), (40, 32.0)]


def case(steps, k):
    sc = synthetic_scene(8, seed=0)
    o, d = orc.camera_rays(W, H, EYE, TARGET, FOV)
    g = np.random.default_rng(1).standard_normal((W * H, 3))
    rec = {"ray_org": o, "ray_dir": d, "grad_out": g.astype(np.float64), "steps": np.int32(steps),
           "smooth_k": np.float64(k)}
    for key in ("centers", "colors", "radius", "light_dir", "ambient"):
        rec["scene_" + key] = np.asarray(sc[key], np.float32)
    for prec, dt in (("f64", np.float64), ("f32", np.float32)):
        out = orc.render_diff(o, d, sc, steps, k, precision=prec)
        gr = orc.render_diff_backward(o, d, sc, steps, k, g.astype(dt), precision=prec)
        rec[f"out_{prec}"] = np.asarray(out, dt)
        for key, v in gr.items():
            rec[f"grad_{key}_{prec}"] = np.asarray(v, dt)
    return rec


def main():
    orc.build()
    out_dir = os.path.join(ROOT, "tests", "golden")
    for steps, k in CASES:
        path = os.path.join(out_dir, f"c1_S{steps}_k{int(k)}.npz")
        np.savez_compressed(path, **case(steps, k))
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
