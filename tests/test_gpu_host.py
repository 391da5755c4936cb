"""GPU tests of the C++ host programs (librm_host.so / rm_train) over libraymarch_hip.so:
generate.rs reproduces the reference's data/ fixtures, the preview reproduces
steps/final_1.png from scene.json, and the full train.rs schedule trains a model whose
final preview is at least as close to the true scene as the reference's own final_1.png."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import DANGO, GOLDEN, gpu_available, load_png

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    if not gpu_available():
        pytest.skip("no GPU")
    from burn_raymarching_amd import host
    host.lib()
    return host


def _psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return 10 * np.log10(255.0 ** 2 / mse)


def test_generate_reproduces_reference_targets(H, tmp_path):
    H.generate(str(tmp_path), prefix="data/")
    assert open(tmp_path / "cameras.json", "rb").read() == open(os.path.join(GOLDEN, "cameras.json"), "rb").read()
    for v in range(10):
        ours = load_png(str(tmp_path / f"target_{v}.png")).astype(int)
        ref = load_png(os.path.join(GOLDEN, f"target_{v}.png")).astype(int)
        diff = np.abs(ours - ref)
        assert diff.max() <= 1 and (diff > 0).sum() <= 64, (v, diff.max(), (diff > 0).sum())


def test_preview_reproduces_final_1(H, tmp_path):
    out = str(tmp_path / "final_1.png")
    H.preview(os.path.join(GOLDEN, "scene.json"), out, radius_offset=0.01)
    diff = np.abs(load_png(out).astype(int) - load_png(os.path.join(GOLDEN, "final_1.png")).astype(int))
    assert diff.max() <= 1 and (diff > 0).sum() <= 16


def _truth_final_view():
    """The generate.rs scene seen from the preview camera (train.rs:37-44), via the GPU renderer."""
    import torch
    from burn_raymarching_amd import render as R
    from oracle import oracle as orc
    dev = torch.device("cuda:0")
    t = [torch.tensor(DANGO[k], device=dev) for k in ("centers", "colors", "radius")]
    img = R.render_camera([([0.0, 0.0, -2.5], [0.0, 0.0, 0.0], 50.0)], 256, 256, *t).cpu().numpy()
    return orc.to_png_bytes(img).reshape(256, 256, 3)


def test_full_training_schedule_matches_reference_quality(H, tmp_path):
    """train.rs end to end (5 stages x 700 steps, batch 16384) on the reference's own targets.

    The outcome of one run is chaotic (prune/split decisions): over 32 seeds the final_1 PSNR
    against the true scene spans 26-35 dB with median 32.3 dB, the reference's own single run
    (final_1.png) sits at 32.5 dB. So 12 seeds are trained and judged as a distribution."""
    truth = _truth_final_view()
    p_ref = _psnr(load_png(os.path.join(GOLDEN, "final_1.png")), truth)
    vals = []
    for seed in range(12):
        out = tmp_path / f"s{seed}"
        cfg = H.train_config(cameras_json=os.path.join(GOLDEN, "cameras.json"), out_dir=str(out), log_every=0,
                             seed=seed, previews=1 if seed == 0 else 0)
        res, raw = H.train(cfg)
        assert res.steps == 3500
        assert np.isfinite(raw).all() and np.isfinite(res.final_loss)
        sc = H.scene_load(str(out / "scene.json"))
        assert sc["num_spheres"] == res.num_spheres and res.num_spheres >= 3
        if seed == 0:
            for s in range(4):
                assert os.path.exists(out / "steps" / f"stage_{s}.png")
            assert os.path.exists(out / "steps" / "final_1.png")
        H.preview(str(out / "scene.json"), str(out / "final.png"))  # the exported scene renders the same view
        vals.append(_psnr(load_png(str(out / "final.png")), truth))
    print(f"final_1 PSNR vs truth over 12 seeds: median {np.median(vals):.2f} dB, max {max(vals):.2f} dB; "
          f"reference run {p_ref:.2f} dB")
    assert np.median(vals) >= p_ref - 3.5
    assert max(vals) >= p_ref - 0.5


def test_cli_generate_then_train(H, tmp_path):
    from burn_raymarching_amd import _build
    exe = os.path.join(_build.LIBDIR, "rm_train")
    data = tmp_path / "data"
    subprocess.run([exe, "generate", "--out", str(data), "--prefix", "", "--size", "64x64"], check=True, timeout=120)
    cams = json.load(open(data / "cameras.json"))
    assert [c["file"] for c in cams] == [f"target_{i}.png" for i in range(10)]
    r = subprocess.run([exe, "train", "--cameras", str(data / "cameras.json"), "--out", str(tmp_path / "run"),
                        "--size", "64x64", "--stages", "2", "--steps", "40", "--batch", "2048", "--log-every", "20"],
                       check=True, timeout=300, capture_output=True, text=True)
    assert "Step 40 | Loss:" in r.stdout
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    assert summary["steps"] == 80 and np.isfinite(summary["final_loss"])
    assert os.path.exists(tmp_path / "run" / "scene.json")
    bad = subprocess.run([exe, "train", "--cameras", str(tmp_path / "missing.json")], capture_output=True, text=True,
                         timeout=60)
    assert bad.returncode == 1 and "cannot read" in bad.stderr


def test_gather_rays_matches_indexing():
    """rm_gather_rays (dataset.rs:75-79) == numpy fancy indexing; out-of-range rows are zero."""
    if not gpu_available():
        pytest.skip("no GPU")
    import ctypes
    import torch
    from burn_raymarching_amd import render as R
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    src = [torch.randn(5000, 3, generator=g) for _ in range(3)]
    idx = torch.randint(0, 5000, (777,), generator=g, dtype=torch.int32)
    idx[5] = 5000
    idx[9] = -1
    d_src = [s.to(dev) for s in src]
    d_idx = idx.to(dev)
    outs = [torch.full((777, 3), 7.0, device=dev) for _ in range(3)]
    ctx = R.context(dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    ctx.check(ctx._lib.rm_gather_rays(ctx.handle, *map(p, d_src), 5000, p(d_idx), 777, *map(p, outs)), "gather")
    ok = (idx >= 0) & (idx < 5000)
    for s, o in zip(src, outs):
        o = o.cpu()
        assert torch.equal(o[ok], s[idx[ok].long()])
        assert not o[~ok].any()


def test_zeroed_config_trains_the_reference_rule(H):
    """a zero-initialised rmh_train_config (a binding that fills only the fields it
    knows and never calls rmh_train_config_default) trains with the reference split rule
    (training.rs:185-188) -- bit for bit the default config's run -- and growth needs the explicit
    negative knobs (rm_train --split-all)."""
    # a small learning rate: no sphere moves the reference's 0.05 (training.rs:188), so the reference
    # rule splits none and split-all splits every one
    kw = dict(cameras_json=os.path.join(GOLDEN, "cameras.json"), out_dir=None, log_every=0, previews=0, stages=3,
              steps_per_stage=30, batch=4096, seed=5, base_lr=0.001)
    ref = H.train_config(**kw)
    zero = H.RmhTrainConfig()  # every field 0 / NULL
    for f in ("cameras_json", "width", "height", "stages", "steps_per_stage", "batch", "march_steps", "max_smooth",
              "base_lr", "weight_decay", "seed", "device"):
        setattr(zero, f, getattr(ref, f))
    assert zero.split_scale == 0.0 and zero.split_move == 0.0 and zero.max_spheres == 0
    r1, raw1 = H.train(ref)
    r2, raw2 = H.train(zero)
    assert r1.num_spheres == r2.num_spheres and np.array_equal(raw1, raw2)
    r3, _ = H.train(H.train_config(**kw, split_scale=-1.0, split_move=-1.0))
    assert r3.num_spheres > r1.num_spheres
