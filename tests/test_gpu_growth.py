"""BASELINE configs[4] as stated -- "4096 spheres after adaptive split/prune, 128 steps, fp16 color /
fp32 SDF" -- grown through prune_and_split (training.rs:87-238, train.rs:306-328) by the C++
driver, at a reduced size:

  * rmh_train on the reference's own targets (tests/golden: data/cameras.json + target PNGs) with
    128 march steps, fp16 colours and the growth knobs split_scale = split_move = -1 (every sphere
    that survives pruning splits; rmh_prune_and_split_ex): the model grows 7 -> 14 -> ... past 32,
    256 and 512 spheres, so the run itself crosses the small -> general kernel switch (M > 32) and
    the split-march thresholds (256 / 512 spheres) at its batch of 16,384 rays, with the split
    march's continuation launch (S = 128);
  * the trained parameters of every generation (rmh_train_config.on_generation) against the fp64
    oracle: one fused train step (forward, compute_loss seed, backward) on 2,048 dataset rays, at
    the kernel the generation's size selects and, from 256 spheres, also with the split march off
    (RM_SPLIT=0: the general kernel's other variant) -- the clustered child pairs prune_and_split
    makes, not the synthetic uniform ball of the other configs[4] tests.

Tolerances: tests/conftest.py (check_grads, mode "train"); the oracle gets the fp16-rounded
colours the kernel reads.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, check_grads, gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

S, K, PROG = 128, 32.0, 0.5


@pytest.fixture(scope="module")
def grown():
    """The growth run: 8 stages x 25 steps, every generation's trained raw parameters."""
    from burn_raymarching_amd import host
    gens = []
    cfg = host.train_config(cameras_json=os.path.join(GOLDEN, "cameras.json"), out_dir=None, log_every=0, previews=0,
                            stages=8, steps_per_stage=25, march_steps=S, seed=11, split_scale=-1.0, split_move=-1.0,
                            color_f16=1)
    host.on_generation(cfg, lambda stage, m, raw: gens.append((stage, m, raw)))
    res, raw = host.train(cfg)
    return res, raw, gens


def test_growth_crosses_every_kernel_switch(grown):
    res, raw, gens = grown
    sizes = [m for _, m, _ in gens]
    assert [s for s, _, _ in gens] == list(range(8))
    assert sizes[0] == 7 and res.num_spheres == sizes[-1]
    # every generation doubles what survives pruning: 7 * 2^stage at most
    for a, b in zip(sizes, sizes[1:]):
        assert a < b <= 2 * a, sizes
    assert any(m <= 32 for m in sizes) and any(32 < m < 256 for m in sizes)
    assert any(256 <= m < 512 for m in sizes) and sizes[-1] >= 512, sizes
    assert np.isfinite(raw).all() and np.isfinite(res.final_loss)
    for _, m, r in gens:
        assert r.shape == (7 * m + 4,) and np.isfinite(r).all()


def _dataset_rays(n, seed):
    """n rays drawn from the reference's training set (the 10 cameras of cameras.json, their
    256x256 target PNGs in linear RGB)."""
    from burn_raymarching_amd import host
    cams = host.cameras_load(os.path.join(GOLDEN, "cameras.json"))
    rng = np.random.default_rng(seed)
    o, d, t = [], [], []
    for c in cams:
        oo, dd = host.camera_rays(256, 256, c["origin"], c["target"], c["fov"])
        tt = host.image_load(os.path.join(GOLDEN, os.path.basename(c["file"])))
        idx = rng.choice(256 * 256, n // len(cams), replace=False)
        o.append(oo[idx])
        d.append(dd[idx])
        t.append(tt[idx])
    return np.concatenate(o), np.concatenate(d), np.concatenate(t)


def _pick_generations(gens):
    """The last generation of at most 32 spheres (small kernel), then the first one in each of
    (32, 256) (general kernel), [256, 512) and [512, inf) (split march at this ray count)."""
    pick = [max((g for g in gens if g[1] <= 32), key=lambda g: g[1])]
    for lo, hi in ((33, 256), (256, 512), (512, 1 << 30)):
        inside = [g for g in gens if lo <= g[1] < hi]
        if inside:
            pick.append(min(inside, key=lambda g: g[1]))
    return pick


def test_each_generation_train_step_against_oracle(grown, oracle, monkeypatch):
    import torch
    from burn_raymarching_amd import model, render
    _, _, gens = grown
    o, d, t = _dataset_rays(2048, 3)
    o64, d64, t64 = (x.astype(np.float64) for x in (o, d, t))
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()  # noqa: E731
    picked = _pick_generations(gens)
    assert len(picked) == 4, [g[1] for g in gens]
    for stage, m, raw in picked:
        sm = model.SceneModel(torch.from_numpy(raw).cuda(), m, color_dtype="f16")
        scene = sm.scene()
        act = model.unpack(sm.activated_packed().cpu().numpy(), m)
        sc = {"centers": act["centers"], "radius": act["radius"], "light_dir": act["light_dir"],
              "ambient": act["ambient"], "colors": scene.colors.float().cpu().numpy()}  # the fp16 colours
        _, loss_ref, g_ref = oracle.train_step(o64, d64, t64, sc, S, K, PROG)
        variants = [None] if m < 256 else [None, "0"]
        for split_env in variants:
            if split_env is None:
                monkeypatch.delenv("RM_SPLIT", raising=False)
            else:
                monkeypatch.setenv("RM_SPLIT", split_env)
            loss, g, _ = render.train_step(dev(o), dev(d), dev(t), scene, K, PROG, S)
            got = loss.cpu().numpy()[0]
            assert abs(got - loss_ref) <= 1e-4 * abs(loss_ref), (stage, m, split_env, got, loss_ref)
            check_grads(g, g_ref, mode="train")
        monkeypatch.delenv("RM_SPLIT", raising=False)
