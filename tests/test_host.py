"""CPU tests of librm_host.so (include/rm_host.h): the reference's host programs in C++.
File formats are pinned byte-for-byte by the reference's own files (cameras.json and
scene.json as serde_json wrote them, the PNGs as the `image` crate wrote them); the camera
rays by the oracle; dataset.rs / training.rs:87-238 logic by restatements in the tests."""
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, load_png

HEADER = os.path.join(ROOT, "include", "rm_host.h")


@pytest.fixture(scope="module")
def H():
    from burn_raymarching_amd import _build, host
    _build.build_host()
    return host


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(rmh_[a-z0-9_]+)\s*\(", text)))


def test_host_lib_exports_every_header_symbol(H):
    import ctypes
    lib = ctypes.CDLL(H._LIB_PATH)
    assert not [f for f in header_functions() if not hasattr(lib, f)]
    assert sorted(H.SIGNATURES) == header_functions()


# ---- util.rs -------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["target_0.png", "target_9.png", "final_1.png"])
def test_png_read_matches_pil(H, name):
    path = os.path.join(GOLDEN, name)
    assert np.array_equal(H.png_read(path), load_png(path))


def test_png_write_roundtrip(H, tmp_path):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)
    p = str(tmp_path / "sub" / "dir" / "x.png")  # parent dirs created like util.rs:14-18
    H.png_write(p, img)
    assert np.array_equal(load_png(p), img)
    assert np.array_equal(H.png_read(p), img)


def test_png_reader_handles_other_colour_types_and_filters(H, tmp_path):
    from PIL import Image
    rng = np.random.default_rng(1)
    rgb = (np.add.outer(np.arange(20), np.arange(30))[..., None] * [3, 5, 7] % 256).astype(np.uint8)
    for mode in ("RGBA", "L", "LA", "P"):
        im = Image.fromarray(rgb).convert(mode)
        p = str(tmp_path / f"{mode}.png")
        im.save(p, optimize=True)  # PIL picks adaptive filters per row
        assert np.array_equal(H.png_read(p), np.asarray(im.convert("RGB"))), mode
    noise = rng.integers(0, 256, (17, 19, 3), dtype=np.uint8)
    p = str(tmp_path / "noise.png")
    Image.fromarray(noise).save(p, compress_level=9)
    assert np.array_equal(H.png_read(p), noise)


def test_png_errors(H, tmp_path):
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"not a png")
    with pytest.raises(H.HostError, match="RMH_ERR_FORMAT"):
        H.png_read(str(bad))
    with pytest.raises(H.HostError, match="RMH_ERR_IO"):
        H.png_read(str(tmp_path / "missing.png"))


def test_gamma_conversions_match_util_rs(H, oracle):
    px = np.arange(256, dtype=np.uint8)
    lin = H.srgb8_to_linear(px)
    ref = np.power(px.astype(np.float32) / np.float32(255.0), np.float32(2.2))
    assert np.max(np.abs(lin - ref) / np.maximum(ref, 1e-30)) < 2e-7
    x = np.concatenate([np.linspace(-0.5, 1.5, 4001, dtype=np.float32), [np.nan, np.inf, -np.inf]]).astype(np.float32)
    assert np.array_equal(H.linear_to_srgb8(x), oracle.to_png_bytes(x))
    # load -> save of a reference PNG is lossless (the 2.2 gamma round trip is exact on 8-bit)
    t = H.image_load(os.path.join(GOLDEN, "target_3.png"))
    assert np.array_equal(H.linear_to_srgb8(t).reshape(256, 256, 3), load_png(os.path.join(GOLDEN, "target_3.png")))


# ---- camera.rs -----------------------------------------------------------------------------
def test_camera_rays_bitwise_equal_oracle(H, oracle):
    cams = json.load(open(os.path.join(GOLDEN, "cameras.json")))
    views = [(c["origin"], c["target"], c["fov"]) for c in cams] + [([0.0, 0.0, -2.5], [0.0, 0.0, 0.0], 50.0)]
    for (w, h) in ((64, 64), (96, 40)):
        for eye, tgt, fov in views:
            o, d = H.camera_rays(w, h, eye, tgt, fov)
            ro, rd = oracle.camera_rays(w, h, eye, tgt, fov)
            assert np.array_equal(o, ro) and np.array_equal(d, rd)


# ---- JSON files ----------------------------------------------------------------------------
def test_cameras_json_roundtrip_is_byte_identical(H, tmp_path):
    path = os.path.join(GOLDEN, "cameras.json")
    cams = H.cameras_load(path)
    ref = json.load(open(path))
    assert [c["file"] for c in cams] == [c["file"] for c in ref]
    for c, r in zip(cams, ref):
        assert np.array_equal(np.float32(c["origin"]), np.float32(r["origin"]))
        assert np.float32(c["fov"]) == np.float32(r["fov"])
    out = str(tmp_path / "cameras.json")
    H.cameras_save(out, cams)
    assert open(out, "rb").read() == open(path, "rb").read()  # serde_json pretty + ryu layout


def test_scene_json_roundtrip_is_byte_identical(H, tmp_path):
    path = os.path.join(GOLDEN, "scene.json")
    sc = H.scene_load(path)
    ref = json.load(open(path))
    assert sc["num_spheres"] == ref["num_spheres"] == 6
    assert np.array_equal(sc["centers"].reshape(-1), np.float32(ref["centers"]))
    out = str(tmp_path / "scene.json")
    H.scene_save(out, sc["centers"], sc["colors"], sc["radii"], sc["light_dir"], sc["ambient_intensity"])
    assert open(out, "rb").read() == open(path, "rb").read()


@pytest.mark.parametrize("x", [1e-7, 1.5e-7, 1e-6, 1e-5, 0.1, 1.0, 100.0, 1e13, 1.2e13, 3.4e38, -2.5, 1.4e-45,
                               123456.79, 0.30000001])
def test_f32_formatting_roundtrips(H, tmp_path, x):
    out = str(tmp_path / "s.json")
    H.scene_save(out, [[x, -x, 0.0]], [[0.5, 0.5, 0.5]], [x], [x, 0.0, 1.0], [0.2])
    text = open(out).read()
    back = json.loads(text)
    assert np.float32(back["centers"][0]) == np.float32(x)
    assert np.float32(back["radii"][0]) == np.float32(x)
    v = re.search(r'"radii": \[\n    ([^\n]+)\n', text).group(1)
    short = abs(float(str(np.float32(x))))  # the shortest round-trip decimal of the f32
    assert ("e" in v) == (short < 1e-6 or short >= 1e13), v  # ryu's f32 layout switch points


def test_json_errors(H, tmp_path):
    p = tmp_path / "c.json"
    p.write_text('[{"file": "a.png", "origin": [0, 0], "target": [0, 0, 0], "fov": 50}]')
    with pytest.raises(H.HostError, match="RMH_ERR_FORMAT"):
        H.cameras_load(str(p))
    p.write_text('[{"file": "a.png", ')
    with pytest.raises(H.HostError, match="RMH_ERR_FORMAT"):
        H.cameras_load(str(p))


# ---- dataset.rs ----------------------------------------------------------------------------
def _golden_targets(H):
    cams = json.load(open(os.path.join(GOLDEN, "cameras.json")))
    return np.concatenate([H.image_load(os.path.join(GOLDEN, os.path.basename(c["file"]))) for c in cams])


def test_dataset_split_matches_dataset_rs(H):
    t = _golden_targets(H)
    ds = H.Dataset(t)
    fg_mask = (t[:, 0] + t[:, 1] + t[:, 2]) > np.float32(0.05)  # dataset.rs:28-33 (f32 sum, left to right)
    assert ds.counts() == (int(fg_mask.sum()), int((~fg_mask).sum()))


@pytest.mark.parametrize("ratio", [0.8, 0.6, 0.4, 0.0, 1.0])
def test_dataset_sample_layout(H, ratio):
    t = _golden_targets(H)
    fg_mask = (t[:, 0] + t[:, 1] + t[:, 2]) > np.float32(0.05)
    ds = H.Dataset(t)
    idx = ds.sample(16384, ratio, H.Rng(7))
    n_uni = int(np.float32(16384) * np.float32(ratio))
    assert idx.shape == (16384,)
    assert idx.min() >= 0 and idx.max() < t.shape[0]
    assert fg_mask[idx[n_uni:]].all()  # the boost part is foreground only (dataset.rs:67-72)
    if n_uni > 1000:  # the uniform part sees the fg fraction of the whole set
        frac = fg_mask[idx[:n_uni]].mean()
        assert abs(frac - fg_mask.mean()) < 5 * np.sqrt(fg_mask.mean() * (1 - fg_mask.mean()) / n_uni)


def test_dataset_small_foreground_and_none(H):
    t = np.zeros((1000, 3), np.float32)
    t[[3, 500, 999]] = 1.0
    ds = H.Dataset(t)
    assert ds.counts() == (3, 997)
    idx = ds.sample(100, 0.5, H.Rng(1))  # fg (3) < 50 boost draws -> 3 fg draws, 97 uniform
    assert idx.shape == (100,) and set(idx[97:]) <= {3, 500, 999}
    empty = H.Dataset(np.zeros((64, 3), np.float32))
    assert empty.sample(10, 0.5, H.Rng(1)).shape == (5,)  # no foreground: the boost part is skipped


def test_sample_count_rule_and_foreground_list(H):
    """The count rule shared by the host sampler, the device sampler and the driver's global ray
    count (dataset.rs:54-67), and the foreground list the device sampler draws from."""
    t = _golden_targets(H)
    ds = H.Dataset(t)
    fg_mask = (t[:, 0] + t[:, 1] + t[:, 2]) > np.float32(0.05)
    assert np.array_equal(ds.foreground(), np.flatnonzero(fg_mask).astype(np.int32))
    for ratio in (0.8, 0.4, 0.0, 1.0):
        nu, nf = ds.sample_count(16384, ratio)
        assert nu == int(np.float32(16384) * np.float32(ratio)) and nu + nf == 16384
        assert ds.sample(16384, ratio, H.Rng(2)).shape == (nu + nf,)
    tt = np.zeros((100, 3), np.float32)
    tt[:3] = 1.0
    small = H.Dataset(tt)
    assert small.sample_count(100, 0.5) == (97, 3)  # fg (3) < 50: the boost shrinks to |fg|
    empty = H.Dataset(np.zeros((64, 3), np.float32))
    assert empty.sample_count(10, 0.5) == (5, 0) and empty.foreground().size == 0


def test_sampler_is_seeded(H):
    t = _golden_targets(H)
    ds = H.Dataset(t)
    a = ds.sample(4096, 0.7, H.Rng(3))
    b = ds.sample(4096, 0.7, H.Rng(3))
    c = ds.sample(4096, 0.7, H.Rng(4))
    assert np.array_equal(a, b) and not np.array_equal(a, c)


def test_rng_ranges(H):
    r = H.Rng(11)
    v = np.array([r.below(10) for _ in range(20000)])
    assert v.min() == 0 and v.max() == 9 and abs(np.bincount(v).std() / 2000) < 0.05
    u = np.array([r.uniform(-1.0, 1.0) for _ in range(20000)])
    assert u.min() >= -1.0 and u.max() < 1.0 and abs(u.mean()) < 0.03


# ---- training.rs:87-238 --------------------------------------------------------------------
def _sp(x):
    x = np.float32(x)
    return np.float32(np.log(np.float32(1.0) + np.exp(x, dtype=np.float32), dtype=np.float32))


def _sig(x):
    return np.float32(np.float32(1.0) / (np.float32(1.0) + np.exp(-np.float32(x), dtype=np.float32)))


def _pack(c, col, r, ld=(0.0, 1.0, 0.0), amb=-1.4):
    return np.concatenate([np.float32(c).reshape(-1), np.float32(col).reshape(-1), np.float32(r).reshape(-1),
                           np.float32(ld), [np.float32(amb)]]).astype(np.float32)


def test_initial_model(H):
    raw = H.initial_model()
    M = 7
    c = raw[:21].reshape(7, 3)
    assert np.array_equal(c[:6], np.float32([[.1, 0, 0], [-.1, 0, 0], [0, .1, 0], [0, -.1, 0], [0, 0, .1], [0, 0, -.1]]))
    assert np.array_equal(c[6], [0, 0, 0])
    assert not raw[3 * M:7 * M].any()
    assert np.array_equal(raw[7 * M:], np.float32([0, 1, 0, -1.4]))


def test_prune_rules(H):
    # sphere: 0 keep, 1 too big (r > 1 - 0.04 stage), 2 too small (r < 0.005), 3 too far (|c|^2 > 1.44),
    # 4 black (sum sigmoid < 0.05), 5 keep (moved little)
    stage = 2
    big = np.log(np.expm1(np.float32(0.95)))
    tiny = np.log(np.expm1(np.float32(0.004)))
    r = np.float32([-3.0, big, tiny, -3.0, -3.0, -3.0])
    c = np.float32([[0.1, 0, 0], [0, 0.2, 0], [0, 0, 0.3], [1.3, 0, 0], [0, 0, 0], [0.2, 0.2, 0.2]])
    col = np.zeros((6, 3), np.float32)
    col[4] = -6.0
    raw = _pack(c, col, r)
    out, m = H.prune_and_split(raw, 6, c, stage, 5, H.Rng(0))
    assert m == 2
    assert np.array_equal(out[:6].reshape(2, 3), c[[0, 5]])
    assert np.array_equal(out[12:14], r[[0, 5]])
    assert np.array_equal(out[-4:], raw[-4:])  # light_dir, ambient carried over


def test_split_rule(H):
    stage, stages = 1, 5
    thr = np.float32(0.25) * np.float32(0.65) ** 1
    r_raw = np.float32(np.log(np.expm1(np.float32(0.3))))  # softplus = 0.3 > thr
    c0 = np.float32([[0.0, 0.0, 0.0], [0.0, 0.0, 0.0], [0.5, 0.0, 0.0]])
    c = np.float32([[0.2, 0.1, 0.0], [0.01, 0.0, 0.0], [0.5, 0.0, 0.0]])  # moved, barely moved, not moved
    col = np.float32([[1, 2, 3], [0, 0, 0], [-1, 0, 1]])
    raw = _pack(c, col, [r_raw, r_raw, r_raw])
    out, m = H.prune_and_split(raw, 3, c0, stage, stages, H.Rng(5))
    assert _sp(r_raw) > thr
    assert m == 4  # sphere 0 split, 1 and 2 kept
    cen = out[:12].reshape(4, 3)
    r = _sp(r_raw)
    mid = (cen[0] + cen[1]) / 2
    assert np.allclose(mid, c[0], atol=1e-6)
    assert np.isclose(np.linalg.norm(cen[0] - c[0]), r * 0.5, rtol=1e-5)
    assert np.array_equal(out[12:24].reshape(4, 3), col[[0, 0, 1, 2]])
    new_raw = np.log(np.maximum(np.expm1(np.maximum(r * np.float32(0.8), np.float32(0.01))), 1e-6))
    assert np.allclose(out[24:26], new_raw, rtol=1e-5)
    assert np.array_equal(out[26:28], [r_raw, r_raw])
    # the last stage never splits (training.rs:183)
    _, m_last = H.prune_and_split(raw, 3, c0, stages - 1, stages, H.Rng(5))
    assert m_last == 3


def test_prune_everything_is_an_error(H):
    raw = _pack([[5.0, 0, 0]], [[0, 0, 0]], [-3.0])
    with pytest.raises(H.HostError, match="every sphere"):
        H.prune_and_split(raw, 1, [[5.0, 0, 0]], 0, 5, H.Rng(0))


def test_split_knobs(H):
    """rmh_prune_and_split_ex: (1, 0.05) is the reference rule bit for bit; (0, 0) splits every
    surviving sphere; the pruning rules stay."""
    stage, stages = 1, 5
    r_raw = np.float32(np.log(np.expm1(np.float32(0.05))))  # softplus 0.05 < 0.25 * 0.65
    c0 = np.float32([[0.0, 0.0, 0.0], [0.0, 0.0, 0.0], [1.3, 0.0, 0.0]])
    c = np.float32([[0.2, 0.1, 0.0], [0.0, 0.0, 0.0], [1.3, 0.0, 0.0]])  # moved, not moved, pruned (far)
    raw = _pack(c, np.ones((3, 3), np.float32), [r_raw, r_raw, r_raw])
    ref, m_ref = H.prune_and_split(raw, 3, c0, stage, stages, H.Rng(7))
    same, m_same = H.prune_and_split(raw, 3, c0, stage, stages, H.Rng(7), split_scale=1.0, split_move=0.05)
    assert m_ref == m_same == 2 and np.array_equal(ref, same)  # nothing splits under the reference rule
    out, m = H.prune_and_split(raw, 3, c0, stage, stages, H.Rng(7), split_scale=0.0, split_move=0.0)
    assert m == 3  # sphere 0 split (moved), sphere 1 kept (move 0 is not > 0), sphere 2 pruned
    out, m = H.prune_and_split(raw, 3, c0, stage, stages, H.Rng(7), split_scale=0.1, split_move=0.0)
    assert m == 3  # 0.05 > 0.1 * 0.1625
    _, m_last = H.prune_and_split(raw, 3, c0, stages - 1, stages, H.Rng(7), split_scale=0.0, split_move=0.0)
    assert m_last == 2  # the last stage never splits
    with pytest.raises(H.HostError):
        H.prune_and_split(raw, 3, c0, stage, stages, H.Rng(7), split_scale=-1.0, split_move=0.0)
    # the cap: six moved spheres that would all split; at most 9 in the next generation
    c6 = np.float32([[0.1 * i, 0.05, 0.0] for i in range(6)])
    raw6 = _pack(c6, np.ones((6, 3), np.float32), [r_raw] * 6)
    z6 = np.zeros((6, 3), np.float32)
    out, m = H.prune_and_split(raw6, 6, z6, stage, stages, H.Rng(7), split_scale=0.0, split_move=0.0)
    assert m == 12
    out, m = H.prune_and_split(raw6, 6, z6, stage, stages, H.Rng(7), split_scale=0.0, split_move=0.0, max_spheres=9)
    assert m == 9  # the first three split (2 + 2 + 2 + 3 kept), in order
    assert np.array_equal(out[18:27].reshape(3, 3), c6[3:])


# ---- the RCCL id rendezvous (rmh_rendezvous_*, used by rmh_collective_rccl_create) -----------
def test_rendezvous_late_reader(H, tmp_path):
    """A rank that starts (or finishes its HIP init) long after rank 0 published the id still
    takes it: no clock is involved (the former mtime check rejected it)."""
    import threading
    import time
    path = str(tmp_path / "id")
    blob = bytes(range(128))
    H.rendezvous_publish(path, "run-A", blob)
    time.sleep(2.5)
    assert H.rendezvous_read(path, "run-A", len(blob), 5.0) == blob
    # a reader that starts before the file exists waits for it
    got = {}
    t = threading.Thread(target=lambda: got.setdefault("b", H.rendezvous_read(path + "2", "run-B", 16, 10.0)))
    t.start()
    time.sleep(0.5)
    H.rendezvous_publish(path + "2", "run-B", b"x" * 16)
    t.join()
    assert got["b"] == b"x" * 16


def test_rendezvous_rejects_other_runs_file(H, tmp_path):
    path = str(tmp_path / "id")
    H.rendezvous_publish(path, "old-run", b"y" * 16)
    with pytest.raises(H.HostError, match="run id 'old-run', expected 'new-run'"):
        H.rendezvous_read(path, "new-run", 16, 0.3)
    with pytest.raises(H.HostError, match="wrong payload size"):
        H.rendezvous_read(path, "old-run", 8, 0.3)
    # the environment supplies the run id when the argument is NULL
    os.environ["RMH_RUN_ID"] = "old-run"
    try:
        assert H.rendezvous_read(path, None, 16, 1.0) == b"y" * 16
    finally:
        del os.environ["RMH_RUN_ID"]


def test_rendezvous_refuses_unnamed_runs(H, tmp_path, monkeypatch):
    """with an empty run id, or torchrun's default 'none', a file a crashed run left at
    the same path would pass for this run's and a late rank would join a dead ncclUniqueId. The
    rendezvous refuses such ids on both sides, and rmh_collective_rccl_create refuses them for
    world > 1 before any GPU call (so this runs on the CPU)."""
    path = str(tmp_path / "id")
    monkeypatch.delenv("RMH_RUN_ID", raising=False)
    monkeypatch.delenv("TORCHELASTIC_RUN_ID", raising=False)
    with pytest.raises(H.HostError, match="needs a run id"):
        H.rendezvous_publish(path, None, b"z" * 16)
    with pytest.raises(H.HostError, match="needs a run id"):
        H.rendezvous_publish(path, "", b"z" * 16)
    H.rendezvous_publish(path, "crashed-run", b"z" * 16)  # a stale file of an earlier run
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    with pytest.raises(H.HostError, match="needs a run id"):
        H.rendezvous_read(path, None, 16, 0.2)
    with pytest.raises(H.HostError, match="rank 1: .*needs a run id"):
        H.rccl_collective(1, 2, 0, path)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "crashed-run")  # an id that names the run is taken
    assert H.rendezvous_read(path, None, 16, 1.0) == b"z" * 16
