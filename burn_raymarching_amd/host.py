"""ctypes binding of librm_host.so (include/rm_host.h): the reference's host programs
(train.rs, generate.rs, dataset.rs, training.rs:87-238, util.rs, camera.rs) in C++.

Every header symbol has an entry in SIGNATURES; tests check the two stay in sync."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import native

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("RMH_LIB_PATH", os.path.join(_HERE, "lib", "librm_host.so"))

RMH_OK = 0
RMH_ERR_GPU = 4
_ERR_NAMES = {1: "RMH_ERR_INVALID_ARG", 2: "RMH_ERR_IO", 3: "RMH_ERR_FORMAT", 4: "RMH_ERR_GPU"}
RMH_PATH_MAX = 512


class HostError(RuntimeError):
    pass


class RmhCameraEntry(ctypes.Structure):
    _fields_ = [("file", ctypes.c_char * RMH_PATH_MAX), ("origin", ctypes.c_float * 3),
                ("target", ctypes.c_float * 3), ("fov", ctypes.c_float)]


class RmhRng(ctypes.Structure):
    _fields_ = [("state", ctypes.c_uint64), ("inc", ctypes.c_uint64)]


ALL_REDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)
BROADCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                ctypes.c_void_p)


ABORT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
WAIT_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
GENERATION_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_float))


class RmhCollective(ctypes.Structure):
    """rmh_collective: sum all-reduce and broadcast of fp32 device buffers on the driver's stream,
    the (nullable) abort a failing rank calls and the (nullable) watchdog wait on the stream."""
    _fields_ = [("state", ctypes.c_void_p), ("rank", ctypes.c_int32), ("world", ctypes.c_int32),
                ("all_reduce_sum", ALL_REDUCE_FN), ("broadcast", BROADCAST_FN), ("abort", ABORT_FN),
                ("wait", WAIT_FN)]


class RmhTrainConfig(ctypes.Structure):
    _fields_ = [("cameras_json", ctypes.c_char_p), ("out_dir", ctypes.c_char_p), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("stages", ctypes.c_int32), ("steps_per_stage", ctypes.c_int32),
                ("batch", ctypes.c_int32), ("march_steps", ctypes.c_int32), ("max_smooth", ctypes.c_float),
                ("base_lr", ctypes.c_float), ("weight_decay", ctypes.c_float), ("log_every", ctypes.c_int32),
                ("previews", ctypes.c_int32), ("seed", ctypes.c_uint64), ("device", ctypes.c_int32),
                ("comm", ctypes.POINTER(RmhCollective)), ("split_scale", ctypes.c_float),
                ("split_move", ctypes.c_float), ("max_spheres", ctypes.c_int32), ("color_f16", ctypes.c_int32), ("on_generation", GENERATION_FN),
                ("user", ctypes.c_void_p)]


class RmhTrainResult(ctypes.Structure):
    _fields_ = [("num_spheres", ctypes.c_int32), ("steps", ctypes.c_int32), ("final_loss", ctypes.c_float),
                ("seconds", ctypes.c_double), ("step_ms", ctypes.c_double)]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F = ctypes.c_float
_S = ctypes.c_char_p
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PP = ctypes.POINTER(ctypes.c_void_p)

SIGNATURES = {
    "rmh_last_error": (ctypes.c_char_p, []),
    "rmh_free": (None, [_P]),
    "rmh_png_read": (ctypes.c_int, [_S, _PI32, _PI32, _PP]),
    "rmh_png_write": (ctypes.c_int, [_S, _P, _I32, _I32]),
    "rmh_srgb8_to_linear": (None, [_P, _I64, _P]),
    "rmh_linear_to_srgb8": (None, [_P, _I64, _P]),
    "rmh_image_load": (ctypes.c_int, [_S, _PI32, _PI32, _PP]),
    "rmh_image_save": (ctypes.c_int, [_S, _P, _I32, _I32]),
    "rmh_camera_rays": (None, [_I32, _I32, _P, _P, _F, _P, _P]),
    "rmh_cameras_load": (ctypes.c_int, [_S, ctypes.POINTER(ctypes.POINTER(RmhCameraEntry)), _PI32]),
    "rmh_cameras_save": (ctypes.c_int, [_S, ctypes.POINTER(RmhCameraEntry), _I32]),
    "rmh_scene_save": (ctypes.c_int, [_S, _I32, _P, _P, _P, _P, _P]),
    "rmh_scene_load": (ctypes.c_int, [_S, _PI32, _PP, _PP, _PP, _P, _P]),
    "rmh_rng_seed": (None, [ctypes.POINTER(RmhRng), ctypes.c_uint64, ctypes.c_uint64]),
    "rmh_rng_u32": (ctypes.c_uint32, [ctypes.POINTER(RmhRng)]),
    "rmh_rng_below": (ctypes.c_uint32, [ctypes.POINTER(RmhRng), ctypes.c_uint32]),
    "rmh_rng_uniform": (ctypes.c_float, [ctypes.POINTER(RmhRng), _F, _F]),
    "rmh_dataset_create": (ctypes.c_int, [_P, _I64, _PP]),
    "rmh_dataset_destroy": (None, [_P]),
    "rmh_dataset_counts": (None, [_P, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "rmh_dataset_sample": (ctypes.c_int, [_P, _I32, _F, ctypes.POINTER(RmhRng), _P, _PI32]),
    "rmh_dataset_sample_count": (None, [_P, _I32, _F, ctypes.POINTER(_I64), ctypes.POINTER(_I64)]),
    "rmh_dataset_fg": (None, [_P, ctypes.POINTER(_PI32), ctypes.POINTER(_I64)]),
    "rmh_prune_and_split": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, ctypes.POINTER(RmhRng), _P, _PI32]),
    "rmh_prune_and_split_ex": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _F, _F, _I32, ctypes.POINTER(RmhRng), _P,
                                              _PI32]),
    "rmh_initial_model": (None, [_P]),
    "rmh_collective_rccl_create": (ctypes.c_int, [_I32, _I32, _I32, _S, _S, ctypes.c_double,
                                                  ctypes.POINTER(RmhCollective)]),
    "rmh_rendezvous_publish": (ctypes.c_int, [_S, _S, _P, _I64]),
    "rmh_rendezvous_read": (ctypes.c_int, [_S, _S, _P, _I64, ctypes.c_double]),
    "rmh_collective_rccl_destroy": (None, [ctypes.POINTER(RmhCollective)]),
    "rmh_train_config_default": (None, [ctypes.POINTER(RmhTrainConfig)]),
    "rmh_train": (ctypes.c_int, [ctypes.POINTER(RmhTrainConfig), ctypes.POINTER(RmhTrainResult), _P, _I32]),
    "rmh_preview": (ctypes.c_int, [_S, _S, _I32, _I32, _P, _P, _F, _F, _I32]),
    "rmh_generate": (ctypes.c_int, [_S, _S, _I32, _I32, _I32]),
    "rmh_version": (ctypes.c_char_p, []),
}

_lib = None


def lib():
    """Load librm_host.so (which pulls in libraymarch_hip.so); raise if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise HostError(f"{_LIB_PATH} is missing: run `python -m burn_raymarching_amd._build`")
        native.lib()  # libraymarch_hip.so first (librm_host.so links it)
        h = ctypes.CDLL(_LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        _lib = h
    return _lib


def _check(rc, what):
    if rc != RMH_OK:
        raise HostError(f"{what} failed with {_ERR_NAMES.get(rc, rc)}: {lib().rmh_last_error().decode()}")


def _f32c(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if shape is not None:
        a = a.reshape(shape)
    return a


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _b(s):
    return os.fsencode(s)


def _take(ptr, n, dtype):
    """Copy n elements out of a malloc'd buffer and free it."""
    try:
        if n == 0:
            return np.zeros(0, dtype)
        buf = (ctypes.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr.value)
        return np.frombuffer(bytes(buf), dtype=dtype).copy()
    finally:
        lib().rmh_free(ptr)


# ---- util.rs ----------------------------------------------------------------------------
def png_read(path) -> np.ndarray:
    w, h, p = _I32(), _I32(), _P()
    _check(lib().rmh_png_read(_b(path), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)), "rmh_png_read")
    return _take(p, w.value * h.value * 3, np.uint8).reshape(h.value, w.value, 3)


def png_write(path, rgb: np.ndarray) -> None:
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    if rgb.ndim != 3 or rgb.shape[2] != 3:
        raise ValueError("rgb must be [h, w, 3] uint8")
    _check(lib().rmh_png_write(_b(path), _p(rgb), rgb.shape[1], rgb.shape[0]), "rmh_png_write")


def srgb8_to_linear(px: np.ndarray) -> np.ndarray:
    px = np.ascontiguousarray(px, dtype=np.uint8)
    out = np.empty(px.shape, np.float32)
    lib().rmh_srgb8_to_linear(_p(px), px.size, _p(out))
    return out


def linear_to_srgb8(x: np.ndarray) -> np.ndarray:
    x = _f32c(x)
    out = np.empty(x.shape, np.uint8)
    lib().rmh_linear_to_srgb8(_p(x), x.size, _p(out))
    return out


def image_load(path) -> np.ndarray:
    w, h, p = _I32(), _I32(), _P()
    _check(lib().rmh_image_load(_b(path), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p)), "rmh_image_load")
    return _take(p, w.value * h.value * 3, np.float32).reshape(h.value * w.value, 3)


def image_save(path, linear: np.ndarray, width: int, height: int) -> None:
    linear = _f32c(linear, (height * width, 3))
    _check(lib().rmh_image_save(_b(path), _p(linear), width, height), "rmh_image_save")


# ---- camera.rs ----------------------------------------------------------------------------
def camera_rays(width, height, eye, target, fov_deg):
    eye = _f32c(eye, (3,))
    target = _f32c(target, (3,))
    o = np.empty((width * height, 3), np.float32)
    d = np.empty((width * height, 3), np.float32)
    lib().rmh_camera_rays(width, height, _p(eye), _p(target), float(fov_deg), _p(o), _p(d))
    return o, d


# ---- JSON files ---------------------------------------------------------------------------
def cameras_load(path) -> list[dict]:
    p = ctypes.POINTER(RmhCameraEntry)()
    n = _I32()
    _check(lib().rmh_cameras_load(_b(path), ctypes.byref(p), ctypes.byref(n)), "rmh_cameras_load")
    try:
        return [{"file": p[i].file.decode(), "origin": list(p[i].origin), "target": list(p[i].target),
                 "fov": p[i].fov} for i in range(n.value)]
    finally:
        lib().rmh_free(ctypes.cast(p, ctypes.c_void_p))


def cameras_save(path, cams: list[dict]) -> None:
    arr = (RmhCameraEntry * max(1, len(cams)))()
    for i, c in enumerate(cams):
        arr[i].file = c["file"].encode()
        arr[i].origin = (ctypes.c_float * 3)(*c["origin"])
        arr[i].target = (ctypes.c_float * 3)(*c["target"])
        arr[i].fov = c["fov"]
    _check(lib().rmh_cameras_save(_b(path), arr, len(cams)), "rmh_cameras_save")


def scene_save(path, centers, colors, radii, light_dir, ambient) -> None:
    c = _f32c(centers).reshape(-1)
    m = c.size // 3
    col = _f32c(colors).reshape(-1)
    r = _f32c(radii).reshape(-1)
    ld = _f32c(light_dir, (3,))
    amb = _f32c(ambient).reshape(-1)[:1]
    _check(lib().rmh_scene_save(_b(path), m, _p(c), _p(col), _p(r), _p(ld), _p(amb)), "rmh_scene_save")


def scene_load(path) -> dict:
    m = _I32()
    pc, pcol, pr = _P(), _P(), _P()
    ld = np.zeros(3, np.float32)
    amb = np.zeros(1, np.float32)
    _check(lib().rmh_scene_load(_b(path), ctypes.byref(m), ctypes.byref(pc), ctypes.byref(pcol), ctypes.byref(pr),
                                _p(ld), _p(amb)), "rmh_scene_load")
    M = m.value
    return {"num_spheres": M, "centers": _take(pc, 3 * M, np.float32).reshape(M, 3),
            "colors": _take(pcol, 3 * M, np.float32).reshape(M, 3), "radii": _take(pr, M, np.float32),
            "light_dir": ld, "ambient_intensity": amb}


# ---- RNG, dataset, prune_and_split ------------------------------------------------------
class Rng:
    def __init__(self, seed: int, stream: int = 0):
        self.s = RmhRng()
        lib().rmh_rng_seed(ctypes.byref(self.s), seed, stream)

    def u32(self) -> int:
        return lib().rmh_rng_u32(ctypes.byref(self.s))

    def below(self, n: int) -> int:
        return lib().rmh_rng_below(ctypes.byref(self.s), n)

    def uniform(self, lo: float, hi: float) -> float:
        return lib().rmh_rng_uniform(ctypes.byref(self.s), lo, hi)


class Dataset:
    """SceneDataset (dataset.rs:4-82): host fg/bg split and the batch index draw."""

    def __init__(self, targets: np.ndarray):
        t = _f32c(targets).reshape(-1, 3)
        self._t = t
        self.h = _P()
        _check(lib().rmh_dataset_create(_p(t), t.shape[0], ctypes.byref(self.h)), "rmh_dataset_create")

    def counts(self):
        fg, bg = _I64(), _I64()
        lib().rmh_dataset_counts(self.h, ctypes.byref(fg), ctypes.byref(bg))
        return fg.value, bg.value

    def sample_count(self, batch: int, uniform_ratio: float):
        """(n_uniform, n_fg) of a batch (dataset.rs:54-67), the rule every sampler shares."""
        nu, nf = _I64(), _I64()
        lib().rmh_dataset_sample_count(self.h, batch, uniform_ratio, ctypes.byref(nu), ctypes.byref(nf))
        return nu.value, nf.value

    def foreground(self) -> np.ndarray:
        """The foreground pixel indices (dataset.rs:26-35), ascending."""
        ptr, n = _PI32(), _I64()
        lib().rmh_dataset_fg(self.h, ctypes.byref(ptr), ctypes.byref(n))
        return np.ctypeslib.as_array(ptr, shape=(n.value,)).copy() if n.value else np.empty(0, np.int32)

    def sample(self, batch: int, uniform_ratio: float, rng: Rng) -> np.ndarray:
        idx = np.empty(batch, np.int32)
        n = _I32()
        _check(lib().rmh_dataset_sample(self.h, batch, uniform_ratio, ctypes.byref(rng.s), _p(idx), ctypes.byref(n)),
               "rmh_dataset_sample")
        return idx[:n.value]

    def close(self):
        if self.h:
            lib().rmh_dataset_destroy(self.h)
            self.h = _P()

    __del__ = close


def prune_and_split(raw_packed, num_spheres, init_centers, stage, stages, rng: Rng, split_scale=None,
                    split_move=None, max_spheres=None):
    """training.rs:87-238; split_scale / split_move / max_spheres (rmh_prune_and_split_ex) default
    to the reference rule (1, 0.05, no cap)."""
    raw = _f32c(raw_packed).reshape(-1)
    if raw.size != 7 * num_spheres + 4:
        raise ValueError("raw_packed must hold 7M+4 floats")
    init = _f32c(init_centers).reshape(-1)
    if init.size != 3 * num_spheres:
        raise ValueError("init_centers must be [M, 3]")
    out = np.empty(14 * num_spheres + 4, np.float32)
    m = _I32()
    if split_scale is None and split_move is None and max_spheres is None:
        _check(lib().rmh_prune_and_split(_p(raw), num_spheres, _p(init), stage, stages, ctypes.byref(rng.s), _p(out),
                                         ctypes.byref(m)), "rmh_prune_and_split")
    else:
        _check(lib().rmh_prune_and_split_ex(_p(raw), num_spheres, _p(init), stage, stages,
                                            1.0 if split_scale is None else split_scale,
                                            0.05 if split_move is None else split_move, max_spheres or 0,
                                            ctypes.byref(rng.s), _p(out), ctypes.byref(m)), "rmh_prune_and_split_ex")
    return out[:7 * m.value + 4].copy(), m.value


def initial_model() -> np.ndarray:
    out = np.empty(7 * 7 + 4, np.float32)
    lib().rmh_initial_model(_p(out))
    return out


# ---- GPU-driving programs ------------------------------------------------------------------
def train_config(**kw) -> RmhTrainConfig:
    cfg = RmhTrainConfig()
    lib().rmh_train_config_default(ctypes.byref(cfg))
    for k, v in kw.items():
        if k in ("cameras_json", "out_dir"):
            v = None if v is None else _b(v)
        setattr(cfg, k, v)
    return cfg


def collective(rank: int, world: int, all_reduce_sum, broadcast, abort=None, wait=None) -> RmhCollective:
    """An rmh_collective over Python callables all_reduce_sum(dev_ptr, count, stream) and
    broadcast(dev_ptr, count, root, stream) (each returns None or raises), abort() (optional:
    called by a rank that fails after the collectives began) and wait(stream) (optional: the
    driver's stream waits; raise to fail the run). The struct keeps the callbacks alive; keep it
    alive while rmh_train runs."""
    def ar(_state, buf, count, stream):
        try:
            all_reduce_sum(buf, count, stream)
            return RMH_OK
        except Exception as e:  # noqa: BLE001 -- reported through the C status
            print(f"all_reduce_sum failed: {e!r}")
            return 4
    def bc(_state, buf, count, root, stream):
        try:
            broadcast(buf, count, root, stream)
            return RMH_OK
        except Exception as e:  # noqa: BLE001
            print(f"broadcast failed: {e!r}")
            return 4
    def ab(_state):
        try:
            abort()
        except Exception as e:  # noqa: BLE001
            print(f"abort failed: {e!r}")
    def wt(_state, stream):
        try:
            wait(stream)
            return RMH_OK
        except Exception as e:  # noqa: BLE001
            print(f"wait failed: {e!r}")
            return 4
    c = RmhCollective(None, rank, world, ALL_REDUCE_FN(ar), BROADCAST_FN(bc),
                      ABORT_FN(ab) if abort is not None else ABORT_FN(),
                      WAIT_FN(wt) if wait is not None else WAIT_FN())
    c._keep = (c.all_reduce_sum, c.broadcast, c.abort, c.wait)
    return c


def rccl_collective(rank: int, world: int, device: int, id_path: str | None, timeout_s: float = 300.0,
                    run_id: str | None = None):
    """rmh_collective_rccl_create (RCCL over xGMI, one process per GPU)."""
    c = RmhCollective()
    _check(lib().rmh_collective_rccl_create(rank, world, device, None if id_path is None else _b(id_path),
                                            None if run_id is None else run_id.encode(), float(timeout_s),
                                            ctypes.byref(c)), "rmh_collective_rccl_create")
    return c


def rendezvous_publish(path, run_id: str | None, blob: bytes) -> None:
    buf = ctypes.create_string_buffer(blob, len(blob))
    _check(lib().rmh_rendezvous_publish(_b(path), None if run_id is None else run_id.encode(), buf, len(blob)),
           "rmh_rendezvous_publish")


def rendezvous_read(path, run_id: str | None, size: int, timeout_s: float) -> bytes:
    buf = ctypes.create_string_buffer(size)
    _check(lib().rmh_rendezvous_read(_b(path), None if run_id is None else run_id.encode(), buf, size,
                                     float(timeout_s)), "rmh_rendezvous_read")
    return buf.raw[:size]


def on_generation(cfg: RmhTrainConfig, fn) -> None:
    """Set cfg.on_generation to call fn(stage, num_spheres, raw_packed_copy) after each stage's
    training (every rank); the config keeps the callback alive."""
    def cb(_user, stage, m, raw):
        fn(stage, m, np.ctypeslib.as_array(raw, shape=(7 * m + 4,)).copy())
    cfg._gen_cb = GENERATION_FN(cb)
    cfg.on_generation = cfg._gen_cb


def train(cfg: RmhTrainConfig, max_spheres: int = 65536):
    res = RmhTrainResult()
    raw = np.empty(7 * max_spheres + 4, np.float32)
    _check(lib().rmh_train(ctypes.byref(cfg), ctypes.byref(res), _p(raw), raw.size), "rmh_train")
    m = res.num_spheres
    return res, raw[:7 * m + 4].copy()


def preview(scene_json, png_path, width=256, height=256, eye=(0.0, 0.0, -2.5), target=(0.0, 0.0, 0.0), fov=50.0,
            radius_offset=0.01, device=0) -> None:
    e = _f32c(eye, (3,))
    t = _f32c(target, (3,))
    _check(lib().rmh_preview(_b(scene_json), _b(png_path), width, height, _p(e), _p(t), fov, radius_offset, device),
           "rmh_preview")


def generate(out_dir, prefix="data/", width=256, height=256, device=0) -> None:
    _check(lib().rmh_generate(_b(out_dir), prefix.encode(), width, height, device), "rmh_generate")
