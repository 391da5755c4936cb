"""ctypes binding of libraymarch_hip.so (include/raymarch.h).

The product path: every compute call goes through this C ABI into the gfx950 HIP
kernels. There is no fallback -- if the library is missing or no GPU is present the
calls raise.
"""
from __future__ import annotations

import ctypes
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RM_LIB_PATH") or os.path.join(_PKG, "lib", "libraymarch_hip.so")

RM_OK = 0
RM_MAX_VIEWS_PER_CALL = 128
_ERR_NAMES = {1: "RM_ERR_INVALID_ARG", 2: "RM_ERR_HIP", 3: "RM_ERR_OOM", 4: "RM_ERR_UNSUPPORTED"}

_P = ctypes.c_void_p
_F = ctypes.c_float
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64


class RmScene(ctypes.Structure):
    _fields_ = [("centers", _P), ("colors", _P), ("radius", _P), ("light_dir", _P), ("ambient", _P),
                ("num_spheres", _I32)]


class RmMarch(ctypes.Structure):
    _fields_ = [("steps", _I32), ("smooth_k", _F), ("normal_eps", _F), ("color_sharpness", _F),
                ("mask_sharpness", _F), ("flags", _I32)]


RM_MARCH_SKIP_ESCAPED = 1
RM_MARCH_ROW_ORDER = 2
RM_MARCH_NO_EARLY_EXIT = 4
RM_MARCH_NATURAL_ORDER = 8
RM_MARCH_VALU_ONLY = 16
RM_MARCH_PER_RAY_ORIGIN = 32
RM_MARCH_STATIC_ORDER = 64
RM_MARCH_FORCE_MAX_SHIFT = 128
RM_MARCH_COLOR_F16 = 256
RM_MARCH_SPLIT = 512
RM_MARCH_NO_SPLIT = 1024


class RmStats(ctypes.Structure):
    _fields_ = [("blocks", _I64), ("blocks_skipped", _I64), ("waves", _I64), ("waves_exited", _I64),
                ("steps_saved", _I64), ("seeded_rays", _I64), ("seeded_rays_a", _I64)]


class RmCamera(ctypes.Structure):
    _fields_ = [("eye", _F * 3), ("target", _F * 3), ("fov_deg", _F)]


class RmGrads(ctypes.Structure):
    _fields_ = [("centers", _P), ("colors", _P), ("radius", _P), ("light_dir", _P), ("ambient", _P)]


# name -> (restype, argtypes): every symbol include/raymarch.h declares
SIGNATURES = {
    "rm_version": (ctypes.c_char_p, []),
    "rm_create": (ctypes.c_int, [_I32, _P, ctypes.POINTER(_P)]),
    "rm_set_stream": (ctypes.c_int, [_P, _P]),
    "rm_bind_step_scalars": (ctypes.c_int, [_P, _P]),
    "rm_destroy": (None, [_P]),
    "rm_last_error": (ctypes.c_char_p, [_P]),
    "rm_march_default": (None, [ctypes.POINTER(RmMarch)]),
    "rm_reserve": (ctypes.c_int, [_P, _I64, _I32]),
    "rm_render_diff": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(RmScene), ctypes.POINTER(RmMarch), _P, _P]),
    "rm_render_diff_camera": (ctypes.c_int, [_P, ctypes.POINTER(RmCamera), _I32, _I32, _I32,
                                             ctypes.POINTER(RmScene), ctypes.POINTER(RmMarch), _P, _P]),
    "rm_render_diff_backward": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(RmScene), ctypes.POINTER(RmMarch),
                                               _P, _P, ctypes.POINTER(RmGrads), _I32]),
    "rm_render_diff_backward_camera": (ctypes.c_int, [_P, ctypes.POINTER(RmCamera), _I32, _I32, _I32,
                                                      ctypes.POINTER(RmScene), ctypes.POINTER(RmMarch), _P, _P,
                                                      ctypes.POINTER(RmGrads), _I32]),
    "rm_train_step": (ctypes.c_int, [_P, _P, _P, _P, _I64, _F, _F, ctypes.POINTER(RmScene),
                                     ctypes.POINTER(RmMarch), ctypes.POINTER(RmGrads), _P, _P, _I32]),
    "rm_train_step_camera": (ctypes.c_int, [_P, ctypes.POINTER(RmCamera), _I32, _I32, _I32, _P, _F, _F,
                                            ctypes.POINTER(RmScene), ctypes.POINTER(RmMarch),
                                            ctypes.POINTER(RmGrads), _P, _P, _I32]),
    "rm_render": (ctypes.c_int, [_P, _P, _P, _I64, _P, _P, _P, _I32, _P]),
    "rm_render_camera": (ctypes.c_int, [_P, ctypes.POINTER(RmCamera), _I32, _I32, _I32, _P, _P, _P, _I32, _P]),
    "rm_gather_rays": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _P, _P, _P]),
    "rm_sample_batch": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _I64, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint64, _P, _P, _P, _P]),
    "rm_train_step_sampled": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _I64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_uint64, _F, _F, ctypes.POINTER(RmScene),
                                             ctypes.POINTER(RmMarch), ctypes.POINTER(RmGrads), _P]),
    "rm_train_step_sampled_prepared": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _I64, ctypes.c_uint64,
                                                      ctypes.c_uint64, ctypes.c_uint64, _F, _F, ctypes.POINTER(RmScene),
                                                      ctypes.POINTER(RmMarch), ctypes.POINTER(RmGrads), _P, _P, _I32,
                                                      _I32, _P]),
    "rm_debug_intermediates": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.POINTER(RmScene),
                                              ctypes.POINTER(RmMarch), _P]),
    "rm_debug_order_counts": (ctypes.c_int, [_P, ctypes.POINTER(_I32), _I32, ctypes.POINTER(_I32),
                                             ctypes.POINTER(_I32)]),
    "rm_debug_stall": (ctypes.c_int, [_P, _I32]),
    "rm_debug_stall_release": (ctypes.c_int, [_P]),
    "rm_timing_enable": (ctypes.c_int, [_P, _I32]),
    "rm_timing_collect": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I64), _I32]),
    "rm_stats_enable": (ctypes.c_int, [_P, _I32]),
    "rm_stats_collect": (ctypes.c_int, [_P, ctypes.POINTER(RmStats), _I32]),
    "rm_scene_activate": (ctypes.c_int, [_P, _P, _I32, _P]),
    "rm_scene_from_packed": (None, [_P, _I32, ctypes.POINTER(RmScene)]),
    "rm_grads_from_packed": (None, [_P, _I32, ctypes.POINTER(RmGrads)]),
    "rm_optimizer_step": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _F, _F, _I32, _P, _P]),
    "rm_optimizer_step_f16": (ctypes.c_int, [_P, _P, _P, _P, _P, _I32, _I32, _F, _F, _I32, _P, _P, _P]),
    "rm_train_step_camera_adam": (ctypes.c_int, [_P, ctypes.POINTER(RmCamera), _I32, _I32, _I32, _P, _F, _F,
                                                  ctypes.POINTER(RmMarch), _P, _P, _P, _P, _P, _I32, _I32, _F, _F,
                                                  _I32, _P, _P, _P]),
    "rm_train_iteration": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _I64, _I64, _I64, ctypes.c_uint64,
                                          ctypes.c_uint64, ctypes.c_uint64, _F, _F, ctypes.POINTER(RmMarch), _P, _P,
                                          _P, _P, _P, _I32, _I32, _F, _F, _I32, _P, _P]),
}

_lib = None
_lock = threading.Lock()


class RaymarchError(RuntimeError):
    pass


def lib():
    """Load libraymarch_hip.so (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RaymarchError(
                    f"{LIB_PATH} is missing: build it with `python -m burn_raymarching_amd._build` "
                    "(there is no CPU fallback for the render path)")
            handle = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


class Context:
    """An rm_context bound to a device and a HIP stream (torch's current stream by default)."""

    def __init__(self, device: int = 0, stream: int | None = None):
        self._lib = lib()
        self.device = device
        h = _P()
        if stream is None:
            stream = self._torch_stream(device)
        rc = self._lib.rm_create(device, _P(stream), ctypes.byref(h))
        if rc != RM_OK:
            raise RaymarchError(f"rm_create(device={device}) failed with {_ERR_NAMES.get(rc, rc)}")
        self.handle = h
        self.stream = stream

    @staticmethod
    def _torch_stream(device):
        import torch
        return torch.cuda.current_stream(device).cuda_stream

    def bind_step_scalars(self, dev_ptr):
        """rm_bind_step_scalars: progress / Adam step of this context's calls from the device
        record at dev_ptr ([step, index, total, reserved] int32; None unbinds)."""
        self.check(self._lib.rm_bind_step_scalars(self.handle, _P(dev_ptr) if dev_ptr else None),
                   "rm_bind_step_scalars")

    def set_stream(self, stream: int):
        self.check(self._lib.rm_set_stream(self.handle, _P(stream)), "rm_set_stream")
        self.stream = stream

    def check(self, rc: int, what: str):
        if rc != RM_OK:
            msg = self._lib.rm_last_error(self.handle)
            raise RaymarchError(f"{what} failed with {_ERR_NAMES.get(rc, rc)}: {msg.decode() if msg else ''}")

    def timing(self, enable: bool = True):
        self.check(self._lib.rm_timing_enable(self.handle, 1 if enable else 0), "rm_timing_enable")

    def collect_timing(self, reset: bool = True):
        """(summed per-ray kernel milliseconds, launches) since the last reset."""
        ms = ctypes.c_double()
        n = _I64()
        self.check(self._lib.rm_timing_collect(self.handle, ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0),
                   "rm_timing_collect")
        return ms.value, n.value

    def stats(self, enable: bool = True):
        self.check(self._lib.rm_stats_enable(self.handle, 1 if enable else 0), "rm_stats_enable")

    def collect_stats(self, reset: bool = True) -> dict:
        """rm_stats since the last reset: blocks, blocks_skipped, waves, waves_exited, steps_saved,
        seeded_rays, seeded_rays_a."""
        st = RmStats()
        self.check(self._lib.rm_stats_collect(self.handle, ctypes.byref(st), 1 if reset else 0), "rm_stats_collect")
        return {name: getattr(st, name) for name, _ in RmStats._fields_}

    def order_counts(self):
        """rm_debug_order_counts: ([3][classes] per-class block counts of the cost-order list sets,
        next_set)."""
        buf = (_I32 * 256)()
        cls = _I32()
        nxt = _I32()
        self.check(self._lib.rm_debug_order_counts(self.handle, buf, 256, ctypes.byref(cls), ctypes.byref(nxt)),
                   "rm_debug_order_counts")
        c = cls.value
        return [list(buf[i * c:(i + 1) * c]) for i in range(3)], nxt.value

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._lib.rm_destroy(self.handle)
            self.handle = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def march_params(steps=40, smooth_k=32.0, normal_eps=1e-4, color_sharpness=10.0, mask_sharpness=15.0,
                 skip_escaped=None, flags=0) -> RmMarch:
    """rm_march; skip_escaped None = the process default (env RM_SKIP_ESCAPED=1, else off);
    env RM_ROW_ORDER=1 adds RM_MARCH_ROW_ORDER (camera-mode row order instead of 16x16 tiles),
    env RM_NO_EARLY_EXIT=1 adds RM_MARCH_NO_EARLY_EXIT, env RM_NATURAL_ORDER=1 adds
    RM_MARCH_NATURAL_ORDER, env RM_VALU_ONLY=1 adds RM_MARCH_VALU_ONLY, env RM_PER_RAY_ORIGIN=1 adds
    RM_MARCH_PER_RAY_ORIGIN, env RM_STATIC_ORDER=1 adds RM_MARCH_STATIC_ORDER, env RM_FORCE_MAX_SHIFT=1 adds
    RM_MARCH_FORCE_MAX_SHIFT (A/B tests); `flags` are ORed in."""
    if skip_escaped is None:
        skip_escaped = os.environ.get("RM_SKIP_ESCAPED", "0") == "1"
    flags = int(flags) | (RM_MARCH_SKIP_ESCAPED if skip_escaped else 0)
    if os.environ.get("RM_ROW_ORDER") == "1":
        flags |= RM_MARCH_ROW_ORDER
    if os.environ.get("RM_NO_EARLY_EXIT") == "1":
        flags |= RM_MARCH_NO_EARLY_EXIT
    if os.environ.get("RM_NATURAL_ORDER") == "1":
        flags |= RM_MARCH_NATURAL_ORDER
    if os.environ.get("RM_VALU_ONLY") == "1":
        flags |= RM_MARCH_VALU_ONLY
    if os.environ.get("RM_PER_RAY_ORIGIN") == "1":
        flags |= RM_MARCH_PER_RAY_ORIGIN
    if os.environ.get("RM_STATIC_ORDER") == "1":
        flags |= RM_MARCH_STATIC_ORDER
    if os.environ.get("RM_FORCE_MAX_SHIFT") == "1":
        flags |= RM_MARCH_FORCE_MAX_SHIFT
    return RmMarch(int(steps), float(smooth_k), float(normal_eps), float(color_sharpness), float(mask_sharpness),
                   flags)


def cameras(cams) -> ctypes.Array:
    """cams: iterable of (eye[3], target[3], fov_deg) or dicts with origin/target/fov (cameras.json)."""
    cams = list(cams)
    arr = (RmCamera * max(len(cams), 1))()
    for i, c in enumerate(cams):
        if isinstance(c, dict):
            eye, tgt, fov = c.get("origin", c.get("eye")), c["target"], c.get("fov", c.get("fov_deg"))
        else:
            eye, tgt, fov = c
        arr[i].eye[:] = [float(x) for x in eye]
        arr[i].target[:] = [float(x) for x in tgt]
        arr[i].fov_deg = float(fov)
    return arr
