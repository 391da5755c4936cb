"""ctypes loader for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module. It wraps ``oracle/_build/liboracle.so`` (built from
oracle/rm_oracle.c by oracle/Makefile), the scalar restatement of the reference's
render path (camera.rs, model/scene.rs, model/sdf.rs, renderer_diff.rs,
renderer.rs, training.rs) in fp32 (reference op order) and fp64.

All arrays are numpy, C-contiguous, AoS ``[n, 3]`` like the reference's tensors.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

_P = ctypes.c_void_p


def build() -> str:
    """Compile the oracle with its Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        for suf, real in (("f32", ctypes.c_float), ("f64", ctypes.c_double)):
            getattr(_lib, f"orc_camera_rays_{suf}").argtypes = [
                ctypes.c_int, ctypes.c_int, _P, _P, ctypes.c_float, _P, _P]
            getattr(_lib, f"orc_render_diff_{suf}").argtypes = [
                ctypes.c_long, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, real, _P, _P]
            getattr(_lib, f"orc_render_diff_backward_{suf}").argtypes = [
                ctypes.c_long, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, real, _P, _P,
                _P, _P, _P, _P, _P]
            getattr(_lib, f"orc_train_step_{suf}").argtypes = [
                ctypes.c_long, _P, _P, _P, real, real, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int,
                real, _P, _P, _P, _P, _P, _P, _P]
            getattr(_lib, f"orc_render_diff_debug_{suf}").argtypes = [
                ctypes.c_long, _P, _P, _P, _P, _P, _P, _P, ctypes.c_int, ctypes.c_int, real, _P]
            getattr(_lib, f"orc_render_{suf}").argtypes = [
                ctypes.c_long, _P, _P, _P, _P, _P, ctypes.c_int, _P]
    return _lib


def set_threads(n: int) -> int:
    """OpenMP threads of the oracle's parallel loops; returns the previous setting."""
    lb = lib()
    lb.orc_max_threads.restype = ctypes.c_int
    prev = lb.orc_max_threads()
    lb.orc_set_threads.argtypes = [ctypes.c_int]
    lb.orc_set_threads(int(n))
    return prev


def _dt(precision: str):
    if precision == "f32":
        return np.float32
    if precision == "f64":
        return np.float64
    raise ValueError(precision)


def _arr(x, dt):
    return np.ascontiguousarray(np.asarray(x, dtype=dt))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def camera_rays(width, height, eye, target, fov_deg, precision="f32"):
    """camera.rs:30-90 create_camera_rays -> (ray_org [W*H,3], ray_dir [W*H,3])."""
    dt = _dt(precision)
    n = width * height
    org = np.empty((n, 3), dt)
    dirs = np.empty((n, 3), dt)
    e = _arr(eye, np.float32)
    t = _arr(target, np.float32)
    getattr(lib(), f"orc_camera_rays_{precision}")(width, height, _ptr(e), _ptr(t), float(fov_deg),
                                                   _ptr(org), _ptr(dirs))
    return org, dirs


def _scene(scene, dt):
    c = _arr(scene["centers"], dt).reshape(-1, 3)
    col = _arr(scene["colors"], dt).reshape(-1, 3)
    r = _arr(scene["radius"], dt).reshape(-1)
    ld = _arr(scene["light_dir"], dt).reshape(3)
    a = _arr(scene["ambient"], dt).reshape(1)
    return c, col, r, ld, a


def render_diff(ray_org, ray_dir, scene, steps, smooth_k, precision="f64", with_t=False):
    """renderer_diff.rs:6-91 forward on activated params. Returns out [N,3] (and t)."""
    dt = _dt(precision)
    o = _arr(ray_org, dt)
    d = _arr(ray_dir, dt)
    c, col, r, ld, a = _scene(scene, dt)
    n = o.shape[0]
    out = np.empty((n, 3), dt)
    t = np.empty((n,), dt)
    getattr(lib(), f"orc_render_diff_{precision}")(n, _ptr(o), _ptr(d), _ptr(c), _ptr(col), _ptr(r), _ptr(ld),
                                                   _ptr(a), c.shape[0], steps, float(smooth_k), _ptr(out),
                                                   _ptr(t))
    return (out, t) if with_t else out


def render_diff_debug(ray_org, ray_dir, scene, steps, smooth_k, precision="f64"):
    """Per-ray intermediates [N,24] (layout of rm_debug_intermediates)."""
    dt = _dt(precision)
    o = _arr(ray_org, dt)
    d = _arr(ray_dir, dt)
    c, col, r, ld, a = _scene(scene, dt)
    n = o.shape[0]
    dbg = np.zeros((n, 24), dt)
    getattr(lib(), f"orc_render_diff_debug_{precision}")(n, _ptr(o), _ptr(d), _ptr(c), _ptr(col), _ptr(r),
                                                         _ptr(ld), _ptr(a), c.shape[0], steps, float(smooth_k),
                                                         _ptr(dbg))
    return dbg


def _grads(m, dt):
    return {"centers": np.zeros((m, 3), dt), "radius": np.zeros((m,), dt), "colors": np.zeros((m, 3), dt),
            "light_dir": np.zeros((3,), dt), "ambient": np.zeros((1,), dt)}


def render_diff_backward(ray_org, ray_dir, scene, steps, smooth_k, grad_out, precision="f64", t_march=None):
    """Analytic burn-autodiff backward of render_diff given g = dL/dout. Returns grads of
    the ACTIVATED params (centers, radius, colors, light_dir (raw), ambient)."""
    dt = _dt(precision)
    o = _arr(ray_org, dt)
    d = _arr(ray_dir, dt)
    g = _arr(grad_out, dt)
    c, col, r, ld, a = _scene(scene, dt)
    n, m = o.shape[0], c.shape[0]
    gr = _grads(m, dt)
    tm = _arr(t_march, dt) if t_march is not None else None
    getattr(lib(), f"orc_render_diff_backward_{precision}")(
        n, _ptr(o), _ptr(d), _ptr(c), _ptr(col), _ptr(r), _ptr(ld), _ptr(a), m, steps, float(smooth_k),
        _ptr(tm) if tm is not None else None, _ptr(g), _ptr(gr["centers"]), _ptr(gr["radius"]),
        _ptr(gr["colors"]), _ptr(gr["light_dir"]), _ptr(gr["ambient"]))
    return gr


def train_step(ray_org, ray_dir, targets, scene, steps, smooth_k, progress, inv_count=None, precision="f64"):
    """Fused forward + compute_loss reconstruction seed (training.rs:17-34) + backward.
    Returns (out, loss_sum, grads); loss = loss_sum * inv_count."""
    dt = _dt(precision)
    o = _arr(ray_org, dt)
    d = _arr(ray_dir, dt)
    tg = _arr(targets, dt)
    c, col, r, ld, a = _scene(scene, dt)
    n, m = o.shape[0], c.shape[0]
    if inv_count is None:
        inv_count = 1.0 / (3.0 * n)
    out = np.empty((n, 3), dt)
    loss = np.zeros((1,), dt)
    gr = _grads(m, dt)
    getattr(lib(), f"orc_train_step_{precision}")(
        n, _ptr(o), _ptr(d), _ptr(tg), float(progress), float(inv_count), _ptr(c), _ptr(col), _ptr(r),
        _ptr(ld), _ptr(a), m, steps, float(smooth_k), _ptr(out), _ptr(loss), _ptr(gr["centers"]),
        _ptr(gr["radius"]), _ptr(gr["colors"]), _ptr(gr["light_dir"]), _ptr(gr["ambient"]))
    return out, float(loss[0]), gr


def render(ray_org, ray_dir, centers, colors, radius, precision="f32"):
    """renderer.rs:4-80 non-differentiable target renderer (generate.rs)."""
    dt = _dt(precision)
    o = _arr(ray_org, dt)
    d = _arr(ray_dir, dt)
    c = _arr(centers, dt).reshape(-1, 3)
    col = _arr(colors, dt).reshape(-1, 3)
    r = _arr(radius, dt).reshape(-1)
    n = o.shape[0]
    out = np.empty((n, 3), dt)
    getattr(lib(), f"orc_render_{precision}")(n, _ptr(o), _ptr(d), _ptr(c), _ptr(col), _ptr(r), c.shape[0],
                                              _ptr(out))
    return out


def to_png_bytes(linear_rgb):
    """util.rs:6-9: (x^(1/2.2)).clamp(0,1)*255 truncated to u8 (NaN -> 0), in f32."""
    x = np.asarray(linear_rgb, dtype=np.float32)
    with np.errstate(invalid="ignore"):
        y = np.power(x, np.float32(1.0) / np.float32(2.2))
        y = np.clip(y, np.float32(0.0), np.float32(1.0)) * np.float32(255.0)
    y = np.where(np.isnan(y), np.float32(0.0), y)
    return np.trunc(y).astype(np.uint8)
