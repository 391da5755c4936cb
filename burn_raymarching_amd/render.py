"""Torch-facing mirror of the reference's render interface, executed by the HIP kernels.

Names and argument meaning follow the reference:
  * ``render_diff(ray_org, ray_dir, centers, colors, radius, light_dir, ambient, smooth_k)``
    -- renderer_diff.rs:6-15, differentiable through ``torch.autograd`` (the gradient
    is the analytic burn-autodiff backward computed by rm_render_diff_backward);
  * ``render_diff_camera(cams, width, height, ...)`` -- the same with rays generated
    in-kernel as create_camera_rays (camera.rs:30-90) would;
  * ``train_step(...)`` -- forward + compute_loss reconstruction seed + backward fused;
  * ``create_camera_rays(width, height, eye, target, fov_deg)`` -- host ray
    generation (camera.rs:30-90, a host loop in the reference too).

Tensors are torch CUDA (HIP) tensors, fp32, ``[N, 3]``; torch provides device memory
and the stream only. Shapes are checked on the host before any launch.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import native
from .native import RmGrads, RmScene

_ctx_cache: dict = {}


def context(device=None) -> native.Context:
    """Per-(device, stream) rm_context, bound to torch's current stream."""
    dev = torch.cuda.current_device() if device is None else (device.index if isinstance(device, torch.device)
                                                              else int(device))
    stream = torch.cuda.current_stream(dev).cuda_stream
    key = (dev, stream)
    ctx = _ctx_cache.get(key)
    if ctx is None:
        ctx = native.Context(dev, stream)
        _ctx_cache[key] = ctx
    return ctx


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _f32(t, shape, name):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor: the render path has no CPU implementation")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    t = t.contiguous()
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
    return t


class Scene:
    """Activated scene parameters (scene.rs:41-45) as device tensors + the rm_scene view."""

    def __init__(self, centers, colors, radius, light_dir, ambient):
        m = centers.shape[0]
        self.centers = _f32(centers, (m, 3), "centers")
        # fp16 colour / fp32 SDF (BASELINE configs[4]): half colours select RM_MARCH_COLOR_F16
        self.color_f16 = isinstance(colors, torch.Tensor) and colors.dtype == torch.float16
        if self.color_f16:
            if not colors.is_cuda or tuple(colors.shape) != (m, 3):
                raise ValueError("fp16 colors must be a [M,3] device tensor")
            self.colors = colors.contiguous()
        else:
            self.colors = _f32(colors, (m, 3), "colors")
        self.radius = _f32(radius.reshape(-1), (m,), "radius")
        self.light_dir = _f32(light_dir.reshape(-1), (3,), "light_dir")
        self.ambient = _f32(ambient.reshape(-1), (1,), "ambient")
        self.num_spheres = m

    @property
    def march_flags(self) -> int:
        return native.RM_MARCH_COLOR_F16 if self.color_f16 else 0

    def march_for(self, march) -> native.RmMarch:
        """A copy of `march` whose RM_MARCH_COLOR_F16 bit matches this scene's colour dtype (the
        caller's struct is never modified: a march shared between an fp16-colour and an fp32
        scene must not carry the bit from one call into the next)."""
        m = native.RmMarch.from_buffer_copy(march)
        m.flags = (m.flags & ~native.RM_MARCH_COLOR_F16) | self.march_flags
        return m

    def c_struct(self) -> RmScene:
        return RmScene(self.centers.data_ptr(), self.colors.data_ptr(), self.radius.data_ptr(),
                       self.light_dir.data_ptr(), self.ambient.data_ptr(), self.num_spheres)


def _grads_like(scene: Scene):
    dev = scene.centers.device
    m = scene.num_spheres
    g = {"centers": torch.empty((m, 3), device=dev), "colors": torch.empty((m, 3), device=dev),
         "radius": torch.empty((m,), device=dev), "light_dir": torch.empty((3,), device=dev),
         "ambient": torch.empty((1,), device=dev)}
    cg = RmGrads(g["centers"].data_ptr(), g["colors"].data_ptr(), g["radius"].data_ptr(),
                 g["light_dir"].data_ptr(), g["ambient"].data_ptr())
    return g, cg


def render_diff_forward(ray_org, ray_dir, scene: Scene, smooth_k, steps=40, *, normal_eps=1e-4,
                        color_sharpness=10.0, mask_sharpness=15.0, return_t=False):
    n = ray_org.shape[0]
    ray_org = _f32(ray_org, (n, 3), "ray_org")
    ray_dir = _f32(ray_dir, (n, 3), "ray_dir")
    out = torch.empty((n, 3), device=ray_org.device)
    t = torch.empty((n,), device=ray_org.device) if return_t else None
    ctx = context(ray_org.device)
    march = native.march_params(steps, smooth_k, normal_eps, color_sharpness, mask_sharpness)
    march = scene.march_for(march)
    ctx.check(ctx._lib.rm_render_diff(ctx.handle, _ptr(ray_org), _ptr(ray_dir), n, ctypes.byref(scene.c_struct()),
                                      ctypes.byref(march), _ptr(out), _ptr(t)), "rm_render_diff")
    return (out, t) if return_t else out


def render_diff_backward(ray_org, ray_dir, scene: Scene, smooth_k, grad_out, steps=40, *, t_march=None,
                         normal_eps=1e-4, color_sharpness=10.0, mask_sharpness=15.0):
    """Gradients of sum(out * grad_out) w.r.t. the activated params (light_dir raw)."""
    n = ray_org.shape[0]
    ray_org = _f32(ray_org, (n, 3), "ray_org")
    ray_dir = _f32(ray_dir, (n, 3), "ray_dir")
    grad_out = _f32(grad_out, (n, 3), "grad_out")
    if t_march is not None:
        t_march = _f32(t_march, (n,), "t_march")
    g, cg = _grads_like(scene)
    ctx = context(ray_org.device)
    march = native.march_params(steps, smooth_k, normal_eps, color_sharpness, mask_sharpness)
    march = scene.march_for(march)
    ctx.check(ctx._lib.rm_render_diff_backward(ctx.handle, _ptr(ray_org), _ptr(ray_dir), n,
                                               ctypes.byref(scene.c_struct()), ctypes.byref(march), _ptr(grad_out),
                                               _ptr(t_march), ctypes.byref(cg), 0), "rm_render_diff_backward")
    return g


class _RenderDiffFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ray_org, ray_dir, centers, colors, radius, light_dir, ambient, smooth_k, steps):
        scene = Scene(centers.detach(), colors.detach(), radius.detach(), light_dir.detach(), ambient.detach())
        out, t = render_diff_forward(ray_org.detach(), ray_dir.detach(), scene, smooth_k, steps, return_t=True)
        ctx.save_for_backward(ray_org, ray_dir, t)
        ctx.scene = scene
        ctx.smooth_k = smooth_k
        ctx.steps = steps
        ctx.radius_shape = radius.shape
        ctx.ambient_shape = ambient.shape
        return out

    @staticmethod
    def backward(ctx, grad_out):
        ray_org, ray_dir, t = ctx.saved_tensors
        g = render_diff_backward(ray_org, ray_dir, ctx.scene, ctx.smooth_k, grad_out.contiguous().float(),
                                 ctx.steps, t_march=t)
        return (None, None, g["centers"], g["colors"], g["radius"].reshape(ctx.radius_shape), g["light_dir"],
                g["ambient"].reshape(ctx.ambient_shape), None, None)


def render_diff(ray_org, ray_dir, centers, colors, radius, light_dir, ambient, smooth_k, steps=40):
    """renderer_diff.rs:6-91 on the GPU. Differentiable w.r.t. centers, colors, radius,
    light_dir, ambient (ray_org / ray_dir are detached inputs, as in the reference's data)."""
    return _RenderDiffFn.apply(ray_org, ray_dir, centers, colors, radius, light_dir, ambient, float(smooth_k),
                               int(steps))


def render_diff_camera(cams, width, height, scene: Scene, smooth_k, steps=40, *, normal_eps=1e-4,
                       color_sharpness=10.0, mask_sharpness=15.0, return_t=False):
    """Forward in camera mode: out [V*H*W, 3] for the given cameras (rays made in-kernel)."""
    cams = list(cams)
    v = len(cams)
    if v == 0:
        raise ValueError("at least one camera is required")
    dev = scene.centers.device
    out = torch.empty((v * height * width, 3), device=dev)
    t = torch.empty((v * height * width,), device=dev) if return_t else None
    ctx = context(dev)
    march = native.march_params(steps, smooth_k, normal_eps, color_sharpness, mask_sharpness)
    march = scene.march_for(march)
    for i in range(0, v, native.RM_MAX_VIEWS_PER_CALL):
        chunk = cams[i:i + native.RM_MAX_VIEWS_PER_CALL]
        off = i * height * width
        o = out[off:off + len(chunk) * height * width]
        tt = t[off:off + len(chunk) * height * width] if t is not None else None
        ctx.check(ctx._lib.rm_render_diff_camera(ctx.handle, native.cameras(chunk), len(chunk), width, height,
                                                 ctypes.byref(scene.c_struct()), ctypes.byref(march), _ptr(o),
                                                 _ptr(tt)), "rm_render_diff_camera")
    return (out, t) if return_t else out


def render_diff_backward_camera(cams, width, height, scene: Scene, smooth_k, grad_out, steps=40, *, t_march=None):
    cams = list(cams)
    if len(cams) > native.RM_MAX_VIEWS_PER_CALL:
        raise ValueError("at most 16 views per backward call")
    n = len(cams) * width * height
    grad_out = _f32(grad_out, (n, 3), "grad_out")
    if t_march is not None:
        t_march = _f32(t_march, (n,), "t_march")
    g, cg = _grads_like(scene)
    ctx = context(scene.centers.device)
    march = native.march_params(steps, smooth_k)
    march = scene.march_for(march)
    ctx.check(ctx._lib.rm_render_diff_backward_camera(ctx.handle, native.cameras(cams), len(cams), width, height,
                                                      ctypes.byref(scene.c_struct()), ctypes.byref(march),
                                                      _ptr(grad_out), _ptr(t_march), ctypes.byref(cg), 0),
              "rm_render_diff_backward_camera")
    return g


def train_step(ray_org, ray_dir, targets, scene: Scene, smooth_k, progress, steps=40, *, inv_count=None,
               with_out=False):
    """Fused forward + training.rs:17-34 seed + backward over rays. Returns (loss_sum, grads, out)."""
    n = ray_org.shape[0]
    ray_org = _f32(ray_org, (n, 3), "ray_org")
    ray_dir = _f32(ray_dir, (n, 3), "ray_dir")
    targets = _f32(targets, (n, 3), "targets")
    if inv_count is None:
        inv_count = 1.0 / (3.0 * n)
    g, cg = _grads_like(scene)
    loss = torch.zeros((1,), device=ray_org.device)
    out = torch.empty((n, 3), device=ray_org.device) if with_out else None
    ctx = context(ray_org.device)
    march = native.march_params(steps, smooth_k)
    march = scene.march_for(march)
    ctx.check(ctx._lib.rm_train_step(ctx.handle, _ptr(ray_org), _ptr(ray_dir), _ptr(targets), n, float(progress),
                                     float(inv_count), ctypes.byref(scene.c_struct()), ctypes.byref(march),
                                     ctypes.byref(cg), _ptr(loss), _ptr(out), 0), "rm_train_step")
    return loss, g, out


def train_step_camera(cams, width, height, targets, scene: Scene, smooth_k, progress, steps=40, *, inv_count=None,
                      grads_packed=None, loss=None, out=None, accumulate=False, march=None, ctx=None):
    """Camera-mode fused train step. If grads_packed ((7M+4) device tensor) is given the
    gradients go there in the packed layout; otherwise a dict is returned. ctx: the rm_context
    to run on (default: the one of torch's current stream)."""
    cams = list(cams)
    if not 1 <= len(cams) <= native.RM_MAX_VIEWS_PER_CALL:
        raise ValueError(f"1..{native.RM_MAX_VIEWS_PER_CALL} views per call")
    n = len(cams) * width * height
    targets = _f32(targets, (n, 3), "targets")
    if inv_count is None:
        inv_count = 1.0 / (3.0 * n)
    if ctx is None:
        ctx = context(scene.centers.device)
    if grads_packed is not None:
        cg = RmGrads()
        ctx._lib.rm_grads_from_packed(_ptr(grads_packed), scene.num_spheres, ctypes.byref(cg))
        g = grads_packed
    else:
        g, cg = _grads_like(scene)
    if loss is None:
        loss = torch.zeros((1,), device=scene.centers.device)
    if march is None:
        march = native.march_params(steps, smooth_k)
    march = scene.march_for(march)
    ctx.check(ctx._lib.rm_train_step_camera(ctx.handle, native.cameras(cams), len(cams), width, height, _ptr(targets),
                                            float(progress), float(inv_count), ctypes.byref(scene.c_struct()),
                                            ctypes.byref(march), ctypes.byref(cg), _ptr(loss), _ptr(out),
                                            1 if accumulate else 0), "rm_train_step_camera")
    return loss, g, out


def create_camera_rays(width, height, eye, target, fov_deg, device="cuda"):
    """camera.rs:30-90 (host loop in f32, like the reference), uploaded as [W*H, 3] tensors."""
    f32 = np.float32
    eye = np.asarray(eye, f32)
    target = np.asarray(target, f32)

    def normalize(v):
        ln = f32(np.sqrt(f32(v[0] * v[0] + v[1] * v[1]) + f32(v[2] * v[2])))
        return np.zeros(3, f32) if ln == 0 else (v / ln).astype(f32)

    fwd = normalize((target - eye).astype(f32))
    up_w = np.array([0, 1, 0], f32)
    right = normalize(np.cross(fwd, up_w).astype(f32))
    up = np.cross(right, fwd).astype(f32)
    aspect = f32(width) / f32(height)
    theta = f32(fov_deg) * (f32(math.pi) / f32(180.0)) / f32(2.0)
    half_h = f32(np.tan(theta))
    half_w = f32(aspect * half_h)
    xs = np.arange(width, dtype=f32)
    ys = np.arange(height, dtype=f32)
    u = (xs / f32(width)) * f32(2) - f32(1)
    v = -((ys / f32(height)) * f32(2) - f32(1))
    rs = (u * half_w)[None, :, None]
    us = (v * half_h)[:, None, None]
    d = (right[None, None, :] * rs + up[None, None, :] * us) + fwd[None, None, :]
    ln = np.sqrt((d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2])[..., None]
    d = (d / ln).astype(f32).reshape(-1, 3)
    o = np.broadcast_to(eye, d.shape).copy()
    return torch.from_numpy(o).to(device), torch.from_numpy(d).to(device)


def render(ray_org, ray_dir, centers, colors, radius):
    """renderer.rs:4-80 (the non-differentiable target renderer of generate.rs) on the GPU."""
    n = ray_org.shape[0]
    m = centers.shape[0]
    ray_org = _f32(ray_org, (n, 3), "ray_org")
    ray_dir = _f32(ray_dir, (n, 3), "ray_dir")
    centers = _f32(centers, (m, 3), "centers")
    colors = _f32(colors, (m, 3), "colors")
    radius = _f32(radius.reshape(-1), (m,), "radius")
    out = torch.empty((n, 3), device=ray_org.device)
    ctx = context(ray_org.device)
    ctx.check(ctx._lib.rm_render(ctx.handle, _ptr(ray_org), _ptr(ray_dir), n, _ptr(centers), _ptr(colors),
                                 _ptr(radius), m, _ptr(out)), "rm_render")
    return out


def render_camera(cams, width, height, centers, colors, radius):
    """renderer.rs:4-80 with in-kernel camera rays: out [V*H*W, 3] (generate.rs:88-104)."""
    cams = list(cams)
    if not 1 <= len(cams) <= native.RM_MAX_VIEWS_PER_CALL:
        raise ValueError(f"1..{native.RM_MAX_VIEWS_PER_CALL} views per call")
    m = centers.shape[0]
    centers = _f32(centers, (m, 3), "centers")
    colors = _f32(colors, (m, 3), "colors")
    radius = _f32(radius.reshape(-1), (m,), "radius")
    out = torch.empty((len(cams) * width * height, 3), device=centers.device)
    ctx = context(centers.device)
    ctx.check(ctx._lib.rm_render_camera(ctx.handle, native.cameras(cams), len(cams), width, height, _ptr(centers),
                                        _ptr(colors), _ptr(radius), m, _ptr(out)), "rm_render_camera")
    return out
