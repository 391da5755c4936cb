"""SceneModel mirror (model/scene.rs:9-57) over a packed raw-parameter buffer, the Adam
optimizer of train.rs:161-198, and the seeded synthetic scenes of BASELINE.md.

Packed layout (7M+4 floats, shared with include/raymarch.h):
    [centers 3M | colors 3M | radius M | light_dir 3 | ambient 1]
Raw values are the Burn ``Param`` tensors; ``activated()`` applies scene.rs:41-45 on
the GPU (rm_scene_activate).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import native
from .render import Scene, context, render_diff_camera, train_step_camera


def packed_size(m: int) -> int:
    return 7 * m + 4


def pack(centers, colors, radius, light_dir, ambient) -> np.ndarray:
    m = np.asarray(centers).reshape(-1, 3).shape[0]
    out = np.empty(packed_size(m), np.float32)
    out[:3 * m] = np.asarray(centers, np.float32).reshape(-1)
    out[3 * m:6 * m] = np.asarray(colors, np.float32).reshape(-1)
    out[6 * m:7 * m] = np.asarray(radius, np.float32).reshape(-1)
    out[7 * m:7 * m + 3] = np.asarray(light_dir, np.float32).reshape(-1)
    out[7 * m + 3] = np.asarray(ambient, np.float32).reshape(-1)[0]
    return out


def unpack(buf, m: int) -> dict:
    b = buf
    return {"centers": b[:3 * m].reshape(m, 3), "colors": b[3 * m:6 * m].reshape(m, 3),
            "radius": b[6 * m:7 * m], "light_dir": b[7 * m:7 * m + 3], "ambient": b[7 * m + 3:7 * m + 4]}


def logit(x):
    x = np.asarray(x, np.float64)
    return np.log(x / (1.0 - x))


def softplus_inv(y):
    y = np.asarray(y, np.float64)
    return np.log(np.expm1(y))


class SceneModel:
    """model/scene.rs:9-57 -- raw parameters on the device; forward renders via HIP."""

    def __init__(self, raw_packed: torch.Tensor, num_spheres: int, color_dtype: str = "f32"):
        if raw_packed.numel() != packed_size(num_spheres):
            raise ValueError("packed buffer size does not match num_spheres")
        if color_dtype not in ("f32", "f16"):
            raise ValueError("color_dtype must be 'f32' or 'f16'")
        self.raw = raw_packed.contiguous().float()
        self.num_spheres = num_spheres
        self._act = torch.empty_like(self.raw)
        self._act_valid = False  # _act == activate(raw); Adam.step keeps it valid
        # fp16 colour / fp32 SDF (BASELINE configs[4]): the render reads half colours
        # (RM_MARCH_COLOR_F16); parameters, moments and gradients stay fp32
        self.color_f16 = color_dtype == "f16"
        self._col_h = torch.empty((num_spheres, 3), dtype=torch.float16, device=self.raw.device) \
            if self.color_f16 else None

    @classmethod
    def from_raw(cls, centers, colors, radius, light_dir, ambient, device="cuda", color_dtype="f32"):
        buf = pack(centers, colors, radius, light_dir, ambient)
        return cls(torch.from_numpy(buf).to(device), np.asarray(centers).reshape(-1, 3).shape[0], color_dtype)

    @classmethod
    def from_activated(cls, centers, colors, radius, light_dir, ambient, device="cuda", color_dtype="f32"):
        """Build raw params whose activations equal the given values (radius includes +0.01)."""
        return cls.from_raw(centers, logit(colors), softplus_inv(np.asarray(radius, np.float64) - 0.01), light_dir,
                            logit(ambient), device=device, color_dtype=color_dtype)

    def invalidate(self):
        """Call after modifying ``raw`` outside the optimizer."""
        self._act_valid = False

    def activated_packed(self) -> torch.Tensor:
        if not self._act_valid:
            ctx = context(self.raw.device)
            ctx.check(ctx._lib.rm_scene_activate(ctx.handle, ctypes.c_void_p(self.raw.data_ptr()),
                                                 self.num_spheres, ctypes.c_void_p(self._act.data_ptr())),
                      "rm_scene_activate")
            if self.color_f16:  # initial fp16 colours (the optimizer writes them from then on)
                m = self.num_spheres
                self._col_h.copy_(self._act[3 * m:6 * m].view(m, 3))
            self._act_valid = True
        return self._act

    def scene(self) -> Scene:
        """scene.rs:41-45 activations as an rm_scene view (half colours for color_dtype f16)."""
        a = self.activated_packed()
        v = unpack(a, self.num_spheres)
        if self.color_f16:
            v["colors"] = self._col_h
        return Scene(*v.values())

    def forward_camera(self, cams, width, height, smooth_k, steps=40):
        return render_diff_camera(cams, width, height, self.scene(), smooth_k, steps)


class Adam:
    """Burn AdamConfig::new().with_weight_decay(1e-5) (train.rs:161-163): beta1 0.9, beta2 0.999,
    eps 1e-5, coupled L2 decay; the compute_loss penalties (training.rs:38-82) are added to the
    gradient inside the same kernel (rm_optimizer_step)."""

    def __init__(self, model: SceneModel, weight_decay=1e-5, with_penalties=True):
        self.model = model
        self.m = torch.zeros_like(model.raw)
        self.v = torch.zeros_like(model.raw)
        self.t = 0
        self.weight_decay = weight_decay
        self.with_penalties = with_penalties

    def step(self, grad_act_packed: torch.Tensor, lr: float, penalty_out: torch.Tensor | None = None):
        self.t += 1
        ctx = context(self.model.raw.device)
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        if self.model.color_f16:  # fp16-colour model: the updated colours also as half
            ctx.check(ctx._lib.rm_optimizer_step_f16(
                ctx.handle, p(self.model.raw), p(grad_act_packed), p(self.m), p(self.v), self.model.num_spheres, self.t,
                float(lr), float(self.weight_decay), 1 if self.with_penalties else 0, p(penalty_out),
                p(self.model._act), p(self.model._col_h)), "rm_optimizer_step_f16")
        else:
            ctx.check(ctx._lib.rm_optimizer_step(
                ctx.handle, p(self.model.raw), p(grad_act_packed), p(self.m), p(self.v), self.model.num_spheres, self.t,
                float(lr), float(self.weight_decay), 1 if self.with_penalties else 0, p(penalty_out),
                p(self.model._act)), "rm_optimizer_step")
        self.model._act_valid = True


    def train_step_camera(self, cams, width, height, targets, smooth_k, progress, lr, steps=40, *, inv_count=None,
                          grads_packed=None, loss=None, penalty_out=None, march=None, ctx=None):
        """rm_train_step_camera_adam: the camera-mode train step of this optimizer's model into
        grads_packed / loss (overwritten), then this optimizer's step on it -- one call; for up to
        64 spheres the optimizer runs inside the gradient reduction. The same results bit for bit
        as render.train_step_camera followed by step()."""
        from . import render as R
        mdl = self.model
        cams = list(cams)
        if not 1 <= len(cams) <= native.RM_MAX_VIEWS_PER_CALL:
            raise ValueError(f"1..{native.RM_MAX_VIEWS_PER_CALL} views per call")
        n = len(cams) * width * height
        targets = R._f32(targets, (n, 3), "targets")
        if inv_count is None:
            inv_count = 1.0 / (3.0 * n)
        dev = mdl.raw.device
        if grads_packed is None:
            grads_packed = torch.zeros(packed_size(mdl.num_spheres), device=dev)
        if loss is None:
            loss = torch.zeros((1,), device=dev)
        if ctx is None:
            ctx = context(dev)
        sc = mdl.scene()  # the activated parameters (and fp16 colours) are current
        if march is None:
            march = native.march_params(steps, smooth_k)
        march = sc.march_for(march)
        self.t += 1
        p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
        ctx.check(ctx._lib.rm_train_step_camera_adam(
            ctx.handle, native.cameras(cams), len(cams), width, height, p(targets), float(progress), float(inv_count),
            ctypes.byref(march), p(mdl._act), p(grads_packed), p(mdl.raw), p(self.m), p(self.v), mdl.num_spheres,
            self.t, float(lr), float(self.weight_decay), 1 if self.with_penalties else 0, p(loss), p(penalty_out),
            p(mdl._col_h)), "rm_train_step_camera_adam")
        mdl._act_valid = True
        return loss, grads_packed


# ---- seeded synthetic scenes (BASELINE.md "Synthetic inputs") ------------------------------
def synthetic_scene(num_spheres: int, seed: int = 0, radius_range=(0.03, 0.12)) -> dict:
    """numpy PCG64 default_rng(seed): centers uniform in the ball of radius 0.6, activated radii
    U[radius_range], colours U[0.05, 0.95], light_dir (-0.5, 0.5, -1), ambient 0.2."""
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(num_spheres, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    rad = 0.6 * rng.random((num_spheres, 1)) ** (1.0 / 3.0)
    return {
        "centers": (v * rad).astype(np.float32),
        "radius": rng.uniform(radius_range[0], radius_range[1], num_spheres).astype(np.float32),
        "colors": rng.uniform(0.05, 0.95, (num_spheres, 3)).astype(np.float32),
        "light_dir": np.array([-0.5, 0.5, -1.0], np.float32),
        "ambient": np.array([0.2], np.float32),
    }


def ring_cameras(num_views: int, radius=2.5, height=0.5, fov=50.0, offset=0):
    """generate.rs:44-63 ring: eye (R cos a, y, R sin a), a = i * 2 pi / num_views, looking at 0."""
    cams = []
    for i in range(offset, offset + num_views):
        a = i * (2.0 * math.pi / num_views)
        cams.append(([radius * math.cos(a), height, radius * math.sin(a)], [0.0, 0.0, 0.0], fov))
    return cams


def scene_tensors(sc: dict, device="cuda") -> Scene:
    return Scene(*(torch.from_numpy(np.ascontiguousarray(sc[k], np.float32)).to(device)
                   for k in ("centers", "colors", "radius", "light_dir", "ambient")))


__all__ = ["SceneModel", "Adam", "synthetic_scene", "ring_cameras", "scene_tensors", "pack", "unpack",
           "packed_size", "train_step_camera", "native"]
