"""Literal op-by-op torch restatement of the reference's render graph, differentiated by
torch autograd (TEST INFRASTRUCTURE ONLY -- the independent pin of the analytic
backward in rm_oracle_impl.h, since the reference ships no gradient fixtures).

Each function mirrors the Burn tensor program it cites, including the detach points
that shape burn-autodiff's graph:
  * sdf.rs:37        -- the LSE max is ``detach()``ed
  * renderer_diff.rs:25 -- every march step's t is ``detach()``ed
  * renderer_diff.rs:41-46 -- the normal is computed from detached p, centers, radius
and Burn's softmax (max-shifted with a detached max), sigmoid and softplus.
Meant for small cases (N*M materialised), in float64 on the CPU.
"""
from __future__ import annotations

import torch


def soft_min_tensor(dists: torch.Tensor, k: float) -> torch.Tensor:
    """sdf.rs:30-44."""
    val = dists * (-k)
    max_val = val.detach().max(dim=1, keepdim=True).values
    ex = (val - max_val).exp()
    sum_exp = ex.sum(dim=1, keepdim=True)
    return (sum_exp.clamp_min(1e-8).log() + max_val) / (-k)


def scene_sdf_value(p, centers, radius, k):
    """scene.rs:60-79 (expansion-form distance)."""
    p_sq = p.pow(2).sum(dim=1, keepdim=True)
    c_sq = centers.pow(2).sum(dim=1, keepdim=True).t()
    p_dot_c = p @ centers.t()
    dists_sq = p_sq + c_sq - p_dot_c * 2.0
    dists = dists_sq.clamp_min(1e-6).sqrt()
    return soft_min_tensor(dists - radius.t(), k)


EPS_F32 = 9.999999747378752e-05  # f32(1e-4): the reference builds the offsets from f32 literals


def calc_normal_scene(p, centers, radius, k, eps=EPS_F32):
    """scene.rs:81-128 (scene.rs:91: eps = 1e-4 as f32)."""
    n = p.shape[0]
    offsets = torch.tensor([eps, 0, 0, -eps, 0, 0, 0, eps, 0, 0, -eps, 0, 0, 0, eps, 0, 0, -eps],
                           dtype=p.dtype).reshape(6, 3)
    p_flat = (p.unsqueeze(1) + offsets.unsqueeze(0)).reshape(n * 6, 3)
    d = scene_sdf_value(p_flat, centers, radius, k).reshape(n, 6)
    nrm = torch.cat([d[:, 0:1] - d[:, 1:2], d[:, 2:3] - d[:, 3:4], d[:, 4:5] - d[:, 5:6]], dim=1)
    length = (nrm.pow(2).sum(dim=1, keepdim=True) + 1e-6).sqrt()
    return nrm / length


def burn_softmax(x, dim):
    """burn::tensor::activation::softmax: x - max(x).detach(), exp, / sum."""
    x = x - x.detach().max(dim=dim, keepdim=True).values
    x = x.exp()
    return x / x.sum(dim=dim, keepdim=True)


def render_diff(ray_org, ray_dir, centers, colors, radius, light_dir, ambient, smooth_k, steps=40):
    """renderer_diff.rs:6-91 (steps is 40 in the reference; exposed for the configs)."""
    n = ray_org.shape[0]
    t = torch.zeros((n, 1), dtype=ray_org.dtype)
    for _ in range(steps):
        p = ray_org + ray_dir * t
        dist = scene_sdf_value(p, centers, radius, smooth_k)
        t = (t + dist).detach()
    p_approx = ray_org + ray_dir * t
    dist_last = scene_sdf_value(p_approx, centers, radius, smooth_k)
    t_final = t + dist_last
    p_final = ray_org + ray_dir * t_final
    normal = calc_normal_scene(p_final.detach(), centers.detach(), radius.detach(), smooth_k)
    ld = light_dir
    ld_sq = ld.pow(2).sum()
    ld_norm = ld / ld_sq.sqrt()
    dot = (normal @ ld_norm.unsqueeze(1)).squeeze(1)
    diffuse = dot.clamp_min(0.0)
    directional = diffuse * (1.0 - ambient)
    lighting = ambient + directional
    p_sq = p_final.pow(2).sum(dim=1, keepdim=True)
    c_sq = centers.pow(2).sum(dim=1, keepdim=True).t()
    p_dot_c = p_final @ centers.t()
    dists_sq = p_sq + c_sq - p_dot_c * 2.0
    dists = dists_sq.clamp_min(1e-6).sqrt() - radius.t()
    weights = burn_softmax(dists * (-10.0), 1)
    mixed = (colors.unsqueeze(0) * weights.unsqueeze(2)).sum(dim=1)
    object_color = mixed * lighting.unsqueeze(1)
    dist_scene = scene_sdf_value(p_final, centers, radius, smooth_k)
    mask = torch.sigmoid(dist_scene * (-15.0))
    return object_color * mask


def activate(raw):
    """scene.rs:41-45: colors sigmoid, radius softplus(beta=1)+0.01, ambient sigmoid."""
    return {
        "centers": raw["centers"],
        "colors": torch.sigmoid(raw["colors"]),
        "radius": torch.log(1.0 + torch.exp(raw["radius"])) + 0.01,
        "light_dir": raw["light_dir"],
        "ambient": torch.sigmoid(raw["ambient"]),
    }


def compute_loss(raw, output, target, progress):
    """training.rs:8-85 (reconstruction + the four parameter penalties) on RAW params."""
    diff = output - target
    abs_diff = diff.abs()
    target_mask = target.sum(dim=1, keepdim=True) > 0.01
    bg_weight = 1.0 + progress * 4.0
    weight_map = torch.where(target_mask, torch.full_like(abs_diff, 10.0), torch.full_like(abs_diff, bg_weight))
    loss = (abs_diff * weight_map).mean()
    centers = raw["centers"]
    radii = torch.log(1.0 + torch.exp(raw["radius"]))
    radius_l1 = radii.abs().mean()
    radius_large = torch.where(radii > 1.0, radii.pow(2), torch.zeros_like(radii)).mean()
    loss = loss + radius_large * 0.04 + radius_l1 * 0.002
    loss = loss + centers.pow(2).mean() * 0.05
    dist_from_origin = (centers.pow(2).sum(dim=1, keepdim=True) + 1e-6).sqrt()
    max_reach = dist_from_origin + radii
    excess = max_reach - 1.2
    prox = torch.where(max_reach > 1.2, excess.pow(2), torch.zeros_like(max_reach)).mean()
    loss = loss + prox * 5.0
    c_sq = centers.pow(2).sum(dim=1, keepdim=True)
    dist_sq = c_sq + c_sq.t() - (centers @ centers.t()) * 2.0
    dist_matrix = dist_sq.clamp_min(1e-6).sqrt()
    eye = torch.eye(centers.shape[0], dtype=centers.dtype)
    repulsion = (dist_matrix + eye * 100.0 + 1e-6).pow(-1.0).mean()
    return loss + repulsion * 0.00001
