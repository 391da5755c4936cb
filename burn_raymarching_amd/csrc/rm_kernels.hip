// rm_kernels.hip -- MI355X (gfx950) kernels of the differentiable SDF-sphere raymarcher
// and the C ABI declared in include/raymarch.h.
//
// Hot path replaced: render_diff (renderer_diff.rs:6-91) and its burn-autodiff
// backward (train.rs:189-190). One thread owns one ray for the whole pipeline:
//
//   in-kernel camera ray (camera.rs:58-78)
//   S fixed soft-min march steps          (renderer_diff.rs:20-26, scene.rs:60-79, sdf.rs:30-44)
//   gradient reconnect sweep at p_approx  (renderer_diff.rs:28-39)
//   6-tap finite-difference normal        (renderer_diff.rs:41-46, scene.rs:81-128)
//   Lambert + ambient                     (renderer_diff.rs:48-62)
//   softmax colour blend + mask soft-min  (renderer_diff.rs:64-90), one shared sweep
//   [train] weighted-L1 seed              (training.rs:17-34)
//   [bwd]   analytic backward: sweep at p_final, then at p_approx
//
// Spheres are staged once per workgroup in LDS (float4 {-2c, |c|^2}, float2 {k*log2e*r, r},
// float4 colour) and read as wave-uniform broadcasts. The soft-min log-sum-exp runs in
// base 2 on v_exp_f32/v_log_f32 with a chunked running max (one rescale per 8-16 spheres,
// one exp per sphere). Per-sphere gradients are summed over the 64 rays of a wave with a
// transposing permlane/DPP reduction, over the 4 waves in LDS, and over workgroups in a
// fixed order by rm_reduce_partials + rm_finalize_grads (deterministic; no atomics).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/raymarch.h"
#include "rm_device.h"

namespace rm {

enum Mode { kFwd = 0, kBwd = 1, kTrain = 2 };

constexpr int kTileMax = 1024;            // spheres per LDS tile (40 B each)
constexpr int kMaxBlocksPerLaunch = 4096; // bounds the partial-gradient workspace per launch
constexpr int kReduceSegs = 32;           // block segments of the first reduction pass

struct KArgs {
  // rays: array mode (org/dir) or camera mode (cams)
  const float* org;
  const float* dir;
  long long ray_begin;  // first ray of this launch
  long long n_rays;     // rays in this launch
  int width, height, num_views;
  CamBasis cams[RM_MAX_VIEWS_PER_CALL];
  // activated scene
  const float* centers;
  const float* colors;
  const float* radius;
  const float* light_dir;
  const float* ambient;
  int M, Mpad, tile;
  // march / shading
  int steps;
  float k, eps, csharp, msharp;
  // io
  float* out;
  float* t_out;
  const float* t_in;
  const float* gout;
  const float* targets;
  float progress, inv_count;
  float* dbg;       // optional per-ray intermediates [n][16] (diagnostics; see rm_debug_intermediates)
  float* partials;  // [gridDim.x][rec], rec = Mpad*12 + 8
  long long rec;
};

// ---- LDS staging --------------------------------------------------------------------
struct Lds {
  float4* geo;  // {-2cx, -2cy, -2cz, |c|^2}
  float4* col;  // {r, g, b, 0}
  float2* krr;  // {kappa * r, r}
  float* slots; // backward wave partials, 2 buffers
};

__device__ __forceinline__ void stage_tile(const KArgs& a, const Lds& L, int t0, int tn, float kappa) {
  for (int jl = threadIdx.x; jl < tn; jl += kBlock) {
    const int j = t0 + jl;
    if (j < a.M) {
      const float cx = a.centers[3 * j], cy = a.centers[3 * j + 1], cz = a.centers[3 * j + 2];
      const float r = a.radius[j];
      L.geo[jl] = make_float4(-2.0f * cx, -2.0f * cy, -2.0f * cz, cx * cx + cy * cy + cz * cz);
      L.col[jl] = make_float4(a.colors[3 * j], a.colors[3 * j + 1], a.colors[3 * j + 2], 0.0f);
      L.krr[jl] = make_float2(kappa * r, r);
    } else {
      // padding sphere at c = (kPadCenter, 0, 0): both the expansion form (|c|^2 term) and the
      // direct form of the normal taps (p - c) see distance ~1e15, so every exp() of its
      // soft-min / softmax terms underflows to exactly 0 and its gradient terms are exactly 0.
      L.geo[jl] = make_float4(-2.0f * kPadCenter, 0.0f, 0.0f, kPadCenter * kPadCenter);
      L.col[jl] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      L.krr[jl] = make_float2(0.0f, 0.0f);
    }
  }
}

// ---- forward sweeps -----------------------------------------------------------------
// q = |p|^2 + |c|^2 - 2 p.c (expansion form, scene.rs:66-71) from the staged record.
__device__ __forceinline__ float qexp(float px, float py, float pz, float pp, const float4& g) {
  return fmaf(pz, g.z, fmaf(py, g.y, fmaf(px, g.x, pp + g.w)));
}

// Base-2 log-sum-exp of v_j = kappa*(r_j - rho_j) over a tile (sdf.rs:36-40), running
// max m and shifted sum s carried across tiles. Chunks of 16: one rescale exp per chunk.
__device__ __forceinline__ void lse_point(float px, float py, float pz, float pp, const Lds& L, int n,
                                          float nkappa, float& m, float& s) {
  for (int j0 = 0; j0 < n; j0 += 16) {
    float v[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      const float4 g = L.geo[j0 + jj];
      const float kr = L.krr[j0 + jj].x;
      v[jj] = fmaf(fsqrt(fmaxf(qexp(px, py, pz, pp, g), 1e-6f)), nkappa, kr);
    }
    float cm = v[0];
#pragma unroll
    for (int jj = 1; jj < 16; ++jj) cm = fmaxf(cm, v[jj]);
    const float mn = fmaxf(m, cm);
    float s0 = s * fexp2(m - mn), s1 = 0.0f;
#pragma unroll
    for (int jj = 0; jj < 16; jj += 2) {
      s0 += fexp2(v[jj] - mn);
      s1 += fexp2(v[jj + 1] - mn);
    }
    s = s0 + s1;
    m = mn;
  }
}

// The six normal taps p +- eps*e_a (scene.rs:93-111) in one pass over the spheres.
// q at a tap is formed from e = p - c in direct form, |e +- eps e_a|^2 = |e|^2 + eps^2 +- 2 eps e_a,
// which keeps the fp32 error of the finite difference ~30x below the expansion form.
__device__ __forceinline__ void lse_taps(const float p[3], const Lds& L, int n, float nkappa, float two_eps,
                                         float eps2, float (&m)[6], float (&s)[6]) {
  for (int j0 = 0; j0 < n; j0 += 8) {
    float v[6][8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const float4 g = L.geo[j0 + jj];
      const float kr = L.krr[j0 + jj].x;
      const float ex = fmaf(0.5f, g.x, p[0]), ey = fmaf(0.5f, g.y, p[1]), ez = fmaf(0.5f, g.z, p[2]);
      const float Q = fmaf(ez, ez, fmaf(ey, ey, fmaf(ex, ex, eps2)));
      const float q[6] = {fmaf(ex, two_eps, Q), fmaf(ex, -two_eps, Q), fmaf(ey, two_eps, Q),
                          fmaf(ey, -two_eps, Q), fmaf(ez, two_eps, Q), fmaf(ez, -two_eps, Q)};
#pragma unroll
      for (int t = 0; t < 6; ++t) v[t][jj] = fmaf(fsqrt(fmaxf(q[t], 1e-6f)), nkappa, kr);
    }
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      float cm = v[t][0];
#pragma unroll
      for (int jj = 1; jj < 8; ++jj) cm = fmaxf(cm, v[t][jj]);
      const float mn = fmaxf(m[t], cm);
      float acc = s[t] * fexp2(m[t] - mn);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) acc += fexp2(v[t][jj] - mn);
      s[t] = acc;
      m[t] = mn;
    }
  }
}

// Shared sweep at p_final: colour softmax over -csharp*delta (renderer_diff.rs:74-82) and
// the mask soft-min over -k*delta (renderer_diff.rs:86). Both maxima sit at min delta,
// so one running minimum dmin shifts both sums.
__device__ __forceinline__ void shade_sweep(float px, float py, float pz, float pp, const Lds& L, int n,
                                            float c10l, float kappa, float& dmin, float& Zw, float (&C)[3],
                                            float& Zb) {
  for (int j0 = 0; j0 < n; j0 += 8) {
    float dl[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const float4 g = L.geo[j0 + jj];
      dl[jj] = fsqrt(fmaxf(qexp(px, py, pz, pp, g), 1e-6f)) - L.krr[j0 + jj].y;
    }
    float cmin = dl[0];
#pragma unroll
    for (int jj = 1; jj < 8; ++jj) cmin = fminf(cmin, dl[jj]);
    const float dn = fminf(dmin, cmin);
    const float sw = fexp2((dn - dmin) * c10l), sb = fexp2((dn - dmin) * kappa);
    Zw *= sw;
    C[0] *= sw;
    C[1] *= sw;
    C[2] *= sw;
    Zb *= sb;
    dmin = dn;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      // (dn - dl) <= 0 exactly: dn is the minimum of these very values, so the exponents can
      // never overflow however large |p| gets (miss rays march to |p| ~ 1e9 and beyond).
      const float dd = dn - dl[jj];
      const float ew = fexp2(dd * c10l);
      const float eb = fexp2(dd * kappa);
      const float4 c = L.col[j0 + jj];
      Zw += ew;
      C[0] = fmaf(ew, c.x, C[0]);
      C[1] = fmaf(ew, c.y, C[1]);
      C[2] = fmaf(ew, c.z, C[2]);
      Zb += eb;
    }
  }
}

// ---- the fused per-ray kernel ----------------------------------------------------------
template <int MODE, bool CAM>
__global__ __launch_bounds__(kBlock) void rm_ray_kernel(const KArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  Lds L;
  L.geo = reinterpret_cast<float4*>(smem);
  L.col = L.geo + a.tile;
  L.krr = reinterpret_cast<float2*>(L.col + a.tile);
  L.slots = reinterpret_cast<float*>(L.krr + a.tile);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long li = (long long)blockIdx.x * kBlock + tid;
  const bool valid = li < a.n_rays;
  const long long ri = a.ray_begin + (valid ? li : 0);

  const float kappa = a.k * kLog2e, nkappa = -kappa, inv_kappa = 1.0f / kappa;
  const bool multi = a.Mpad > a.tile;

  // ray (camera.rs:58-87 in camera mode)
  float o[3], d[3];
  if constexpr (CAM) {
    const long long npix = (long long)a.width * a.height;
    const int v = (int)(ri / npix);
    const long long pix = ri - (long long)v * npix;
    const int y = (int)(pix / a.width), x = (int)(pix - (long long)y * a.width);
    camera_ray(a.cams[v], x, y, a.width, a.height, o, d);
  } else {
    o[0] = a.org[3 * ri];
    o[1] = a.org[3 * ri + 1];
    o[2] = a.org[3 * ri + 2];
    d[0] = a.dir[3 * ri];
    d[1] = a.dir[3 * ri + 1];
    d[2] = a.dir[3 * ri + 2];
  }

  if (!multi) {
    stage_tile(a, L, 0, a.Mpad, kappa);
    __syncthreads();
  }
  // Visit every sphere tile (restaging LDS only when M exceeds one tile).
  auto for_tiles = [&](auto&& body) {
    for (int t0 = 0; t0 < a.Mpad; t0 += a.tile) {
      const int tn = min(a.tile, a.Mpad - t0);
      if (multi) {
        __syncthreads();
        stage_tile(a, L, t0, tn, kappa);
        __syncthreads();
      }
      body(t0, tn);
    }
  };
  // soft-min scene SDF at one point (scene.rs:60-79 + sdf.rs:30-44); returns D, keeps (m, s)
  auto soft_min = [&](const float p[3], float& m, float& s) {
    const float pp = fmaf(p[2], p[2], fmaf(p[1], p[1], p[0] * p[0]));
    m = -INFINITY;
    s = 0.0f;
    for_tiles([&](int, int tn) { lse_point(p[0], p[1], p[2], pp, L, tn, nkappa, m, s); });
    return -(flog2(fmaxf(s, 1e-8f)) + m) * inv_kappa;
  };

  // ---- march: t <- (t + sdf(o + d t)).detach(), S times (renderer_diff.rs:20-26)
  float t = 0.0f;
  if (MODE == kBwd && a.t_in != nullptr) {
    t = a.t_in[ri];
  } else {
    for (int st = 0; st < a.steps; ++st) {
      const float p[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
      float m, s;
      t += soft_min(p, m, s);
    }
  }
  if (MODE == kFwd && a.t_out != nullptr && valid) a.t_out[ri] = t;

  // ---- reconnect: t_final = t + sdf(p_approx) (renderer_diff.rs:30-39)
  const float pa[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
  float mA, sA;
  const float tf = t + soft_min(pa, mA, sA);
  const float p[3] = {fmaf(d[0], tf, o[0]), fmaf(d[1], tf, o[1]), fmaf(d[2], tf, o[2])};

  // ---- detached 6-tap normal (scene.rs:81-128)
  float nrm[3];
  float D6[6];
  {
    float m6[6], s6[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      m6[q] = -INFINITY;
      s6[q] = 0.0f;
    }
    const float eps = a.eps;
    for_tiles([&](int, int tn) { lse_taps(p, L, tn, nkappa, 2.0f * eps, eps * eps, m6, s6); });
#pragma unroll
    for (int q = 0; q < 6; ++q) D6[q] = -(flog2(fmaxf(s6[q], 1e-8f)) + m6[q]) * inv_kappa;
    const float nx = D6[0] - D6[1], ny = D6[2] - D6[3], nz = D6[4] - D6[5];
    const float inv_len = frsq(fmaf(nz, nz, fmaf(ny, ny, fmaf(nx, nx, 1e-6f))));
    nrm[0] = nx * inv_len;
    nrm[1] = ny * inv_len;
    nrm[2] = nz * inv_len;
  }

  // ---- lighting (renderer_diff.rs:48-62)
  const float ld0 = a.light_dir[0], ld1 = a.light_dir[1], ld2 = a.light_dir[2];
  const float amb = a.ambient[0];
  const float ldlen = sqrtf(ld0 * ld0 + ld1 * ld1 + ld2 * ld2);
  const float ldn[3] = {ld0 / ldlen, ld1 / ldlen, ld2 / ldlen};
  const float sdot = fmaf(nrm[2], ldn[2], fmaf(nrm[1], ldn[1], nrm[0] * ldn[0]));
  const float dif = fmaxf(sdot, 0.0f);
  const float Lgt = fmaf(dif, 1.0f - amb, amb);

  // ---- colour softmax + mask (renderer_diff.rs:64-90)
  const float c10l = a.csharp * kLog2e;
  const float pp = fmaf(p[2], p[2], fmaf(p[1], p[1], p[0] * p[0]));
  float dmin = INFINITY, Zw = 0.0f, Zb = 0.0f, C[3] = {0.0f, 0.0f, 0.0f};
  for_tiles([&](int, int tn) { shade_sweep(p[0], p[1], p[2], pp, L, tn, c10l, kappa, dmin, Zw, C, Zb); });
  const float invZw = frcp(Zw);
  const float mix[3] = {C[0] * invZw, C[1] * invZw, C[2] * invZw};
  const float Df = dmin - flog2(fmaxf(Zb, 1e-8f)) * inv_kappa;
  const float mu = frcp(1.0f + fexp2(a.msharp * kLog2e * Df));  // sigmoid(-msharp * D)
  const float scale = Lgt * mu;
  const float outv[3] = {mix[0] * scale, mix[1] * scale, mix[2] * scale};

  if (MODE == kFwd && a.dbg != nullptr && valid) {
    float* q = a.dbg + 24 * ri;
    const float vals[24] = {t, tf, nrm[0], nrm[1], nrm[2], Lgt, mix[0], mix[1], mix[2], Df, mu, sdot, dmin,
                            Zw, Zb, 0.0f, D6[0], D6[1], D6[2], D6[3], D6[4], D6[5], 0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 24; ++c) q[c] = vals[c];
  }
  const bool write_out = (MODE == kFwd || MODE == kTrain) && a.out != nullptr && valid;
  if (write_out) {
    a.out[3 * ri] = outv[0];
    a.out[3 * ri + 1] = outv[1];
    a.out[3 * ri + 2] = outv[2];
  }
  if constexpr (MODE == kFwd) return;

  // ---- seed g = dL/dout
  float g[3] = {0.0f, 0.0f, 0.0f};
  float loss = 0.0f;
  if (valid) {
    if constexpr (MODE == kBwd) {
      g[0] = a.gout[3 * ri];
      g[1] = a.gout[3 * ri + 1];
      g[2] = a.gout[3 * ri + 2];
    } else {  // training.rs:17-34
      const float t0 = a.targets[3 * ri], t1 = a.targets[3 * ri + 1], t2 = a.targets[3 * ri + 2];
      const float W = (t0 + t1 + t2) > 0.01f ? 10.0f : fmaf(a.progress, 4.0f, 1.0f);
      const float tg[3] = {t0, t1, t2};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float df = outv[c] - tg[c];
        loss = fmaf(fabsf(df), W, loss);
        const float sg = df > 0.0f ? 1.0f : (df < 0.0f ? -1.0f : 0.0f);
        g[c] = W * sg * a.inv_count;
      }
    }
  }

  // ---- backward seeds (out = mix * L * mu)
  const float gdotm = fmaf(g[2], mix[2], fmaf(g[1], mix[1], g[0] * mix[0]));
  const float gm[3] = {g[0] * scale, g[1] * scale, g[2] * scale};
  const float gL = gdotm * mu, gmu = gdotm * Lgt;
  const float gamb = gL * (1.0f - dif);
  const float gs = sdot >= 0.0f ? gL * (1.0f - amb) : 0.0f;  // clamp_min passes at x >= min
  const float gell[3] = {gs * nrm[0], gs * nrm[1], gs * nrm[2]};
  const float cmu = gmu * mu * (1.0f - mu) * (-a.msharp);
  const float mg = fmaf(mix[2], gm[2], fmaf(mix[1], gm[1], mix[0] * gm[0]));
  const float b_scale = cmu * frcp(Zb);
  const float ncs = -a.csharp;

  float* rec = a.partials + (long long)blockIdx.x * a.rec;
  float* slots = L.slots;
  int chunk_ctr = 0;

  // ---- backward sweep 1 at p_final: colour softmax + mask soft-min + p_final(t_final)
  float gp[3] = {0.0f, 0.0f, 0.0f};
  for_tiles([&](int t0, int tn) {
    for (int jc = 0; jc < tn; jc += kChunkBwd, ++chunk_ctr) {
      float* sb = slots + (chunk_ctr & 1) * (kWaves * kChunkBwd * 8);
      for (int jj = 0; jj < kChunkBwd; ++jj) {
        const int j = jc + jj;
        const float4 gg = L.geo[j];
        const float2 kr = L.krr[j];
        const float4 c4 = L.col[j];
        const float q = qexp(p[0], p[1], p[2], pp, gg);
        const float rho = fsqrt(fmaxf(q, 1e-6f));  // bitwise the forward's value (shade_sweep)
        const float dl = rho - kr.y;
        const float ir = frcp(rho);
        const float dd = dmin - dl;                 // <= 0 exactly
        const float w = fexp2(dd * c10l) * invZw;
        const float bt = fexp2(dd * kappa) * b_scale;
        const float cg = fmaf(c4.z, gm[2], fmaf(c4.y, gm[1], c4.x * gm[0]));
        const float gd = fmaf(w * ncs, cg - mg, bt);
        const float gu = q >= 1e-6f ? gd * ir : 0.0f;  // clamp_min(1e-6) gate
        const float ex = fmaf(0.5f, gg.x, p[0]), ey = fmaf(0.5f, gg.y, p[1]), ez = fmaf(0.5f, gg.z, p[2]);
        gp[0] = fmaf(gu, ex, gp[0]);
        gp[1] = fmaf(gu, ey, gp[1]);
        gp[2] = fmaf(gu, ez, gp[2]);
        const float vals[8] = {-gu * ex, -gu * ey, -gu * ez, -gd, w * gm[0], w * gm[1], w * gm[2], 0.0f};
        const float red = wave_reduce8(vals, lane);
        if ((lane & 7) == 7) sb[(wave * kChunkBwd + jj) * 8 + (lane >> 3)] = red;
      }
      __syncthreads();
      {
        const float* s0 = sb + tid;
        float acc = s0[0];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) acc += s0[w * kChunkBwd * 8];
        rec[(long long)(t0 + jc) * 8 + tid] = acc;
      }
    }
  });
  __syncthreads();

  // ---- backward sweep 2 at p_approx: t_final = t + D(p_approx) -> g_t * softmax(-k dist_a)
  const float gt = fmaf(gp[2], d[2], fmaf(gp[1], d[1], gp[0] * d[0]));
  const float hsc = gt * frcp(sA);
  const float ppa = fmaf(pa[2], pa[2], fmaf(pa[1], pa[1], pa[0] * pa[0]));
  for_tiles([&](int t0, int tn) {
    for (int jc = 0; jc < tn; jc += kChunkBwd, ++chunk_ctr) {
      float* sb = slots + (chunk_ctr & 1) * (kWaves * kChunkBwd * 8);
      for (int jj = 0; jj < kChunkBwd; jj += 2) {
        float vals[8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int j = jc + jj + u;
          const float4 gg = L.geo[j];
          const float kr = L.krr[j].x;
          const float q = qexp(pa[0], pa[1], pa[2], ppa, gg);
          const float rho = fsqrt(fmaxf(q, 1e-6f));  // bitwise the reconnect sweep's value
          const float ir = frcp(rho);
          const float h = fexp2(fmaf(rho, nkappa, kr) - mA) * hsc;  // v - mA <= 0 exactly
          const float hu = q >= 1e-6f ? h * ir : 0.0f;
          vals[4 * u + 0] = -hu * fmaf(0.5f, gg.x, pa[0]);
          vals[4 * u + 1] = -hu * fmaf(0.5f, gg.y, pa[1]);
          vals[4 * u + 2] = -hu * fmaf(0.5f, gg.z, pa[2]);
          vals[4 * u + 3] = -h;
        }
        const float red = wave_reduce8(vals, lane);
        if ((lane & 7) == 7) sb[(wave * kChunkBwd + jj) * 4 + (lane >> 3)] = red;
      }
      __syncthreads();
      if (tid < kChunkBwd * 4) {
        const float* s0 = sb + tid;
        float acc = s0[0];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) acc += s0[w * kChunkBwd * 4];
        rec[(long long)a.Mpad * 8 + (long long)(t0 + jc) * 4 + tid] = acc;
      }
    }
  });
  __syncthreads();

  // ---- per-ray scalars: light (pre-projection), ambient, loss
  {
    const float vals[8] = {gell[0], gell[1], gell[2], gamb, loss, 0.0f, 0.0f, 0.0f};
    const float red = wave_reduce8(vals, lane);
    if ((lane & 7) == 7) slots[wave * 8 + (lane >> 3)] = red;
    __syncthreads();
    if (tid < 8) {
      float acc = slots[tid];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) acc += slots[w * 8 + tid];
      rec[(long long)a.Mpad * 12 + tid] = acc;
    }
  }
}

// ---- cross-block reduction (fixed order => deterministic) --------------------------------
// Pass 1: S[seg][col] = sum over blocks b in segment seg of P[b][col].
__global__ __launch_bounds__(256) void rm_reduce_partials(const float* __restrict__ P, long long rec,
                                                          int nblocks, int seg_len, float* __restrict__ S) {
  const long long col = (long long)blockIdx.x * 256 + threadIdx.x;
  if (col >= rec) return;
  const int b0 = blockIdx.y * seg_len;
  const int b1 = min(b0 + seg_len, nblocks);
  float acc = 0.0f;
  for (int b = b0; b < b1; ++b) acc += P[(long long)b * rec + col];
  S[(long long)blockIdx.y * rec + col] = acc;
}

// Pass 2: sum the segments in order and scatter into the caller's gradient layout.
// gld = (g_ell - ldn (ldn . g_ell)) / |ld| applies the Jacobian of ld / |ld| (renderer_diff.rs:49-50).
__global__ __launch_bounds__(256) void rm_finalize_grads(const float* __restrict__ S, long long rec, int nseg,
                                                         int M, int Mpad, const float* __restrict__ light_dir,
                                                         float* gc, float* gcol, float* gr, float* gld, float* gamb,
                                                         float* loss_sum, int accumulate) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < M) {
    float v[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) v[c] = 0.0f;
    for (int s = 0; s < nseg; ++s) {
      const float* r1 = S + (long long)s * rec + (long long)j * 8;
      const float* r2 = S + (long long)s * rec + (long long)Mpad * 8 + (long long)j * 4;
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] += r1[c];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[8 + c] += r2[c];
    }
    const float gcv[3] = {v[0] + v[8], v[1] + v[9], v[2] + v[10]};
    const float grv = v[3] + v[11];
    if (gc) {
#pragma unroll
      for (int c = 0; c < 3; ++c) gc[3 * j + c] = accumulate ? gc[3 * j + c] + gcv[c] : gcv[c];
    }
    if (gr) gr[j] = accumulate ? gr[j] + grv : grv;
    if (gcol) {
#pragma unroll
      for (int c = 0; c < 3; ++c) gcol[3 * j + c] = accumulate ? gcol[3 * j + c] + v[4 + c] : v[4 + c];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float r[5] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    for (int s = 0; s < nseg; ++s) {
      const float* r0 = S + (long long)s * rec + (long long)Mpad * 12;
#pragma unroll
      for (int c = 0; c < 5; ++c) r[c] += r0[c];
    }
    const float l0 = light_dir[0], l1 = light_dir[1], l2 = light_dir[2];
    const float len = sqrtf(l0 * l0 + l1 * l1 + l2 * l2);
    const float ln[3] = {l0 / len, l1 / len, l2 / len};
    const float proj = ln[0] * r[0] + ln[1] * r[1] + ln[2] * r[2];
    if (gld) {
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float gv = (r[c] - ln[c] * proj) / len;
        gld[c] = accumulate ? gld[c] + gv : gv;
      }
    }
    if (gamb) gamb[0] = accumulate ? gamb[0] + r[3] : r[3];
    if (loss_sum) loss_sum[0] = accumulate ? loss_sum[0] + r[4] : r[4];
  }
}

// ---- model helpers (scene.rs:41-45, training.rs:38-82, Burn Adam) -------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// burn::tensor::activation::softplus(x, 1) = log(1 + exp(x))
__device__ __forceinline__ float softplusf_(float x) { return logf(1.0f + expf(x)); }

__global__ __launch_bounds__(256) void rm_activate_kernel(const float* __restrict__ raw, int M,
                                                          float* __restrict__ act) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = 7 * M + 4;
  if (i >= n) return;
  const float x = raw[i];
  float y;
  if (i < 3 * M) y = x;                       // centers
  else if (i < 6 * M) y = sigmoidf_(x);       // colors = sigmoid(raw)      scene.rs:41
  else if (i < 7 * M) y = softplusf_(x) + 0.01f;  // radius = softplus+0.01  scene.rs:43
  else if (i < 7 * M + 3) y = x;              // light_dir raw               scene.rs:44
  else y = sigmoidf_(x);                      // ambient = sigmoid(raw)      scene.rs:45
  act[i] = y;
}

// One thread per parameter element: chain rule of the activations, the compute_loss penalties
// (training.rs:38-82; O(M) per center element for the repulsion row), coupled weight decay and
// Burn's Adam update. Penalty value: block 0 reduces; O(M^2) repulsion summed by the threads
// of the center rows.
__global__ __launch_bounds__(256) void rm_optimizer_kernel(const float* __restrict__ raw, float* __restrict__ raw_out,
                                                           const float* __restrict__ gact,
                                                           float* __restrict__ m1, float* __restrict__ m2, int M,
                                                           int step, float lr, float wd, int with_pen,
                                                           float* __restrict__ pen_parts) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = 7 * M + 4;
  float pen = 0.0f;
  if (i < n) {
    const float x = raw[i];
    float gv = gact[i];
    if (i < 3 * M) {  // centers (identity activation)
      if (with_pen) {
        const int s = i / 3, ax = i - 3 * s;
        const float cx = raw[3 * s], cy = raw[3 * s + 1], cz = raw[3 * s + 2];
        const float rs = softplusf_(raw[6 * M + s]);  // penalties use softplus without +0.01 (training.rs:41)
        // [b] center attraction: mean(c^2) over [M,3] * 0.05
        gv += 0.05f * 2.0f * x / (3.0f * M);
        // [c] camera-proximity barrier: mean(mask * (|c| + r - 1.2)^2) * 5
        const float csq = cx * cx + cy * cy + cz * cz;
        const float dist = sqrtf(csq + 1e-6f);
        const float reach = dist + rs;
        if (reach > 1.2f) gv += 5.0f / M * 2.0f * (reach - 1.2f) * (x / dist);
        // [d] repulsion: mean((dist_ij + 100 I + 1e-6)^-1) * 1e-5 over [M,M]; d/dc_s of both (s,j) and (j,s)
        float acc = 0.0f;
        for (int j = 0; j < M; ++j) {
          const float ox = raw[3 * j], oy = raw[3 * j + 1], oz = raw[3 * j + 2];
          const float q = (csq + (ox * ox + oy * oy + oz * oz)) - (cx * ox + cy * oy + cz * oz) * 2.0f;
          if (j == s || q < 1e-6f) continue;  // clamp_min(1e-6) gate; diagonal: q ~ 0
          const float rho = sqrtf(q);
          const float den = rho + 1e-6f;
          const float xo = ax == 0 ? ox : (ax == 1 ? oy : oz);
          acc += -2.0f / (den * den) * (x - xo) / rho;
        }
        gv += 1e-5f / ((float)M * (float)M) * acc;
        if (ax == 0) {  // penalty value, once per sphere
          pen += 0.05f * csq / (3.0f * M);
          if (reach > 1.2f) pen += 5.0f / M * (reach - 1.2f) * (reach - 1.2f);
          float rep = 0.0f;
          for (int j = 0; j < M; ++j) {
            const float ox = raw[3 * j], oy = raw[3 * j + 1], oz = raw[3 * j + 2];
            const float q = (csq + (ox * ox + oy * oy + oz * oz)) - (cx * ox + cy * oy + cz * oz) * 2.0f;
            const float rho = sqrtf(fmaxf(q, 1e-6f));
            rep += 1.0f / (rho + (j == s ? 100.0f : 0.0f) + 1e-6f);
          }
          pen += 1e-5f / ((float)M * (float)M) * rep;
        }
      }
    } else if (i < 6 * M) {  // colors: d sigmoid = c (1 - c)
      const float c = sigmoidf_(x);
      gv *= c * (1.0f - c);
    } else if (i < 7 * M) {  // radius: d softplus = sigmoid
      const float sg = sigmoidf_(x);
      gv *= sg;
      if (with_pen) {
        const int s = i - 6 * M;
        const float rs = softplusf_(x);
        gv += 0.002f / M * (rs > 0.0f ? 1.0f : (rs < 0.0f ? -1.0f : 0.0f)) * sg;  // [a] L1
        pen += 0.002f / M * fabsf(rs);
        if (rs > 1.0f) {  // [a] large-radius
          gv += 0.04f / M * 2.0f * rs * sg;
          pen += 0.04f / M * rs * rs;
        }
        const float cx = raw[3 * s], cy = raw[3 * s + 1], cz = raw[3 * s + 2];
        const float reach = sqrtf(cx * cx + cy * cy + cz * cz + 1e-6f) + rs;
        if (reach > 1.2f) gv += 5.0f / M * 2.0f * (reach - 1.2f) * sg;  // [c] wrt radius
      }
    } else if (i < 7 * M + 3) {
      // light_dir raw: identity
    } else {  // ambient: d sigmoid
      const float a = sigmoidf_(x);
      gv *= a * (1.0f - a);
    }
    // Burn Adam with coupled weight decay: g += wd * theta; m, v moments; bias correction.
    gv = fmaf(wd, x, gv);
    const float b1 = 0.9f, b2 = 0.999f, eps = 1e-5f;
    const float mm = fmaf(b1, m1[i], (1.0f - b1) * gv);
    const float vv = fmaf(b2, m2[i], (1.0f - b2) * gv * gv);
    m1[i] = mm;
    m2[i] = vv;
    const float mh = mm / (1.0f - powf(b1, (float)step));
    const float vh = vv / (1.0f - powf(b2, (float)step));
    raw_out[i] = x - lr * (mh / (sqrtf(vh) + eps));
  }
  if (pen_parts != nullptr) {
    __shared__ float red[256];
    red[threadIdx.x] = pen;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) pen_parts[blockIdx.x] = red[0];
  }
}

__global__ void rm_sum_small(const float* __restrict__ parts, int n, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) acc += parts[i];
    out[0] = acc;
  }
}

}  // namespace rm

// =======================================================================================
// C ABI
// =======================================================================================
struct rm_context {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  void* ws = nullptr;  // partials | segment sums | small scratch
  size_t ws_bytes = 0;
};

namespace {

using namespace rm;

int fail(rm_context* ctx, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int fail(rm_context* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}

#define RM_HIP(ctx, call)                                                                        \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess) return fail(ctx, RM_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

int pad_spheres(int M) { return (M + kSphereAlign - 1) / kSphereAlign * kSphereAlign; }

long long rec_floats(int Mpad) { return (long long)Mpad * 12 + 8; }

size_t ws_need(long long max_rays, int M) {
  const int Mpad = pad_spheres(M);
  long long blocks = (max_rays + kBlock - 1) / kBlock;
  blocks = std::min<long long>(blocks, kMaxBlocksPerLaunch);
  const long long rec = rec_floats(Mpad);
  return (size_t)(blocks * rec + (long long)kReduceSegs * rec + 4096) * sizeof(float);
}

int ensure_ws(rm_context* ctx, size_t bytes) {
  if (ctx->ws_bytes >= bytes) return RM_OK;
  if (ctx->ws) {
    RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    RM_HIP(ctx, hipFree(ctx->ws));
    ctx->ws = nullptr;
    ctx->ws_bytes = 0;
  }
  hipError_t e = hipMalloc(&ctx->ws, bytes);
  if (e != hipSuccess) {
    ctx->ws = nullptr;
    return fail(ctx, RM_ERR_OOM, "workspace allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
  }
  ctx->ws_bytes = bytes;
  return RM_OK;
}

// camera.rs:40-52 on the host, in f32 like the reference.
int make_basis(rm_context* ctx, const rm_camera& c, int W, int H, CamBasis& b) {
  auto normalize = [](const float v[3], float out[3]) {
    const float len = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (len == 0.0f) {
      out[0] = out[1] = out[2] = 0.0f;
    } else {
      out[0] = v[0] / len;
      out[1] = v[1] / len;
      out[2] = v[2] / len;
    }
  };
  auto cross = [](const float a[3], const float bb[3], float out[3]) {
    out[0] = a[1] * bb[2] - a[2] * bb[1];
    out[1] = a[2] * bb[0] - a[0] * bb[2];
    out[2] = a[0] * bb[1] - a[1] * bb[0];
  };
  const float up_w[3] = {0.0f, 1.0f, 0.0f};
  const float fr[3] = {c.target[0] - c.eye[0], c.target[1] - c.eye[1], c.target[2] - c.eye[2]};
  float rr[3];
  normalize(fr, b.fwd);
  cross(b.fwd, up_w, rr);
  normalize(rr, b.right);
  cross(b.right, b.fwd, b.up);
  const float aspect = (float)W / (float)H;
  const float rads_per_deg = 3.14159265358979323846f / 180.0f;
  const float theta = c.fov_deg * rads_per_deg / 2.0f;
  b.half_h = std::tan(theta);
  b.half_w = aspect * b.half_h;
  for (int i = 0; i < 3; ++i) b.eye[i] = c.eye[i];
  if (!std::isfinite(b.half_h) || !(c.fov_deg > 0.0f && c.fov_deg < 180.0f))
    return fail(ctx, RM_ERR_INVALID_ARG, "camera fov_deg %g out of (0, 180)", (double)c.fov_deg);
  return RM_OK;
}

int check_scene(rm_context* ctx, const rm_scene* s) {
  if (!s) return fail(ctx, RM_ERR_INVALID_ARG, "scene is NULL");
  if (s->num_spheres < 1 || s->num_spheres > RM_MAX_SPHERES)
    return fail(ctx, RM_ERR_INVALID_ARG, "num_spheres %d out of [1, %d]", s->num_spheres, RM_MAX_SPHERES);
  if (!s->centers || !s->colors || !s->radius || !s->light_dir || !s->ambient)
    return fail(ctx, RM_ERR_INVALID_ARG, "scene has a NULL parameter pointer");
  return RM_OK;
}

int check_march(rm_context* ctx, const rm_march* m) {
  if (!m) return fail(ctx, RM_ERR_INVALID_ARG, "march is NULL");
  if (m->steps < 0 || m->steps > 100000) return fail(ctx, RM_ERR_INVALID_ARG, "steps %d out of range", m->steps);
  if (!(m->smooth_k > 0.0f) || !std::isfinite(m->smooth_k))
    return fail(ctx, RM_ERR_INVALID_ARG, "smooth_k must be finite and > 0 (got %g)", (double)m->smooth_k);
  if (!(m->normal_eps > 0.0f)) return fail(ctx, RM_ERR_INVALID_ARG, "normal_eps must be > 0");
  return RM_OK;
}

struct Call {
  int mode;  // Mode
  bool cam;
  const float* org = nullptr;
  const float* dir = nullptr;
  long long n = 0;
  const rm_camera* cams = nullptr;
  int views = 0, W = 0, H = 0;
  const rm_scene* scene = nullptr;
  const rm_march* march = nullptr;
  float* out = nullptr;
  float* t_out = nullptr;
  const float* t_in = nullptr;
  const float* gout = nullptr;
  const float* targets = nullptr;
  float progress = 0.0f, inv_count = 0.0f;
  float* dbg = nullptr;
  const rm_grads* grads = nullptr;
  float* loss_sum = nullptr;
  int accumulate = 0;
};

template <int MODE>
void launch_ray(bool cam, dim3 grid, size_t lds, hipStream_t st, const KArgs& a) {
  if (cam)
    hipLaunchKernelGGL((rm_ray_kernel<MODE, true>), grid, dim3(kBlock), lds, st, a);
  else
    hipLaunchKernelGGL((rm_ray_kernel<MODE, false>), grid, dim3(kBlock), lds, st, a);
}

int run(rm_context* ctx, const Call& c) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  int rc;
  if ((rc = check_scene(ctx, c.scene)) != RM_OK) return rc;
  if ((rc = check_march(ctx, c.march)) != RM_OK) return rc;
  KArgs a;
  std::memset(&a, 0, sizeof a);
  if (c.cam) {
    if (!c.cams) return fail(ctx, RM_ERR_INVALID_ARG, "cams is NULL");
    if (c.views < 1 || c.views > RM_MAX_VIEWS_PER_CALL)
      return fail(ctx, RM_ERR_INVALID_ARG, "num_views %d out of [1, %d]", c.views, RM_MAX_VIEWS_PER_CALL);
    if (c.W < 1 || c.H < 1 || (long long)c.W * c.H > (1LL << 28))
      return fail(ctx, RM_ERR_INVALID_ARG, "bad image size %dx%d", c.W, c.H);
    for (int v = 0; v < c.views; ++v)
      if ((rc = make_basis(ctx, c.cams[v], c.W, c.H, a.cams[v])) != RM_OK) return rc;
    a.width = c.W;
    a.height = c.H;
    a.num_views = c.views;
  } else {
    if (c.n < 0) return fail(ctx, RM_ERR_INVALID_ARG, "num_rays %lld < 0", c.n);
    if (c.n > 0 && (!c.org || !c.dir)) return fail(ctx, RM_ERR_INVALID_ARG, "ray_org/ray_dir is NULL");
  }
  const long long n = c.cam ? (long long)c.views * c.W * c.H : c.n;
  if (c.mode == kFwd && n > 0 && !c.out && !c.t_out && !c.dbg) return fail(ctx, RM_ERR_INVALID_ARG, "no output requested");
  if (c.mode == kBwd && n > 0 && !c.gout) return fail(ctx, RM_ERR_INVALID_ARG, "grad_out is NULL");
  if (c.mode == kTrain && n > 0 && !c.targets) return fail(ctx, RM_ERR_INVALID_ARG, "targets is NULL");
  if (c.mode != kFwd && !c.grads) return fail(ctx, RM_ERR_INVALID_ARG, "grads is NULL");

  const int M = c.scene->num_spheres;
  const int Mpad = pad_spheres(M);
  const int tile = std::min(Mpad, kTileMax);
  a.org = c.org;
  a.dir = c.dir;
  a.centers = c.scene->centers;
  a.colors = c.scene->colors;
  a.radius = c.scene->radius;
  a.light_dir = c.scene->light_dir;
  a.ambient = c.scene->ambient;
  a.M = M;
  a.Mpad = Mpad;
  a.tile = tile;
  a.steps = c.march->steps;
  a.k = c.march->smooth_k;
  a.eps = c.march->normal_eps;
  a.csharp = c.march->color_sharpness;
  a.msharp = c.march->mask_sharpness;
  a.out = c.out;
  a.t_out = c.t_out;
  a.t_in = c.t_in;
  a.gout = c.gout;
  a.targets = c.targets;
  a.progress = c.progress;
  a.inv_count = c.inv_count;
  a.dbg = c.dbg;
  a.rec = rec_floats(Mpad);
  const size_t lds = (size_t)tile * (16 + 16 + 8) + (size_t)2 * kWaves * kChunkBwd * 8 * sizeof(float);

  if (c.mode != kFwd) {
    if ((rc = ensure_ws(ctx, ws_need(std::max<long long>(n, 1), M))) != RM_OK) return rc;
  }
  float* P = static_cast<float*>(ctx->ws);

  if (n == 0) {  // nothing to render; backward/train still define their outputs
    if (c.mode == kFwd) return RM_OK;
  }
  long long done = 0;
  bool first = true;
  do {
    const long long blocks_left = (n - done + kBlock - 1) / kBlock;
    const long long nb = std::min<long long>(blocks_left, kMaxBlocksPerLaunch);
    const long long nr = std::min<long long>(n - done, nb * kBlock);
    a.ray_begin = done;
    a.n_rays = nr;
    a.partials = P;
    if (nb > 0) {
      dim3 grid((unsigned)nb);
      if (c.mode == kFwd) launch_ray<kFwd>(c.cam, grid, lds, ctx->stream, a);
      else if (c.mode == kBwd) launch_ray<kBwd>(c.cam, grid, lds, ctx->stream, a);
      else launch_ray<kTrain>(c.cam, grid, lds, ctx->stream, a);
      RM_HIP(ctx, hipGetLastError());
    }
    if (c.mode != kFwd) {
      const int nblocks = (int)nb;
      float* S = P + (long long)std::max<long long>(nb, 1) * a.rec;
      int segs = std::min(kReduceSegs, std::max(nblocks, 1));
      const int seg_len = nblocks > 0 ? (nblocks + segs - 1) / segs : 0;
      if (nblocks > 0) segs = (nblocks + seg_len - 1) / seg_len;
      if (nblocks > 0) {
        dim3 g1((unsigned)((a.rec + 255) / 256), (unsigned)segs);
        hipLaunchKernelGGL(rm_reduce_partials, g1, dim3(256), 0, ctx->stream, P, a.rec, nblocks, seg_len, S);
        RM_HIP(ctx, hipGetLastError());
      } else {
        RM_HIP(ctx, hipMemsetAsync(S, 0, sizeof(float) * a.rec, ctx->stream));
        segs = 1;
      }
      const rm_grads* gp = c.grads;
      const int acc = (first ? c.accumulate : 1);
      hipLaunchKernelGGL(rm_finalize_grads, dim3((M + 255) / 256), dim3(256), 0, ctx->stream, S, a.rec, segs, M,
                         Mpad, c.scene->light_dir, gp->centers, gp->colors, gp->radius, gp->light_dir,
                         gp->ambient, c.mode == kTrain ? c.loss_sum : nullptr, acc);
      RM_HIP(ctx, hipGetLastError());
    }
    done += nr;
    first = false;
  } while (done < n);
  return RM_OK;
}

}  // namespace

extern "C" {

const char* rm_version(void) { return "burn_raymarching_amd 0.1.0 (gfx950)"; }

int rm_create(int32_t device, void* stream, rm_context** out_ctx) {
  if (!out_ctx) return RM_ERR_INVALID_ARG;
  *out_ctx = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RM_ERR_HIP;
  if (hipSetDevice(device) != hipSuccess) return RM_ERR_HIP;
  rm_context* ctx = new rm_context();
  ctx->device = device;
  ctx->stream = static_cast<hipStream_t>(stream);
  *out_ctx = ctx;
  return RM_OK;
}

int rm_set_stream(rm_context* ctx, void* stream) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->stream = static_cast<hipStream_t>(stream);
  return RM_OK;
}

void rm_destroy(rm_context* ctx) {
  if (!ctx) return;
  if (ctx->ws) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->ws);
  }
  delete ctx;
}

const char* rm_last_error(const rm_context* ctx) { return ctx ? ctx->err.c_str() : "NULL context"; }

void rm_march_default(rm_march* m) {
  if (!m) return;
  m->steps = 40;             // renderer_diff.rs:22
  m->smooth_k = 32.0f;       // train.rs:131 MAX_SMOOTH / preview train.rs:355
  m->normal_eps = 1e-4f;     // scene.rs:91
  m->color_sharpness = 10.0f; // renderer_diff.rs:74
  m->mask_sharpness = 15.0f;  // renderer_diff.rs:88
}

int rm_reserve(rm_context* ctx, int64_t max_rays, int32_t max_spheres) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (max_rays < 0 || max_spheres < 1 || max_spheres > RM_MAX_SPHERES)
    return fail(ctx, RM_ERR_INVALID_ARG, "bad reserve sizes");
  return ensure_ws(ctx, ws_need(std::max<int64_t>(max_rays, 1), max_spheres));
}

int rm_render_diff(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
                   const rm_scene* scene, const rm_march* march, float* out, float* t_march) {
  Call c;
  c.mode = kFwd;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = num_rays;
  c.scene = scene;
  c.march = march;
  c.out = out;
  c.t_out = t_march;
  return run(ctx, c);
}

int rm_render_diff_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width, int32_t height,
                          const rm_scene* scene, const rm_march* march, float* out, float* t_march) {
  Call c;
  c.mode = kFwd;
  c.cam = true;
  c.cams = cams;
  c.views = num_views;
  c.W = width;
  c.H = height;
  c.scene = scene;
  c.march = march;
  c.out = out;
  c.t_out = t_march;
  return run(ctx, c);
}

int rm_render_diff_backward(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
                            const rm_scene* scene, const rm_march* march, const float* grad_out,
                            const float* t_march, const rm_grads* grads, int32_t accumulate) {
  Call c;
  c.mode = kBwd;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = num_rays;
  c.scene = scene;
  c.march = march;
  c.gout = grad_out;
  c.t_in = t_march;
  c.grads = grads;
  c.accumulate = accumulate;
  return run(ctx, c);
}

int rm_render_diff_backward_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width,
                                   int32_t height, const rm_scene* scene, const rm_march* march,
                                   const float* grad_out, const float* t_march, const rm_grads* grads,
                                   int32_t accumulate) {
  Call c;
  c.mode = kBwd;
  c.cam = true;
  c.cams = cams;
  c.views = num_views;
  c.W = width;
  c.H = height;
  c.scene = scene;
  c.march = march;
  c.gout = grad_out;
  c.t_in = t_march;
  c.grads = grads;
  c.accumulate = accumulate;
  return run(ctx, c);
}

int rm_train_step(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                  int64_t num_rays, float progress, float inv_count, const rm_scene* scene, const rm_march* march,
                  const rm_grads* grads, float* loss_sum, float* out, int32_t accumulate) {
  Call c;
  c.mode = kTrain;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = num_rays;
  c.targets = targets;
  c.progress = progress;
  c.inv_count = inv_count;
  c.scene = scene;
  c.march = march;
  c.grads = grads;
  c.loss_sum = loss_sum;
  c.out = out;
  c.accumulate = accumulate;
  return run(ctx, c);
}

int rm_train_step_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width, int32_t height,
                         const float* targets, float progress, float inv_count, const rm_scene* scene,
                         const rm_march* march, const rm_grads* grads, float* loss_sum, float* out,
                         int32_t accumulate) {
  Call c;
  c.mode = kTrain;
  c.cam = true;
  c.cams = cams;
  c.views = num_views;
  c.W = width;
  c.H = height;
  c.targets = targets;
  c.progress = progress;
  c.inv_count = inv_count;
  c.scene = scene;
  c.march = march;
  c.grads = grads;
  c.loss_sum = loss_sum;
  c.out = out;
  c.accumulate = accumulate;
  return run(ctx, c);
}

int rm_debug_intermediates(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
                           const rm_scene* scene, const rm_march* march, float* dbg) {
  if (!dbg) return fail(ctx, RM_ERR_INVALID_ARG, "dbg is NULL");
  Call c;
  c.mode = kFwd;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = num_rays;
  c.scene = scene;
  c.march = march;
  c.dbg = dbg;
  return run(ctx, c);
}

int rm_scene_activate(rm_context* ctx, const float* raw_packed, int32_t num_spheres, float* act_packed) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (!raw_packed || !act_packed) return fail(ctx, RM_ERR_INVALID_ARG, "NULL packed buffer");
  if (num_spheres < 1 || num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  const int n = 7 * num_spheres + 4;
  hipLaunchKernelGGL(rm::rm_activate_kernel, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, raw_packed,
                     num_spheres, act_packed);
  RM_HIP(ctx, hipGetLastError());
  return RM_OK;
}

void rm_scene_from_packed(const float* act, int32_t M, rm_scene* s) {
  if (!s) return;
  s->centers = act;
  s->colors = act + 3 * M;
  s->radius = act + 6 * M;
  s->light_dir = act + 7 * M;
  s->ambient = act + 7 * M + 3;
  s->num_spheres = M;
}

void rm_grads_from_packed(float* g, int32_t M, rm_grads* o) {
  if (!o) return;
  o->centers = g;
  o->colors = g + 3 * M;
  o->radius = g + 6 * M;
  o->light_dir = g + 7 * M;
  o->ambient = g + 7 * M + 3;
}

int rm_optimizer_step(rm_context* ctx, float* raw_packed, const float* grad_act_packed, float* adam_m,
                      float* adam_v, int32_t num_spheres, int32_t step, float lr, float weight_decay,
                      int32_t with_penalties, float* loss_penalty) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (!raw_packed || !grad_act_packed || !adam_m || !adam_v)
    return fail(ctx, RM_ERR_INVALID_ARG, "NULL optimizer buffer");
  if (num_spheres < 1 || num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  if (step < 1) return fail(ctx, RM_ERR_INVALID_ARG, "step counts from 1");
  const int n = 7 * num_spheres + 4;
  const int nb = (n + 255) / 256;
  // The penalties read every sphere's pre-step center while the update writes raw_packed:
  // the kernel reads a snapshot taken on the stream and writes raw_packed.
  const size_t need = ((size_t)n + (size_t)nb + 64) * sizeof(float);
  int rc = ensure_ws(ctx, std::max(ctx->ws_bytes, need));
  if (rc != RM_OK) return rc;
  float* snap = static_cast<float*>(ctx->ws);
  float* parts = loss_penalty ? snap + n : nullptr;
  RM_HIP(ctx, hipMemcpyAsync(snap, raw_packed, sizeof(float) * n, hipMemcpyDeviceToDevice, ctx->stream));
  hipLaunchKernelGGL(rm::rm_optimizer_kernel, dim3(nb), dim3(256), 0, ctx->stream, snap, raw_packed,
                     grad_act_packed, adam_m, adam_v, num_spheres, step, lr, weight_decay, with_penalties, parts);
  RM_HIP(ctx, hipGetLastError());
  if (loss_penalty) {
    hipLaunchKernelGGL(rm::rm_sum_small, dim3(1), dim3(64), 0, ctx->stream, parts, nb, loss_penalty);
    RM_HIP(ctx, hipGetLastError());
  }
  return RM_OK;
}

}  // extern "C"
