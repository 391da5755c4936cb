// rm_small.h -- the small-scene train / render kernel (included by rm_kernels.hip inside
// namespace rm, after the reduction kernels).
//
// The reference's own training loop (train.rs:169-199) renders a random 16,384-ray batch of a
// scene of 7-20 spheres, 40 march steps, per step: 64 ray blocks, one wave per SIMD on a quarter
// of the SIMDs. There the general kernel (rm_ray_kernel) is bound by the latency of one wave's
// march step (its matrix-core tiles, LDS exchange and fragment loads serve 32-sphere row blocks,
// 23 of 32 padding at M = 9) and by the three small launches around it (records, reduction,
// finalize). This kernel is written for that regime, M <= kSmallMaxM:
//  * one launch per call: every block builds the sphere data it needs from the activated
//    parameters itself (LDS, then registers), and the last block to finish sums the blocks'
//    partial records in block order and writes the gradients (a release / acquire hand-off on an
//    arrival counter; launches of more than kSmallFinalMaxBlocks blocks write partial records for
//    rm_reduce_partials / rm_finalize_grads instead);
//  * the sphere data of the march live in VGPRs (uniform values: a small launch has one wave per
//    SIMD, registers are free), the sphere loop runs over the real spheres in groups of four (a
//    group past M is skipped by a scalar branch; the 1-3 padding spheres of the last group sit at
//    x = 1e15 and contribute exact zeros, as in rm_prep_kernel);
//  * every soft-min takes the reference's exact maximum shift (sdf.rs:36-40) per ray: two passes
//    over the spheres held in registers, no wave-uniform path choice, no matrix-core exchange;
//  * the backward keeps one ray per lane and sums each sphere's seven gradient terms over the
//    wave with the transposing 8-value reduction (wave_reduce8), the four waves in LDS in order.
// Deterministic: every sum has a fixed order (lanes, waves, blocks).
#pragma once

constexpr int kSmallMaxM = 32;           // spheres handled by the small kernel
constexpr int kSmallGroup = 4;           // sphere loop granularity (scalar-branch groups)
constexpr int kSmallFinalMaxBlocks = 256;  // in-kernel final reduction up to this many blocks

struct SmallArgs {
  FinalArgs fin;          // where the last block writes the gradients and the loss
  unsigned* arrivals;     // arrival counter (zero between launches; the last block resets it)
  int final_in_kernel;    // 1: the last block reduces and finalizes; 0: partial records only
};

// Per-sphere march data in registers: gx = -2c, cc = |c|^2 (expansion form, scene.rs:66-71),
// kr = kappa r (kappa = smooth_k log2 e).
template <int MB>
struct SmallSpheres {
  float gx[MB], gy[MB], gz[MB], cc[MB], kr[MB];
};

// Soft-min scene SDF at p (scene.rs:60-79 + sdf.rs:30-44) in base 2 with the exact per-ray max
// shift: D = -(log2(sum_j 2^(v_j - m)) + m) / kappa, v_j = kappa (r_j - rho_j). RSQ: rho = q rsq(q)
// (the reconnect: backward sweep 2 recomputes the same v_j bit for bit); else rho = sqrt(q).
template <int MB, bool RSQ>
__device__ __forceinline__ float small_softmin(const float p[3], const SmallSpheres<MB>& S, int M, float kappa,
                                               float inv_kappa, float& m_out, float& s_out) {
  const float pp = psq(p);
  float v[MB];
  float m = -INFINITY;
#pragma unroll
  for (int j0 = 0; j0 < MB; j0 += kSmallGroup) {
    if (j0 < M) {
#pragma unroll
      for (int j = j0; j < j0 + kSmallGroup; ++j) {
        const float q = qclamp(fmaf(p[2], S.gz[j], fmaf(p[1], S.gy[j], fmaf(p[0], S.gx[j], pp + S.cc[j]))), 1e-6f);
        const float rho = RSQ ? q * frsq(q) : fsqrt(q);
        v[j] = fmaf(-kappa, rho, S.kr[j]);
        m = fmaxf(m, v[j]);
      }
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int j0 = 0; j0 < MB; j0 += kSmallGroup) {
    if (j0 < M) {
#pragma unroll
      for (int j = j0; j < j0 + kSmallGroup; ++j) s += fexp2(v[j] - m);
    }
  }
  m_out = m;
  s_out = s;
  return -(flog2(fmaxf(s, 1e-8f)) + m) * inv_kappa;
}

template <int MODE, bool CAM, int MB>
__global__ __launch_bounds__(kBlock, 1) void rm_small_kernel(const KArgs a, const SmallArgs sa) {
  static_assert(MB % kSmallGroup == 0 && MB <= kSmallMaxM, "sphere bucket");
  constexpr int kRec = kSmallMaxM * 8 + 8;  // per-wave slot of the cross-wave sums
  __shared__ float4 s_geo[MB];              // {gx, gy, gz, cc}
  __shared__ float4 s_mat[MB];              // {kr, r, 0, 0}
  __shared__ float4 s_col[MB];              // {red, green, blue, 0}
  __shared__ float s_red[kWaves * kRec];    // per-wave sums: [wave][sphere][8] | [wave][8 scalars]
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.M;
  const float kappa = a.k * kLog2e, inv_kappa = 1.0f / kappa;

  // ---- sphere data of the activated scene (scene.rs:41-45 values), padding spheres far away
  if (tid < MB) {
    const int j = tid;
    if (j < M) {
      const float cx = a.centers[3 * j], cy = a.centers[3 * j + 1], cz = a.centers[3 * j + 2], r = a.radius[j];
      s_geo[j] = make_float4(-2.0f * cx, -2.0f * cy, -2.0f * cz, cx * cx + cy * cy + cz * cz);
      s_mat[j] = make_float4(kappa * r, r, 0.0f, 0.0f);
      if (a.colors_h != nullptr)
        s_col[j] = make_float4((float)a.colors_h[3 * j], (float)a.colors_h[3 * j + 1], (float)a.colors_h[3 * j + 2], 0.0f);
      else
        s_col[j] = make_float4(a.colors[3 * j], a.colors[3 * j + 1], a.colors[3 * j + 2], 0.0f);
    } else {
      s_geo[j] = make_float4(-2.0f * kPadCenter, 0.0f, 0.0f, kPadCenter * kPadCenter);
      s_mat[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      s_col[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  }

  // ---- the ray (camera.rs:58-87 in camera mode)
  const long long blk = blockIdx.x;
  const long long li = blk * kBlock + tid;
  const bool valid = li < a.n_rays;
  long long ri = a.ray_begin + (valid ? li : 0);
  float o[3], d[3];
  int view;
  setup_ray<CAM>(a, ri, o, d, view);
  __syncthreads();
  SmallSpheres<MB> S;
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    const float4 g = s_geo[j];
    S.gx[j] = g.x;
    S.gy[j] = g.y;
    S.gz[j] = g.z;
    S.cc[j] = g.w;
    S.kr[j] = s_mat[j].x;
  }

  // ---- march: t <- (t + sdf(o + d t)).detach(), S times (renderer_diff.rs:20-26)
  float t = 0.0f;
  if (MODE == kBwd && a.t_in != nullptr) {
    t = a.t_in[ri];
  } else {
    for (int st = 0; st < a.steps; ++st) {
      const float p[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
      float m, s;
      t = fminf(t + small_softmin<MB, false>(p, S, M, kappa, inv_kappa, m, s), kTMax);
    }
  }
  if (MODE == kFwd && a.t_out != nullptr && valid) a.t_out[ri] = t;

  // ---- reconnect: t_final = t + sdf(p_approx) (renderer_diff.rs:30-39)
  const float pa[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
  float mA, sA;
  const float Da = small_softmin<MB, true>(pa, S, M, kappa, inv_kappa, mA, sA);
  const float tf = t + Da;
  const float p[3] = {fmaf(d[0], tf, o[0]), fmaf(d[1], tf, o[1]), fmaf(d[2], tf, o[2])};

  // ---- shade sweep at p_final: colour softmax over -csharp delta (renderer_diff.rs:64-82),
  // mask soft-min over -k delta (renderer_diff.rs:86-90) and the detached normal as the eps -> 0
  // limit of scene.rs:81-128 (2 eps grad D, grad D = sum beta_j (p - c_j) / rho_j), two passes:
  // the exact minimum delta, then the sums relative to it (exponents <= 0 exactly)
  const float c10l = a.csharp * kLog2e;
  const float pp = psq(p);
  float dl[MB], ir[MB];
  float dmin = INFINITY;
#pragma unroll
  for (int j0 = 0; j0 < MB; j0 += kSmallGroup) {
    if (j0 < M) {
#pragma unroll
      for (int j = j0; j < j0 + kSmallGroup; ++j) {
        const float4 mt = s_mat[j];
        const float q = fmaf(p[2], S.gz[j], fmaf(p[1], S.gy[j], fmaf(p[0], S.gx[j], pp + S.cc[j])));
        const float qc = qclamp(q, 1e-6f);
        const float r = frsq(qc);
        dl[j] = qc * r - mt.y;  // delta_j = rho_j - r_j
        ir[j] = q >= 1e-6f ? r : 0.0f;  // clamp_min(1e-6) gate: that distance carries no gradient
        dmin = fminf(dmin, dl[j]);
      }
    }
  }
  float Zw = 0.0f, Zb = 0.0f, C[3] = {0.0f, 0.0f, 0.0f}, G[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int j0 = 0; j0 < MB; j0 += kSmallGroup) {
    if (j0 < M) {
#pragma unroll
      for (int j = j0; j < j0 + kSmallGroup; ++j) {
        const float dd = dmin - dl[j];
        const float ew = fexp2(dd * c10l), eb = fexp2(dd * kappa);
        const float4 col = s_col[j];
        Zw += ew;
        C[0] = fmaf(ew, col.x, C[0]);
        C[1] = fmaf(ew, col.y, C[1]);
        C[2] = fmaf(ew, col.z, C[2]);
        Zb += eb;
        const float wr = eb * ir[j];
        G[0] = fmaf(wr, fmaf(0.5f, S.gx[j], p[0]), G[0]);
        G[1] = fmaf(wr, fmaf(0.5f, S.gy[j], p[1]), G[1]);
        G[2] = fmaf(wr, fmaf(0.5f, S.gz[j], p[2]), G[2]);
      }
    }
  }
  const float te = 2.0f * a.eps * frcp(Zb);
  const float nx = te * G[0], ny = te * G[1], nz = te * G[2];
  const float inv_len = frsq(fmaf(nz, nz, fmaf(ny, ny, fmaf(nx, nx, 1e-6f))));
  const float nrm[3] = {nx * inv_len, ny * inv_len, nz * inv_len};
  // ---- lighting (renderer_diff.rs:48-62)
  const float ld0 = a.light_dir[0], ld1 = a.light_dir[1], ld2 = a.light_dir[2];
  const float amb = a.ambient[0];
  const float ldlen = sqrtf(ld0 * ld0 + ld1 * ld1 + ld2 * ld2);
  const float ldn[3] = {ld0 / ldlen, ld1 / ldlen, ld2 / ldlen};
  const float sdot = fmaf(nrm[2], ldn[2], fmaf(nrm[1], ldn[1], nrm[0] * ldn[0]));
  const float dif = fmaxf(sdot, 0.0f);
  const float Lgt = fmaf(dif, 1.0f - amb, amb);
  const float Df = dmin - flog2(fmaxf(Zb, 1e-8f)) * inv_kappa;
  const float invZw = frcp(Zw);
  const float mix[3] = {C[0] * invZw, C[1] * invZw, C[2] * invZw};
  const float mu = frcp(1.0f + fexp2(a.msharp * kLog2e * Df));  // sigmoid(-msharp D)
  const float scale = Lgt * mu;
  const float outv[3] = {mix[0] * scale, mix[1] * scale, mix[2] * scale};
  if (MODE != kBwd && a.out != nullptr && valid) {
    a.out[3 * ri] = outv[0];
    a.out[3 * ri + 1] = outv[1];
    a.out[3 * ri + 2] = outv[2];
  }
  if constexpr (MODE == kFwd) return;

  // ---- seed g = dL/dout (training.rs:17-34 in the train step)
  float g[3] = {0.0f, 0.0f, 0.0f};
  float loss = 0.0f;
  if (valid) {
    if constexpr (MODE == kBwd) {
      g[0] = a.gout[3 * ri];
      g[1] = a.gout[3 * ri + 1];
      g[2] = a.gout[3 * ri + 2];
    } else {
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
  // backward seeds (out = mix L mu), as rm_ray_kernel
  const float gdotm = fmaf(g[2], mix[2], fmaf(g[1], mix[1], g[0] * mix[0]));
  const float gm[3] = {g[0] * scale, g[1] * scale, g[2] * scale};
  const float gL = gdotm * mu, gmu = gdotm * Lgt;
  const float gamb = gL * (1.0f - dif);
  const float gs = sdot >= 0.0f ? gL * (1.0f - amb) : 0.0f;  // clamp_min passes at x >= min
  const float cmu = gmu * mu * (1.0f - mu) * (-a.msharp);
  const float mg = fmaf(mix[2], gm[2], fmaf(mix[1], gm[1], mix[0] * gm[0]));
  const float b_scale = cmu * frcp(Zb);
  float* red = s_red + wave * kRec;
  {
    const float vals[8] = {gs * nrm[0], gs * nrm[1], gs * nrm[2], gamb, loss, 0.0f, 0.0f, 0.0f};
    const float rs = wave_reduce8(vals, lane);
    if ((lane & 7) == 7) red[kSmallMaxM * 8 + (lane >> 3)] = rs;
  }

  // ---- backward sweep 1 at p_final: g_delta_j (colour softmax + mask soft-min), g_p -> g_t
  float gdj[MB], wj[MB];
  float gp[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int j0 = 0; j0 < MB; j0 += kSmallGroup) {
    if (j0 < M) {
#pragma unroll
      for (int j = j0; j < j0 + kSmallGroup; ++j) {
        const float dd = dmin - dl[j];  // <= 0 exactly
        const float w = fexp2(dd * c10l) * invZw;
        const float bt = fexp2(dd * kappa) * b_scale;
        const float4 col = s_col[j];
        const float cgm = fmaf(col.z, gm[2], fmaf(col.y, gm[1], col.x * gm[0]));
        const float gd = fmaf(w * -a.csharp, cgm - mg, bt);
        const float gu = gd * ir[j];
        gp[0] = fmaf(gu, fmaf(0.5f, S.gx[j], p[0]), gp[0]);
        gp[1] = fmaf(gu, fmaf(0.5f, S.gy[j], p[1]), gp[1]);
        gp[2] = fmaf(gu, fmaf(0.5f, S.gz[j], p[2]), gp[2]);
        gdj[j] = gd;
        wj[j] = w;
      }
    }
  }
  const float gt = fmaf(gp[2], d[2], fmaf(gp[1], d[1], gp[0] * d[0]));  // t_final = t + D(p_a)
  const float hs = gt * frcp(sA);
  // ---- sweep 2 at p_approx (alpha = softmax(-k dist_a)) and the per-sphere wave sums
  const float ppa = psq(pa);
#pragma unroll
  for (int j0 = 0; j0 < MB; j0 += kSmallGroup) {
    if (j0 < M) {
#pragma unroll
      for (int j = j0; j < j0 + kSmallGroup; ++j) {
        const float qa = fmaf(pa[2], S.gz[j], fmaf(pa[1], S.gy[j], fmaf(pa[0], S.gx[j], ppa + S.cc[j])));
        const float qac = qclamp(qa, 1e-6f);
        const float ra = frsq(qac);
        const float h = fexp2(fmaf(-kappa, qac * ra, S.kr[j]) - mA) * hs;  // v - mA <= 0 exactly
        const float hu = qa >= 1e-6f ? h * ra : 0.0f;
        const float gu = gdj[j] * ir[j];
        const float ex = fmaf(0.5f, S.gx[j], p[0]), ey = fmaf(0.5f, S.gy[j], p[1]), ez = fmaf(0.5f, S.gz[j], p[2]);
        const float ax = fmaf(0.5f, S.gx[j], pa[0]), ay = fmaf(0.5f, S.gy[j], pa[1]), az = fmaf(0.5f, S.gz[j], pa[2]);
        const float vals[8] = {-fmaf(gu, ex, hu * ax), -fmaf(gu, ey, hu * ay), -fmaf(gu, ez, hu * az), -(gdj[j] + h),
                               wj[j] * gm[0], wj[j] * gm[1], wj[j] * gm[2], 0.0f};
        const float rs = wave_reduce8(vals, lane);
        if ((lane & 7) == 7) red[j * 8 + (lane >> 3)] = rs;
      }
    }
  }
  __syncthreads();

  // ---- the block's partial record [Mpad][8] | 8 scalars (the rm_reduce_partials layout), the
  // four waves summed in order; padding spheres and the unused column 7 are 0
  const int Mpad = a.Mpad;
  const int ncols = Mpad * 8 + 8;
  float* rec = a.partials + blk * a.rec;
  for (int e = tid; e < ncols; e += kBlock) {
    const int src = e < Mpad * 8 ? e : kSmallMaxM * 8 + (e - Mpad * 8);
    const bool zero = e < Mpad * 8 ? ((e >> 3) >= M || (e & 7) == 7) : (e - Mpad * 8) >= 5;
    float v = 0.0f;
    if (!zero) {
      v = s_red[src];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) v += s_red[w * kRec + src];
    }
    if (e == ncols - 1) v = 1.0f;  // scalar 7: live flag (rm_reduce_partials reads every column)
    rec[e] = v;
  }
  if (!sa.final_in_kernel) return;

  // ---- last block: sum the blocks' records in block order and write the gradients
  // (rm_finalize_grads' layout and light-direction Jacobian). Hand-off: every wave drains its
  // stores, the block barrier, one lane's agent-scope release fence and arrival; the block whose
  // arrival is the last acquires and reads (MI355X_MICROARCH.md, inter-workgroup visibility).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's record stores are done
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(sa.arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1 ? 1 : 0;
  }
  __syncthreads();
  if (!s_last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const int nb = gridDim.x;
  const FinalArgs& f = sa.fin;
  for (int e = tid; e < ncols; e += kBlock) {
    // one addition chain per column in block order, eight rows in flight
    float acc = 0.0f;
    for (int b0 = 0; b0 < nb; b0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = a.partials[(long long)min(b0 + u, nb - 1) * a.rec + e];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (b0 + u < nb) acc += v[u];
    }
    s_red[e] = acc;
  }
  __syncthreads();
  for (int e = tid; e < Mpad * 8; e += kBlock) {
    const int j = e >> 3, comp = e & 7;
    if (j >= M || comp == 7) continue;
    float* dst = comp < 3 ? (f.gc ? f.gc + 3 * j + comp : nullptr)
                          : (comp == 3 ? (f.gr ? f.gr + j : nullptr) : (f.gcol ? f.gcol + 3 * j + (comp - 4) : nullptr));
    if (dst) *dst = f.accumulate ? *dst + s_red[e] : s_red[e];
  }
  if (tid == 0) {
    const float* sc = s_red + Mpad * 8;
    if (f.gld) {
      const float l0 = f.light_dir[0], l1 = f.light_dir[1], l2 = f.light_dir[2];
      const float len = sqrtf(l0 * l0 + l1 * l1 + l2 * l2);
      const float ln[3] = {l0 / len, l1 / len, l2 / len};
      const float proj = ln[0] * sc[0] + ln[1] * sc[1] + ln[2] * sc[2];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float gv = (sc[c] - ln[c] * proj) / len;
        f.gld[c] = f.accumulate ? f.gld[c] + gv : gv;
      }
    }
    if (f.gamb) f.gamb[0] = f.accumulate ? f.gamb[0] + sc[3] : sc[3];
    if (f.loss_sum) f.loss_sum[0] = f.accumulate ? f.loss_sum[0] + sc[4] : sc[4];
    __hip_atomic_store(sa.arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
  }
}
