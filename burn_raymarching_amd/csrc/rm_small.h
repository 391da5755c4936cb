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
//    partial records and writes the gradients (write-through record stores, an arrival counter,
//    an agent-scope acquire in the last block; launches of more than kSmallFinalMaxBlocks blocks
//    write partial records for rm_reduce_partials / rm_finalize_grads instead);
//  * the sphere data of the march live in VGPRs as pairs (uniform values: a small launch has one
//    wave per SIMD, registers are free), every sweep handles two spheres per packed instruction
//    over the MB spheres of the kernel's bucket (M rounded up to a multiple of 4: straight-line
//    code the scheduler interleaves; the 0-3 padding spheres sit at x = 1e15 and contribute exact
//    zeros, as in rm_prep_kernel);
//  * every soft-min takes the reference's exact maximum shift (sdf.rs:36-40) per ray: two passes
//    over the spheres held in registers, no wave-uniform path choice, no matrix-core exchange;
//  * the backward keeps one ray per lane and sums each sphere's seven gradient terms over the
//    wave with the transposing 8-value reduction (wave_reduce8), the four waves in LDS in order.
// Deterministic: every sum has a fixed order (lanes, waves, blocks).
// FUSED (rm_train_iteration): the reference loop's whole step in this one launch -- the batch drawn
// and gathered per ray, and the optimizer step run by the last block after the gradient sums;
// with sa.adam = 0 (rm_train_step_sampled, the data-parallel step) the draw, render and gradient
// only, the optimizer left for after the all-reduce.
#pragma once

constexpr int kSmallMaxM = 32;             // spheres handled by the small kernel
#ifndef RM_SMALL_PAR_TOTALS
#define RM_SMALL_PAR_TOTALS 1  // final block: column totals formed once in parallel (0: per use)
#endif
#ifndef RM_SMALL_FIN_BATCH
#define RM_SMALL_FIN_BATCH 32  // record rows in flight per thread in the final block's sums
#endif
constexpr int kSmallFinalMaxBlocks = 128;  // in-kernel final reduction up to this many blocks

struct SmallArgs {
  FinalArgs fin;          // where the last block writes the gradients and the loss
  unsigned* arrivals;     // arrival counter (zero between launches; the last block resets it)
  int final_in_kernel;    // 1: the last block reduces and finalizes; 0: partial records only
  int acquire;            // 1: the last block runs an agent-scope acquire before its loads
  // The fused training iteration (rm_train_iteration; kernel template FUSED): the batch is drawn
  // and gathered in the kernel (rm_sample_kernel's rows: ray i of the call reads row j of the
  // dataset arrays) and the last block runs the optimizer step on the gradient it has summed.
  const float* src_org;
  const float* src_dir;
  const float* src_tgt;
  const int32_t* fg;
  long long num_src, num_fg, n_uniform;
  unsigned long long key;
  float* raw;             // optimizer (opt_small_pre / opt_small_post): raw parameters, moments
  float* m1;
  float* m2;
  int step, with_pen;
  float lr, wd;
  float* loss_penalty;    // nullable
  float* act_out;         // the next render's activated parameters (the scene this launch read)
  float* opt_pre;         // FUSED: [4][kOptPreStride] chain-rule factor and penalty terms per element,
                          // then Adam's two bias corrections (the extra block -> the final block)
  int adam;               // FUSED: 1 -- the extra block and the optimizer step (rm_train_iteration);
                          // 0 -- the drawn batch's gradient only, for an all-reduce (rm_train_step_sampled);
                          // 2 -- that, and the extra block's optimizer part left in opt_pre for the
                          // update after the all-reduce (rm_train_step_sampled_prepared)
};
constexpr int kOptPreStride = 256;  // >= 7 kSmallMaxM + 4 elements
static_assert(7 * kSmallMaxM + 4 <= kOptPreStride, "one opt_pre column per element");

// Per-sphere march data in registers, pair p = spheres (2p, 2p + 1): gx = -2c, cc = |c|^2
// (expansion form, scene.rs:66-71), kr = kappa r (kappa = smooth_k log2 e).
// *dst = v, or *dst += v when accumulating: the load only on the accumulate branch (a select
// would let the compiler issue it anyway, a memory round trip on the last block's tail)
__device__ __forceinline__ void store_or_add(float* dst, float v, int accumulate) {
  if (accumulate) {
    *dst += v;
  } else {
    *dst = v;
  }
}

template <int MB>
struct SmallSpheres {
  f2 gx[MB / 2], gy[MB / 2], gz[MB / 2], cc[MB / 2], kr[MB / 2];
};

// Soft-min scene SDF at p (scene.rs:60-79 + sdf.rs:30-44) in base 2 with the exact per-ray max
// shift: D = -(log2(sum_j 2^(v_j - m)) + m) / kappa, v_j = kappa (r_j - rho_j). RSQ: rho = q rsq(q)
// (the reconnect: backward sweep 2 recomputes the same v_j bit for bit); else rho = sqrt(q).
template <int MB, bool RSQ>
__device__ __forceinline__ float small_softmin(const float p[3], const SmallSpheres<MB>& S, float kappa,
                                               float inv_kappa, float& m_out, float& s_out) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), NK = sp(-kappa);
  f2 v[MB / 2];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < MB / 2; ++i) {
    f2 q = clamp_q(fma2(PZ, S.gz[i], fma2(PY, S.gy[i], fma2(PX, S.gx[i], PP + S.cc[i]))));
    const f2 rho = RSQ ? q * rsq2(q) : sqrt2(q);
    v[i] = fma2(rho, NK, S.kr[i]);
    m = fmaxf(m, fmaxf(v[i].x, v[i].y));
  }
  const f2 MN = sp(m);
  f2 acc = sp(0.0f);
#pragma unroll
  for (int i = 0; i < MB / 2; ++i) acc += exp2v(v[i] - MN);
  const float s = acc.x + acc.y;
  m_out = m;
  s_out = s;
  return -(flog2(fmaxf(s, 1e-8f)) + m) * inv_kappa;
}

// The two lanes of a ray (LPR = 2) exchange their halves with one DPP move (quad_perm 1,0,3,2).
__device__ __forceinline__ float lane_xor1(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));
}

// small_softmin over half of the spheres in each of the two lanes of a ray (LPR = 2): the exact
// maximum of both halves (max is exact), each lane's shifted sum, the two sums added
// (commutative: both lanes get the same bits) -- the march's D, identical in the two lanes.
template <int MBH>
__device__ __forceinline__ float small_softmin_half(const float p[3], const SmallSpheres<MBH>& S, float kappa,
                                                    float inv_kappa) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), NK = sp(-kappa);
  f2 v[MBH / 2];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < MBH / 2; ++i) {
    const f2 q = clamp_q(fma2(PZ, S.gz[i], fma2(PY, S.gy[i], fma2(PX, S.gx[i], PP + S.cc[i]))));
    v[i] = fma2(sqrt2(q), NK, S.kr[i]);
    m = fmaxf(m, fmaxf(v[i].x, v[i].y));
  }
  m = fmaxf(m, lane_xor1(m));
  const f2 MN = sp(m);
  f2 acc = sp(0.0f);
#pragma unroll
  for (int i = 0; i < MBH / 2; ++i) acc += exp2v(v[i] - MN);
  const float sl = acc.x + acc.y;
  const float s = sl + lane_xor1(sl);
  return -(flog2(fmaxf(s, 1e-8f)) + m) * inv_kappa;
}

// The arrival of a block (after its write-through record stores): every storing wave drained
// before the block barrier, one lane's agent-scope add to the launch's counter. True in the block
// that arrives last (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ bool small_arrive(const SmallArgs& sa, int* s_last) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(sa.arrivals, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_last = prev == gridDim.x - 1 ? 1 : 0;
  }
  __syncthreads();
  return *s_last != 0;
}

// The last block: sum the nrows blocks' records and write the gradients (rm_finalize_grads'
// layout and light-direction Jacobian, light_grad: contraction off); FUSED: then the optimizer update on that gradient, with the
// gradient-independent part the launch's extra block left in sa.opt_pre. s_red: the kernel's
// cross-wave LDS buffer (free by now).
template <bool FUSED>
__device__ __forceinline__ void small_final(const KArgs& a, const SmallArgs& sa, int nrows, float* s_red) {
  const int tid = threadIdx.x;
  const int M = a.M, Mpad = a.Mpad;
  const int nneed = M * 8 + 8;  // columns of the real spheres, then the scalars
  auto col_of = [&](int idx) { return idx < M * 8 ? idx : Mpad * 8 + (idx - M * 8); };
  // FUSED: the optimizer's parameters and moments load while the block sums the records
  OptPrefetch pf;
  if constexpr (FUSED) {
    if (sa.adam == 1) pf = opt_prefetch(sa.raw, sa.m1, sa.m2, M);
  }
  // The records are read with write-through-cache (sc1) loads only, stored sc1 by every block,
  // each storing wave drained (vmcnt(0)) before the barrier behind which one lane adds to the one
  // counter whose last add tells this block: the hand-off row of MI355X_MICROARCH.md
  // (inter-workgroup visibility) under which sc1 loads may replace the agent-scope acquire. The
  // acquire is kept (sa.acquire, env RM_SMALL_ACQUIRE=0 drops it): without it the tail measured
  // the same (tools/small_trace.py: 4.96 vs 5.12 us at 128 blocks).
  if (sa.acquire && tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  RM_TRACE(11, __builtin_amdgcn_s_memrealtime());
  // FUSED: the extra block's optimizer part, loaded with the records (the same hand-off)
  [[maybe_unused]] OptPre opre;
  if (FUSED && sa.adam == 1) {
    const int n = 7 * M + 4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = tid + 256 * h;
      float v[4] = {1.0f, 0.0f, 0.0f, 0.0f};
      if (i < n)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] = __hip_atomic_load(sa.opt_pre + k * kOptPreStride + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      opre.e[h] = ElemPre{v[0], v[1], v[2], v[3], 0.0f};
    }
    opre.bias.c1 = __hip_atomic_load(sa.opt_pre + 4 * kOptPreStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    opre.bias.c2 = __hip_atomic_load(sa.opt_pre + 4 * kOptPreStride + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // each needed column is summed by `chains` threads (rows b = k mod chains, in order), the chains
  // then added in order: a fixed order for every launch of this size. The write-through loads
  // miss the local L2 (~1 us each round trip): kFinBatch rows in flight per thread, so that a
  // launch of up to kSmallFinalMaxBlocks blocks takes one or two rounds.
  constexpr int kFinBatch = RM_SMALL_FIN_BATCH;
  const int nb = nrows;
  // A load's address is a 32-bit byte offset from the records' base (saddr form), clamped into
  // the last record instead of branching around the load (a launch's records are
  // nb * rec <= 128 * 264 floats; a clamped row's value is dropped below): three full-rate
  // instructions per load instead of a 64-bit multiply, quarter-rate integer multiplies and an
  // exec-mask branch around each (issuing a thread's 32 loads was part of the sums' critical path)
  const int chains = max(1, min(8, kBlock / nneed));
  const int rec32 = (int)a.rec;
  const int stride = chains * rec32;  // one row of a chain to its next
  const int last_row = (nb - 1) * rec32;
  const char* pbytes = reinterpret_cast<const char*>(a.partials);
  for (int w = tid; w < nneed * chains; w += kBlock) {
    const int idx = w % nneed, ch = w / nneed;
    const int e = (int)col_of(idx);
    float acc = 0.0f;
    for (int b0 = ch; b0 < nb; b0 += kFinBatch * chains) {
      const unsigned off0 = (unsigned)(b0 * rec32 + e);
      float v[kFinBatch];
#pragma unroll
      for (int u = 0; u < kFinBatch; ++u) {
        const unsigned off = min(off0 + (unsigned)(u * stride), (unsigned)(last_row + e));  // floats
        v[u] = __hip_atomic_load(reinterpret_cast<const float*>(pbytes + 4u * off), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int u = 0; u < kFinBatch; ++u)
        if (b0 + u * chains < nb) acc += v[u];
    }
    s_red[ch * nneed + idx] = acc;
  }
  __syncthreads();
  RM_TRACE(2, __builtin_amdgcn_s_memrealtime());
  const FinalArgs& f = sa.fin;
  // a column's total: its chains added in order. RM_SMALL_PAR_TOTALS: every column's total formed
  // once, by all threads in parallel, behind one barrier (the same adds in the same order as
  // forming it in each lane that uses it; s_red holds chains * nneed <= kBlock + 8 floats, the
  // totals go above them)
  static_assert(2 * (kBlock + 32) + 8 <= kWaves * (kSmallMaxM * 8 + 8), "s_red holds the chains and the totals");
#if RM_SMALL_PAR_TOTALS
  float* s_tot = s_red + kBlock + 32;
  for (int idx = tid; idx < nneed; idx += kBlock) {
    float v = s_red[idx];
    for (int ch = 1; ch < chains; ++ch) v += s_red[ch * nneed + idx];
    s_tot[idx] = v;
  }
  __syncthreads();
  auto total = [&](int idx) { return s_tot[idx]; };
#else
  auto total = [&](int idx) {
    float v = s_red[idx];
    for (int ch = 1; ch < chains; ++ch) v += s_red[ch * nneed + idx];
    return v;
  };
#endif
  // FUSED: the gradient also goes to LDS in the packed layout the optimizer reads
  [[maybe_unused]] float* s_gact = nullptr;
  if constexpr (FUSED) {
    __shared__ float s_gact_buf[7 * kSmallMaxM + 4];
    s_gact = s_gact_buf;
  }
  for (int idx = tid; idx < M * 8; idx += kBlock) {
    const int j = idx >> 3, comp = idx & 7;
    if (comp == 7) continue;
    float* dst = comp < 3 ? (f.gc ? f.gc + 3 * j + comp : nullptr)
                          : (comp == 3 ? (f.gr ? f.gr + j : nullptr) : (f.gcol ? f.gcol + 3 * j + (comp - 4) : nullptr));
    const float v = total(idx);
    if (dst) store_or_add(dst, v, f.accumulate);
    if constexpr (FUSED) s_gact[comp < 3 ? 3 * j + comp : (comp == 3 ? 6 * M + j : 3 * M + 3 * j + (comp - 4))] = v;
  }
  // the scalars: lanes 0-2 the light direction's three components (each forms the same
  // projection), lane 3 ambient, loss and the counter reset
  if (tid < 3) {
    if (f.gld) {
      const float sc[3] = {total(M * 8), total(M * 8 + 1), total(M * 8 + 2)};
      const float gv = light_grad(sc, a.light_dir, tid);
      store_or_add(f.gld + tid, gv, f.accumulate);
      if constexpr (FUSED) s_gact[7 * M + tid] = gv;
    }
  } else if (tid == 3) {
    const float s3 = total(M * 8 + 3), s4 = total(M * 8 + 4);
    if constexpr (FUSED) s_gact[7 * M + 3] = s3;
    if (f.gamb) store_or_add(f.gamb, s3, f.accumulate);
    if (f.loss_sum) store_or_add(f.loss_sum, s4, f.accumulate);
    __hip_atomic_store(sa.arrivals, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
  }
  RM_TRACE(9, __builtin_amdgcn_s_memrealtime());
  RM_TRACE(1, __builtin_amdgcn_s_memrealtime());
  if (FUSED && sa.adam == 1) {
    // the optimizer step (rm_optimizer_step: penalties + Adam, train.rs:198) on the gradient just
    // summed (its LDS copy in the packed layout). Every other block has arrived, so nothing reads
    // the activated or raw parameters any more when act_out and raw are overwritten.
    __syncthreads();
    const int n = 7 * M + 4;
    const float g[2] = {tid < n ? s_gact[tid] : 0.0f, tid + 256 < n ? s_gact[tid + 256] : 0.0f};
    opt_small_post(opre, pf, g, sa.raw, sa.m1, sa.m2, M, sa.lr, sa.wd, sa.act_out, nullptr);
    RM_TRACE(10, __builtin_amdgcn_s_memrealtime());
    RM_TRACE(1, __builtin_amdgcn_s_memrealtime());
  }
}

// LPR (lanes per ray, train steps): 2 -- the S march steps run with each ray's spheres split over
// two lanes (128 rays per block, twice the waves: the reference loop's 16,384-ray batch fills
// half of the SIMDs instead of a quarter), then the rays go through LDS to waves 0-1, which run
// the post-march forward and the backward with one ray per lane as for LPR = 1.
template <int MODE, int MB, bool FUSED = false, int LPR = 1>
__global__ __launch_bounds__(kBlock, 1) void rm_small_kernel(const KArgs a, const SmallArgs sa) {
  static_assert(MB % 2 == 0 && MB <= kSmallMaxM, "sphere bucket");
  static_assert(!FUSED || MODE == kTrain, "the fused iteration is a train step");
  static_assert(LPR == 1 || (LPR == 2 && MODE == kTrain && MB % 4 == 0), "split march: train steps");
  constexpr int kRec = kSmallMaxM * 8 + 8;  // per-wave slot of the cross-wave sums
  constexpr int NP = MB / 2;
  constexpr int RPB = kBlock / LPR;         // rays per block
  constexpr int kPostWaves = kWaves / LPR;  // waves of the post-march phases
  __shared__ float4 s_geo[MB];              // {gx, gy, gz, cc}
  __shared__ float4 s_mat[MB];              // {kr, r, 0, 0}
  __shared__ float4 s_col[MB];              // {red, green, blue, 0}
  __shared__ float s_red[kWaves * kRec];    // per-wave sums: [wave][sphere][8] | [wave][8 scalars]
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.M;
  const float kappa = a.k * kLog2e, inv_kappa = 1.0f / kappa;
  // measurement build (-DRM_BLOCK_TRACE): per wave, the s_memrealtime stamps of the phases
  // (0 start, 1 end, 4 sphere data + ray, 5 march, 6 post-march forward, 7 backward sweeps,
  // 8 record + arrival, 11 acquire, 2 record sums, 9 final reduction, 10 optimizer; 3 = block;
  // tools/small_trace.py)
  RM_TRACE(0, __builtin_amdgcn_s_memrealtime());
  RM_TRACE(3, (unsigned long long)blockIdx.x);
  if constexpr (FUSED) {
    // the launch's extra last block: the optimizer's gradient-independent part (snapshot,
    // repulsion rows, chain-rule factors, penalty terms and loss, Adam's bias corrections) on a CU
    // of its own while the ray blocks run, handed to the final block through sa.opt_pre
    // (write-through stores before the arrival, as the records)
    if (sa.adam && blockIdx.x == gridDim.x - 1) {
      const OptPrefetch pf = opt_prefetch(sa.raw, sa.m1, sa.m2, M);
      const OptPre o = opt_small_pre(pf, M, sa.step, sa.with_pen, sa.loss_penalty);
      const int n = 7 * M + 4;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int i = tid + 256 * h;
        if (i < n) {
          const float v[4] = {o.e[h].fac, o.e[h].t0, o.e[h].t1, o.e[h].t2};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            __hip_atomic_store(sa.opt_pre + k * kOptPreStride + i, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (tid == 0) {
        __hip_atomic_store(sa.opt_pre + 4 * kOptPreStride, o.bias.c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sa.opt_pre + 4 * kOptPreStride + 1, o.bias.c2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const bool last = small_arrive(sa, &s_last);
      RM_TRACE(8, __builtin_amdgcn_s_memrealtime());
      RM_TRACE(1, __builtin_amdgcn_s_memrealtime());
      if (last) small_final<FUSED>(a, sa, (int)gridDim.x - 1, s_red);
      return;
    }
  }

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
  long long li = blk * RPB + tid / LPR;
  bool valid = li < a.n_rays;
  long long ri = a.ray_begin + (valid ? li : 0);
  float o[3], d[3];
  int view;
  long long ti;  // the row of the target (setup_ray turns ri into the ray's row)
  if constexpr (FUSED) {  // SceneDataset::sample_batch (dataset.rs:47-82), as rm_sample_kernel
    const unsigned long long r = splitmix64(sa.key + (unsigned long long)(ri + 1) * 0x9E3779B97F4A7C15ull);
    const long long j = ri < sa.n_uniform ? (long long)__umul64hi(r, (unsigned long long)sa.num_src)
                                          : (long long)sa.fg[__umul64hi(r, (unsigned long long)sa.num_fg)];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      o[c] = sa.src_org[3 * j + c];
      d[c] = sa.src_dir[3 * j + c];
    }
    ti = j;
  } else {
    if (a.num_views > 0) setup_ray<true>(a, ri, o, d, view);
    else setup_ray<false>(a, ri, o, d, view);
    ti = ri;
  }
  // train steps: the loss target, loaded here so that its latency (a random row in the fused
  // iteration) hides behind the march instead of opening the backward
  float tgv[3] = {0.0f, 0.0f, 0.0f};
  if constexpr (MODE == kTrain) {
    const float* tgt = FUSED ? sa.src_tgt : a.targets;
    if (valid) {
#pragma unroll
      for (int c = 0; c < 3; ++c) tgv[c] = tgt[3 * ti + c];
    }
  }
  __syncthreads();
  auto load_spheres = [&](auto& S, int first) {  // pairs of spheres first, first + 1, ... from LDS
    constexpr int n = sizeof(S.gx) / sizeof(S.gx[0]);
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const float4 g0 = s_geo[first + 2 * i], g1 = s_geo[first + 2 * i + 1];
      S.gx[i] = f2{g0.x, g1.x};
      S.gy[i] = f2{g0.y, g1.y};
      S.gz[i] = f2{g0.z, g1.z};
      S.cc[i] = f2{g0.w, g1.w};
      S.kr[i] = f2{s_mat[first + 2 * i].x, s_mat[first + 2 * i + 1].x};
    }
  };

  RM_TRACE(4, __builtin_amdgcn_s_memrealtime());
  // ---- march: t <- (t + sdf(o + d t)).detach(), S times (renderer_diff.rs:20-26)
  float t = 0.0f;
  if constexpr (LPR == 2) {
    SmallSpheres<MB / 2> SH;  // this lane's half: spheres (tid & 1) * MB / 2 ...
    load_spheres(SH, (tid & 1) * (MB / 2));
    for (int st = 0; st < a.steps; ++st) {
      const float p[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
      t = fminf(t + small_softmin_half<MB / 2>(p, SH, kappa, inv_kappa), kTMax);
    }
    // the rays to waves 0-1, one per lane: origin, direction, t, rows
    __shared__ float s_rf[10][RPB];
    __shared__ long long s_rr[2][RPB];
    const int rl = tid >> 1;
    if ((tid & 1) == 0) {
      s_rf[0][rl] = o[0];
      s_rf[1][rl] = o[1];
      s_rf[2][rl] = o[2];
      s_rf[3][rl] = d[0];
      s_rf[4][rl] = d[1];
      s_rf[5][rl] = d[2];
      s_rf[6][rl] = t;
      s_rf[7][rl] = tgv[0];
      s_rf[8][rl] = tgv[1];
      s_rf[9][rl] = tgv[2];
      s_rr[0][rl] = ri;
      s_rr[1][rl] = ti;
    }
    __syncthreads();
    // waves 0-1: ray tid of the block; waves 2-3 repeat the rays of waves 0-1 as invalid rays
    // (no outputs, zero seeds, their sums not added: block_sum takes waves 0-1), so that every
    // loop and barrier below keeps the full block
    const int r2 = tid % RPB;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      o[c] = s_rf[c][r2];
      d[c] = s_rf[3 + c][r2];
    }
    t = s_rf[6][r2];
#pragma unroll
    for (int c = 0; c < 3; ++c) tgv[c] = s_rf[7 + c][r2];
    ri = s_rr[0][r2];
    ti = s_rr[1][r2];
    li = blk * RPB + r2;
    valid = li < a.n_rays && wave < kPostWaves;
  }
  SmallSpheres<MB> S;
  load_spheres(S, 0);
  if constexpr (LPR == 1) {
    if (MODE == kBwd && a.t_in != nullptr) {
      t = a.t_in[ri];
    } else {
      for (int st = 0; st < a.steps; ++st) {
        const float p[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
        float m, s;
        t = fminf(t + small_softmin<MB, false>(p, S, kappa, inv_kappa, m, s), kTMax);
      }
    }
  }
  if (MODE == kFwd && a.t_out != nullptr && valid) a.t_out[ri] = t;
  RM_TRACE(5, __builtin_amdgcn_s_memrealtime());

  // ---- reconnect: t_final = t + sdf(p_approx) (renderer_diff.rs:30-39)
  const float pa[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
  float mA, sA;
  const float Da = small_softmin<MB, true>(pa, S, kappa, inv_kappa, mA, sA);
  const float tf = t + Da;
  const float p[3] = {fmaf(d[0], tf, o[0]), fmaf(d[1], tf, o[1]), fmaf(d[2], tf, o[2])};

  // ---- shade sweep at p_final: colour softmax over -csharp delta (renderer_diff.rs:64-82),
  // mask soft-min over -k delta (renderer_diff.rs:86-90) and the detached normal as the eps -> 0
  // limit of scene.rs:81-128 (2 eps grad D, grad D = sum beta_j (p - c_j) / rho_j), two passes:
  // the exact minimum delta, then the sums relative to it (exponents <= 0 exactly)
  const float c10l = a.csharp * kLog2e;
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), HALF = sp(0.5f);
  f2 dl[NP], ir[NP];
  float dmin = INFINITY;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const f2 q = fma2(PZ, S.gz[i], fma2(PY, S.gy[i], fma2(PX, S.gx[i], PP + S.cc[i])));
    const f2 qc = clamp_q(q);
    const f2 r = rsq2(qc);
    dl[i] = qc * r - f2{s_mat[2 * i].y, s_mat[2 * i + 1].y};  // delta_j = rho_j - r_j
    // clamp_min(1e-6) gate: a clamped distance is constant and carries no gradient
    ir[i] = f2{q.x >= 1e-6f ? r.x : 0.0f, q.y >= 1e-6f ? r.y : 0.0f};
    dmin = fminf(dmin, fminf(dl[i].x, dl[i].y));
  }
  const f2 DM = sp(dmin), CL = sp(c10l), KA = sp(kappa);
  f2 Zw2 = sp(0.0f), Zb2 = sp(0.0f), C2[3] = {sp(0.0f), sp(0.0f), sp(0.0f)}, G2[3] = {sp(0.0f), sp(0.0f), sp(0.0f)};
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const f2 dd = DM - dl[i];
    const f2 ew = exp2v(dd * CL), eb = exp2v(dd * KA);
    const float4 c0 = s_col[2 * i], c1 = s_col[2 * i + 1];
    Zw2 += ew;
    C2[0] = fma2(ew, f2{c0.x, c1.x}, C2[0]);
    C2[1] = fma2(ew, f2{c0.y, c1.y}, C2[1]);
    C2[2] = fma2(ew, f2{c0.z, c1.z}, C2[2]);
    Zb2 += eb;
    const f2 wr = eb * ir[i];
    G2[0] = fma2(wr, fma2(HALF, S.gx[i], PX), G2[0]);
    G2[1] = fma2(wr, fma2(HALF, S.gy[i], PY), G2[1]);
    G2[2] = fma2(wr, fma2(HALF, S.gz[i], PZ), G2[2]);
  }
  const float Zw = Zw2.x + Zw2.y, Zb = Zb2.x + Zb2.y;
  const float te = 2.0f * a.eps * frcp(Zb);
  const float nx = te * (G2[0].x + G2[0].y), ny = te * (G2[1].x + G2[1].y), nz = te * (G2[2].x + G2[2].y);
  const float inv_len = frsq(fmaf(nz, nz, fmaf(ny, ny, fmaf(nx, nx, 1e-6f))));
  const float nrm[3] = {nx * inv_len, ny * inv_len, nz * inv_len};
  // ---- lighting (renderer_diff.rs:48-62)
  const float amb = a.ambient[0];
  float ldn[3];
  light_unit(a.light_dir, ldn);
  const float sdot = fmaf(nrm[2], ldn[2], fmaf(nrm[1], ldn[1], nrm[0] * ldn[0]));
  const float dif = fmaxf(sdot, 0.0f);
  const float Lgt = fmaf(dif, 1.0f - amb, amb);
  const float Df = dmin - flog2(fmaxf(Zb, 1e-8f)) * inv_kappa;
  const float invZw = frcp(Zw);
  const float mix[3] = {(C2[0].x + C2[0].y) * invZw, (C2[1].x + C2[1].y) * invZw, (C2[2].x + C2[2].y) * invZw};
  const float mu = frcp(1.0f + fexp2(a.msharp * kLog2e * Df));  // sigmoid(-msharp D)
  const float scale = Lgt * mu;
  const float outv[3] = {mix[0] * scale, mix[1] * scale, mix[2] * scale};
  if (MODE != kBwd && a.out != nullptr && valid) {
    a.out[3 * ri] = outv[0];
    a.out[3 * ri + 1] = outv[1];
    a.out[3 * ri + 2] = outv[2];
  }
  RM_TRACE(6, __builtin_amdgcn_s_memrealtime());
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
      const float t0 = tgv[0], t1 = tgv[1], t2 = tgv[2];
      const float W = (t0 + t1 + t2) > 0.01f ? 10.0f : fmaf(progress_of(a), 4.0f, 1.0f);
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
  f2 gdj[NP], wj[NP];
  f2 gp2[3] = {sp(0.0f), sp(0.0f), sp(0.0f)};
  const f2 G0 = sp(gm[0]), G1 = sp(gm[1]), G2c = sp(gm[2]), MG = sp(mg), NCS = sp(-a.csharp), IZ = sp(invZw),
           BS = sp(b_scale);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const f2 dd = DM - dl[i];  // <= 0 exactly
    const f2 w = exp2v(dd * CL) * IZ;
    const f2 bt = exp2v(dd * KA) * BS;
    const float4 c0 = s_col[2 * i], c1 = s_col[2 * i + 1];
    const f2 cgm = fma2(f2{c0.z, c1.z}, G2c, fma2(f2{c0.y, c1.y}, G1, f2{c0.x, c1.x} * G0));
    const f2 gd = fma2(w * NCS, cgm - MG, bt);
    const f2 gu = gd * ir[i];
    gp2[0] = fma2(gu, fma2(HALF, S.gx[i], PX), gp2[0]);
    gp2[1] = fma2(gu, fma2(HALF, S.gy[i], PY), gp2[1]);
    gp2[2] = fma2(gu, fma2(HALF, S.gz[i], PZ), gp2[2]);
    gdj[i] = gd;
    wj[i] = w;
  }
  const float gp[3] = {gp2[0].x + gp2[0].y, gp2[1].x + gp2[1].y, gp2[2].x + gp2[2].y};
  const float gt = fmaf(gp[2], d[2], fmaf(gp[1], d[1], gp[0] * d[0]));  // t_final = t + D(p_a)
  // ---- sweep 2 at p_approx (alpha = softmax(-k dist_a)) and the per-sphere wave sums
  const f2 AX = sp(pa[0]), AY = sp(pa[1]), AZ = sp(pa[2]), AP = sp(psq(pa)), NK = sp(-kappa), MA = sp(mA),
           HS = sp(gt * frcp(sA));
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const f2 qa = fma2(AZ, S.gz[i], fma2(AY, S.gy[i], fma2(AX, S.gx[i], AP + S.cc[i])));
    const f2 qac = clamp_q(qa);
    const f2 ra = rsq2(qac);
    const f2 h = exp2v(fma2(qac * ra, NK, S.kr[i]) - MA) * HS;  // v - mA <= 0 exactly
    const f2 hr = h * ra;
    const f2 hu = f2{qa.x >= 1e-6f ? hr.x : 0.0f, qa.y >= 1e-6f ? hr.y : 0.0f};
    const f2 gu = gdj[i] * ir[i];
    const f2 ex = fma2(HALF, S.gx[i], PX), ey = fma2(HALF, S.gy[i], PY), ez = fma2(HALF, S.gz[i], PZ);
    const f2 ax = fma2(HALF, S.gx[i], AX), ay = fma2(HALF, S.gy[i], AY), az = fma2(HALF, S.gz[i], AZ);
    const f2 vc[3] = {-fma2(gu, ex, hu * ax), -fma2(gu, ey, hu * ay), -fma2(gu, ez, hu * az)};
    const f2 vr = -(gdj[i] + h);
    const f2 vl[3] = {wj[i] * G0, wj[i] * G1, wj[i] * G2c};
    const float va[8] = {vc[0].x, vc[1].x, vc[2].x, vr.x, vl[0].x, vl[1].x, vl[2].x, 0.0f};
    const float vb[8] = {vc[0].y, vc[1].y, vc[2].y, vr.y, vl[0].y, vl[1].y, vl[2].y, 0.0f};
    const float ra0 = wave_reduce8(va, lane), rb0 = wave_reduce8(vb, lane);
    if ((lane & 7) == 7) {
      red[(2 * i) * 8 + (lane >> 3)] = ra0;
      red[(2 * i + 1) * 8 + (lane >> 3)] = rb0;
    }
  }
  RM_TRACE(7, __builtin_amdgcn_s_memrealtime());
  __syncthreads();

  // ---- the block's partial record [Mpad][8] | 8 scalars (the rm_reduce_partials layout), the
  // four waves summed in order; padding spheres and the unused column 7 are 0. For the in-kernel
  // final reduction the stores are write-through (sc1) and only the columns it reads are written.
  const int Mpad = a.Mpad;
  const int ncols = Mpad * 8 + 8;
  const int nneed = M * 8 + 8;  // columns of the real spheres, then the scalars
  float* rec = a.partials + blk * a.rec;
  auto col_of = [&](int idx) { return idx < M * 8 ? idx : Mpad * 8 + (idx - M * 8); };
  auto block_sum = [&](int e) {  // record column e: the four waves in order
    const int src = e < Mpad * 8 ? e : kSmallMaxM * 8 + (e - Mpad * 8);
    const bool zero = e < Mpad * 8 ? ((e >> 3) >= M || (e & 7) == 7) : (e - Mpad * 8) >= 5;
    float v = 0.0f;
    if (!zero) {
      v = s_red[src];
#pragma unroll
      for (int w = 1; w < kPostWaves; ++w) v += s_red[w * kRec + src];
    }
    return e == ncols - 1 ? 1.0f : v;  // scalar 7: live flag (rm_reduce_partials reads every column)
  };
  if (!sa.final_in_kernel) {
    for (int e = tid; e < ncols; e += kBlock) rec[e] = block_sum(e);
    return;
  }
  for (int idx = tid; idx < nneed; idx += kBlock) {
    const int e = col_of(idx);
    __hip_atomic_store(rec + e, block_sum(e), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

  const bool last = small_arrive(sa, &s_last);
  RM_TRACE(8, __builtin_amdgcn_s_memrealtime());
  RM_TRACE(1, __builtin_amdgcn_s_memrealtime());
  if (!last) return;
  small_final<FUSED>(a, sa, FUSED && sa.adam ? (int)gridDim.x - 1 : (int)gridDim.x, s_red);
}

// The update after an all-reduce when the sampled launch's extra block prepared it
// (rm_train_step_sampled_prepared -> rm_optimizer_step): rm_optimizer_small's opt_small_post on the
// gradient-independent part read from opt_pre -- the values rm_optimizer_small would compute, so
// the same bits.
__global__ __launch_bounds__(256) void rm_optimizer_post_small(float* __restrict__ raw, const float* __restrict__ gact,
                                                               float* __restrict__ m1, float* __restrict__ m2, int M,
                                                               float lr, float wd, float* __restrict__ act_out,
                                                               _Float16* __restrict__ col_h_out,
                                                               const float* __restrict__ opt_pre) {
  const OptPrefetch pf = opt_prefetch(raw, m1, m2, M);
  const int n = 7 * M + 4, tid = (int)threadIdx.x;
  OptPre o;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = tid + 256 * h;
    float v[4] = {1.0f, 0.0f, 0.0f, 0.0f};
    if (i < n)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = opt_pre[k * kOptPreStride + i];
    o.e[h] = ElemPre{v[0], v[1], v[2], v[3], 0.0f};
  }
  o.bias.c1 = opt_pre[4 * kOptPreStride];
  o.bias.c2 = opt_pre[4 * kOptPreStride + 1];
  const float g[2] = {tid < n ? gact[tid] : 0.0f, tid + 256 < n ? gact[tid + 256] : 0.0f};
  opt_small_post(o, pf, g, raw, m1, m2, M, lr, wd, act_out, col_h_out);
}
