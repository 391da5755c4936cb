// rm_device.h -- device-side building blocks of the gfx950 render kernels.
//
// Everything here is written for CDNA4 wave64: native transcendentals
// (v_exp_f32 / v_log_f32 / v_sqrt_f32 / v_rsq_f32 / v_rcp_f32), and a
// transposing 8-value wave reduction built from v_permlane32_swap,
// v_permlane16_swap and DPP row ops (no LDS round trip, no ds_swizzle).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rm {

#ifndef RM_BLOCK
#define RM_BLOCK 256
#endif
constexpr int kBlock = RM_BLOCK;         // threads per block (256 = 4 waves)
#ifndef RM_MIN_WAVES
#define RM_MIN_WAVES 4
#endif
constexpr int kMinWavesPerSimd = RM_MIN_WAVES;  // register budget: 4 -> <= 128 VGPRs
constexpr int kWaves = kBlock / 64;
constexpr int kSphereAlign = 32;         // M is padded to a multiple of this
constexpr int kChunkBwd = 32;            // spheres per backward partial-combine chunk
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kSafeRho = 4e-3f;        // rho >= this => max(q, 1e-6) is a no-op (q >= 1.6e-5)
constexpr float kPadCenter = 1e15f;      // padding sphere center x: distance ~1e15 -> exp() underflows to 0
// March t is capped here: a ray 1e15 from the scene has mask (and out, and every gradient term)
// exactly 0, and the cap keeps |p|^2 and the k^2-scaled matrix-core operands finite. (Rays that
// leave the scene radially double their distance every step: without the cap t overflows to inf
// after ~120 steps and the fp32 arithmetic turns into NaN; the reference's own march does.)
constexpr float kTMax = 1e15f;
// A live wave's post-march forward and backward sweeps in march-step units (the cost-ordered
// dispatch's estimate; tools/bench_parts.py: ~8-10).
#ifndef RM_POST_COST
#define RM_POST_COST 10
#endif
constexpr int kPostCost = RM_POST_COST;

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float flog2(float x) { return __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float frsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float u2f(unsigned u) { return __uint_as_float(u); }
__device__ __forceinline__ unsigned f2u(float f) { return __float_as_uint(f); }

// a+b where lanes [0,32) of the result hold (a_lo + a_hi) and lanes [32,64) hold
// (b_lo + b_hi): one v_permlane32_swap + one add halves two values over lane bit 5.
__device__ __forceinline__ float swap32_sum(float a, float b) {
  auto r = __builtin_amdgcn_permlane32_swap(f2u(a), f2u(b), false, false);
  return u2f(r[0]) + u2f(r[1]);
}
// Same over lane bit 4 (rows of 16): rows 0/2 keep a, rows 1/3 keep b.
__device__ __forceinline__ float swap16_sum(float a, float b) {
  auto r = __builtin_amdgcn_permlane16_swap(f2u(a), f2u(b), false, false);
  return u2f(r[0]) + u2f(r[1]);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, true));
}

// Transposing wave reduction of 8 per-lane values a[0..7] over all 64 lanes.
// Result: lane l with (l & 7) == 7 holds sum over lanes of a[l >> 3].
// 18 wave instructions for 8 sums (a per-value butterfly would take 48).
__device__ __forceinline__ float wave_reduce8(const float (&a)[8], int lane) {
  // bit 5: pairs (0,4) (1,5) (2,6) (3,7)
  float b0 = swap32_sum(a[0], a[4]);  // lanes<32: a0, lanes>=32: a4
  float b1 = swap32_sum(a[1], a[5]);
  float b2 = swap32_sum(a[2], a[6]);
  float b3 = swap32_sum(a[3], a[7]);
  // bit 4: rows 0..3 of c0 = a0 a2 a4 a6, of c1 = a1 a3 a5 a7
  float c0 = swap16_sum(b0, b2);
  float c1 = swap16_sum(b1, b3);
  // bit 3: within each row, lanes 0-7 keep c0, lanes 8-15 keep c1 (row_ror:8 == xor 8)
  const bool hi8 = (lane & 8) != 0;
  float keep = hi8 ? c1 : c0;
  float send = hi8 ? c0 : c1;
  float d = keep + dpp<0x128>(send);
  // bits 2..0: shift-adds inside each 8-lane group; lane 7 of the group ends with the total
  d = d + dpp<0x114>(d);  // row_shr:4
  d = d + dpp<0x112>(d);  // row_shr:2
  d = d + dpp<0x111>(d);  // row_shr:1
  return d;
}

// ---- camera ----------------------------------------------------------------
// Basis of create_camera_rays (camera.rs:41-52), computed on the host in fp32.
struct CamBasis {
  float eye[3];
  float right[3];
  float up[3];
  float fwd[3];
  float half_w, half_h;
};

// camera.rs:58-78 for pixel (x, y), bit-identical to the reference's f32 loop:
//  * no FMA contraction (hipcc contracts by default and __fmul_rn/__fadd_rn are plain * and +,
//    so only the pragma stops it);
//  * f32 division is correctly rounded on gfx950, but sqrtf/__fsqrt_rn lower to v_sqrt_f32,
//    which is not (measured: 14.9% of inputs in [1,4) off by 1 ulp); the f64 sqrt rounded to
//    f32 is exact. Once per ray: free.
__device__ __forceinline__ void camera_ray(const CamBasis& c, int x, int y, int W, int H, float o[3],
                                           float d[3]) {
#pragma clang fp contract(off)
  const float u = ((float)x / (float)W) * 2.0f - 1.0f;
  const float v = -(((float)y / (float)H) * 2.0f - 1.0f);
  const float rs = u * c.half_w, us = v * c.half_h;
  const float dx = c.right[0] * rs + c.up[0] * us + c.fwd[0];
  const float dy = c.right[1] * rs + c.up[1] * us + c.fwd[1];
  const float dz = c.right[2] * rs + c.up[2] * us + c.fwd[2];
  const float len = (float)__builtin_sqrt((double)(dx * dx + dy * dy + dz * dz));
  d[0] = dx / len;
  d[1] = dy / len;
  d[2] = dz / len;
  o[0] = c.eye[0];
  o[1] = c.eye[1];
  o[2] = c.eye[2];
}

}  // namespace rm
