// rm_kernels.hip -- MI355X (gfx950) kernels of the differentiable SDF-sphere raymarcher
// and the C ABI declared in include/raymarch.h.
//
// Hot path replaced: render_diff (renderer_diff.rs:6-91) and its burn-autodiff
// backward (train.rs:189-190). One thread owns one ray for the whole pipeline:
//
//   in-kernel camera ray (camera.rs:58-78), 16x16 pixel tiles per block, centre-out dispatch
//   S fixed soft-min march steps          (renderer_diff.rs:20-26, scene.rs:60-79, sdf.rs:30-44)
//     squared distances on the matrix cores (bf16 three-way splits, lse_mfma), sqrt/exp2 on
//     the vector units; waves whose rays provably escape leave early (exact)
//   gradient reconnect sweep at p_approx  (renderer_diff.rs:28-39)
//   detached normal: one soft-min gradient sweep, the eps -> 0 limit of the six central
//     differences of scene.rs:81-128 (renderer.rs mode: the six taps)
//   Lambert + ambient                     (renderer_diff.rs:48-62)
//   softmax colour blend + mask soft-min  (renderer_diff.rs:64-90), one shared sweep
//   [train] weighted-L1 seed              (training.rs:17-34)
//   [bwd]   analytic backward: sweep at p_final, then at p_approx
//
// Sphere records are built once per call (rm_prep_kernel) and read through the constant
// address space into SGPRs (vector sweeps, two spheres per packed instruction) or as bf16
// MFMA fragments (march). The soft-min log-sum-exp runs in base 2 on v_exp_f32/v_log_f32 with
// the cheapest provably safe shift. Per-sphere gradients are summed over the 64 rays of a
// wave with a transposing permlane/DPP reduction, over the live waves in LDS, and over
// workgroups in a fixed order by rm_reduce_partials (deterministic; no floating-point
// atomics). DESIGN.md §4 has the details and the measurements.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdarg>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/raymarch.h"
#include "rm_device.h"

#ifndef RM_PRIO_RAMP
// s_setprio ramp over the march / post-march / backward phases: paid off when one launch filled
// the GPU once (it evened out the co-resident waves' finish); with 10 views per launch and
// partly-dead blocks backfilled it costs 4 % (1094 vs 1141 Mrays/s), so it is off by default.
#define RM_PRIO_RAMP 0
#endif
#ifndef RM_BWD_TRANSPOSED
#define RM_BWD_TRANSPOSED 1  // backward sweeps with one sphere per lane (0: one ray per lane)
#endif
#ifndef RM_BWD_PSQ_REG
#define RM_BWD_PSQ_REG 0  // backward sweeps form |p|^2 from p in registers (1) or read it from LDS (0)
#endif
#ifndef RM_DEAD_EARLY
// backward modes: a wave whose rays all escaped ends at the hand-off instead of waiting at its
// barrier (A/B switch; measured equal, Appendix A of DESIGN.md)
#define RM_DEAD_EARLY 0
#endif
#ifndef RM_MARCH_SCHED
#define RM_MARCH_SCHED 1  // scheduling barriers in the matrix-core march loop (0: compiler's order)
#endif
#if RM_MARCH_SCHED
#define RM_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define RM_SCHED_BARRIER() ((void)0)
#endif
#ifndef RM_MARCH_BUFLOAD
#define RM_MARCH_BUFLOAD 1  // matrix-core fragments by buffer loads (0: global loads)
#endif
#ifndef RM_MARCH_PK
#define RM_MARCH_PK 1  // lse_mfma accumulates with v_pk_fma_f32 (two chains per ray; 0: one fma chain)
#endif
#ifndef RM_MFMA32
#define RM_MFMA32 0  // the march's matrix-core tiles as v_mfma_f32_32x32x16_bf16 (32 spheres x 32 rays)
#endif
#ifndef RM_CYCLE_MAX
#define RM_CYCLE_MAX 2  // longest period (2..4) the march's cycle exit detects (3, 4: no measurable gain)
#endif
#ifndef RM_HEAVY_PRIO
#define RM_HEAVY_PRIO 0  // s_setprio(2) for the blocks of the RM_HEAVY_PRIO dearest cost classes
#endif
#ifndef RM_ORDER_CLASSES
#define RM_ORDER_CLASSES 16  // cost classes of the cost-ordered dispatch (order_append)
#endif
// ints between the three list sets' class counts and before the turn word: each on cache lines of
// its own (every block of a launch reads the turn and the previous set's counts while the blocks'
// appends hit the current set's counts with atomics; sharing a 128-byte line made every launch
// that appended to the set next to the turn word 50 % slower at C2: tools/order_probe.py)
#ifndef RM_ORDER_CLS_STRIDE
// ints between a set's class counts: each class on a 128-byte line of its own, as the reduction's
// arrival counters below (both: C2cj 4348-4404 vs 4305-4315 Mrays/s with neither, the metric
// equal; tools/gpu_ab.sh, profiles/r05e_ab.txt)
#define RM_ORDER_CLS_STRIDE 32
#endif
#ifndef RM_ORDER_CNT_STRIDE
#define RM_ORDER_CNT_STRIDE (RM_ORDER_CLASSES * RM_ORDER_CLS_STRIDE > 64 ? RM_ORDER_CLASSES * RM_ORDER_CLS_STRIDE : 64)
#endif
static_assert(RM_ORDER_CNT_STRIDE >= RM_ORDER_CLASSES * RM_ORDER_CLS_STRIDE && RM_ORDER_CNT_STRIDE % 32 == 0,
              "128-byte lines per set");
#ifndef RM_RED_ARR_STRIDE
#define RM_RED_ARR_STRIDE 32  // unsigneds between rm_reduce_partials' arrival counters: a 128-byte line each
#endif

namespace rm {

// kRender: the non-differentiable target renderer of renderer.rs:4-80 (generate.rs)
enum Mode { kFwd = 0, kBwd = 1, kTrain = 2, kRender = 3 };

// bounds the partial-gradient workspace per launch: 16 views of 512x512
// 128 views of 512 x 512 in one launch (per-launch ramp-down and the per-call record, origin
// and reduction launches amortised over all the views of a step)
constexpr int kMaxBlocksPerLaunch = 131072 * (256 / kBlock);
// camera bases carried in the kernel arguments; calls with more views read a device table
constexpr int kInlineCams = 16;
// automatic split march (RM_MARCH_SPLIT): from kSplitMinSpheres spheres for launches of at most
// kSplitMaxRays rays (about one fill of the GPU: 1024 resident 256-ray blocks), from
// kSplitMinSpheresWide for launches of at most kSplitMaxRaysWide (four fills) -- measured
// (tools/gpu_split_sweep.sh): split wins at 1 view from 256 spheres and at 4 views of 512x512
// from 512, loses at 10 views of 256 spheres and at 4 views of 1024x1024
constexpr int kSplitMinSpheres = 256;
constexpr int kSplitMinSpheresWide = 512;
constexpr long long kSplitMaxRaysWide = 1048576;
#ifndef RM_SPLIT_WAVES
#define RM_SPLIT_WAVES 4
#endif
#ifndef RM_SPLIT_MIN_WAVES
#define RM_SPLIT_MIN_WAVES 3  // register budget of the split kernels (waves per SIMD): 3 = 168 VGPRs, no
                              // spills (4: 128 VGPRs, 4-12 VGPR spills, 20 B/lane scratch; C5 equal either way)
#endif
#ifndef RM_CONT_MIN_WAVES
#define RM_CONT_MIN_WAVES RM_SPLIT_MIN_WAVES  // register budget of the split continuation kernel
#endif
constexpr int kSplitWaves = RM_SPLIT_WAVES;  // waves per ray group of the split march (2 or 4)
static_assert(kSplitWaves == 2 || kSplitWaves == 4, "split blocks have 2 or 4 waves");
#ifndef RM_SPLIT_RAYS
#define RM_SPLIT_RAYS 32  // (same box, the work-unit backward: C5 +3.5 %, C5g +5 % against 64)
#endif
// Rays per split block (64, 32 or 16). Below 64 every wave of the block holds each of its rays
// 64 / kSplitRays times (lane l and l + kSplitRays carry the same ray, bit for bit) and the
// march's matrix-core tiles run kSplitRays / 16 column blocks instead of 4: a march step of a
// block costs its waves kSplitRays / 64 of the 64-ray step, so heavy rays hold their SIMDs for
// shorter and the blocks that march to the end are smaller work units (configs[4]).
constexpr int kSplitRays = RM_SPLIT_RAYS;
static_assert(kSplitRays == 64 || kSplitRays == 32 || kSplitRays == 16, "split blocks hold 64, 32 or 16 rays");
constexpr int kSplitCB = kSplitRays / 16;  // column blocks of 16 rays in the split march's tiles
constexpr int kContClasses = 4;  // classes of the split continuation's block lists
constexpr long long kSplitMaxRays = 262144;
#ifndef RM_REDUCE_SEGS
#define RM_REDUCE_SEGS 128
#endif
constexpr int kReduceSegs = RM_REDUCE_SEGS;  // block segments of the reduction (128: 12.6 + 6.9 us at 10 views vs 20.3 + 4.9 with 64)

struct KArgs {
  // rays: array mode (org/dir) or camera mode (cams)
  const float* org;
  const float* dir;
  long long ray_begin;  // first ray of this launch
  long long n_rays;     // rays in this launch
  int width, height, num_views;
  int tiling;  // camera mode pixel order: 2 = 16x16 tile per block (8x8 per wave), 0 = rows
  int cull;    // skip blocks whose rays provably escape the scene (RM_MARCH_SKIP_ESCAPED)
  float cull_min_d;  // scene distance at which the silhouette mask is exactly 0
  float lse_slack;  // ln(M) / k (rounded up): the hard min exceeds the soft-min by at most this
  unsigned long long* stats;  // nullable: [0] += 1 per escaped (skipped) block, [1] exited waves,
                              // [2] march steps saved, [3] RM_LANE_STATS, [4] / [5] rays the two
                              // backward sweeps run for (non-zero seeds)
  float gone_d;               // > 0: rays that provably escape past this distance are `gone` (see the march)
  int early_exit;             // waves whose rays are all gone stop marching
  int split;                  // split march (RM_MARCH_SPLIT): 64 rays per block, a quarter of the spheres per wave
  int mfma;                   // march sums on the matrix cores (lse_mfma) instead of lse_weighted
  int shift_max;              // RM_MARCH_FORCE_MAX_SHIFT: every march step takes the running-max shift
  const int* esc_flags;       // nullable: per-block escape flags of this launch (rm_escape_kernel)
  const int* block_order;     // nullable: heavy-first dispatch order of the tiles of a view (ray_block)
  int order_views, order_tiles;
  // cost-ordered dispatch: [class][kMaxBlocksPerLaunch] block lists + [class] counts of the
  // previous launch (read, nullable), of this launch (appended, nullable) and the counts to clear
  // for the next launch (nullable)
  const int* olist_r;
  const int* ocnt_r;
  int* olist_w;
  int* ocnt_w;
  int* ocnt_z;
  // nullable: the device word naming the list set this launch appends to (0..2); with it the five
  // pointers above point to set 0 and the launch picks its sets from the word (read: the set
  // before, clear: the set after), and the call's reduction advances the word -- the rotation
  // lives on the device, so a launch captured in a hipGraph keeps rotating when replayed
  const int* oturn;
  CamBasis cams[kInlineCams];  // views <= kInlineCams
  const CamBasis* cams_dev;    // more views: the bases in device memory (cams unused), else NULL
  // activated scene
  const float* centers;
  const float* colors;
  const _Float16* colors_h;  // RM_MARCH_COLOR_F16: the colours as IEEE half [M,3] (colors is then NULL)
  const float* radius;
  const float* light_dir;
  const float* ambient;
  int M, Mpad;
  const float4* rec_buf;  // sphere records of this call (rm_prep_kernel), see Lds
  float* origin;  // camera mode, nullable: per view, the first march step's D at the eye (write_origins)
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
  const rm_step_scalars* sdev;  // nullable (rm_bind_step_scalars): progress = index / total from here
  float light_fixed[3];  // kRender: renderer.rs:27-32 light, normalised on the host in f32
  float* dbg;       // optional per-ray intermediates [n][16] (diagnostics; see rm_debug_intermediates)
  float* partials;  // [gridDim.x][rec], rec = Mpad*8 + 8
  long long rec;
  // Continuation of a split launch (split_cont_steps, see run()): with cont_cap > 0 a block whose
  // rays still march at step cont_cap saves its march state, appends its logical block to
  // cont_list_w and ends; a launch with cont_resume = that step runs the saved blocks
  // (cont_list[0..*cont_count)) from there (and may defer again at its own cont_cap). The lists
  // are kContClasses class lists of cont_stride entries each, with kContClasses counts: a deferred
  // block goes to the class of the march steps its slowest ray is predicted to need (the most
  // first), and a continuation launch runs the classes in order -- the blocks likely to march to
  // the end start first.
  // cont_state: [7][cont_rays] per ray (t, lb, D_prev, t one and two steps back, gone, rho_lb) then
  // [blocks][2] per block (choice history, steps saved).
  int cont_cap, cont_resume;
  float* cont_state;
  const int* cont_list;
  const int* cont_count;
  int* cont_list_w;
  int* cont_count_w;
  int cont_stride;   // entries per class list
  int cont_order;    // 0: every deferred block in class 0 (arrival order)
  long long cont_rays;
  // Ray mode (split launches; RM_RAY_MODE): every march step takes the scene-uniform fixed shift
  // (the running maximum where the scene does not admit it), so a ray's step is a function of its
  // own state alone. Then a ray whose t repeats with period 2 retires with its final t by itself
  // (the wave-level cycle exit generalised), and at a continuation cap the still-marching RAYS,
  // not their groups, go on: the group saves every ray's state (cont_state gets an eighth per-ray
  // row, the ray's choice history), appends itself to cont_list_w (class 0) and its marching rays
  // to ray_list_w. A ray_cont launch marches 32 listed rays per block (ray_list[0..*ray_count),
  // any groups) from cont_resume to its cap or to the end and writes their states back; the
  // groups' post-march forward and backward then run in a resume launch (cont_resume = steps).
  // The grouping of rays changes no bit.
  int ray_mode;
  int ray_cont;
  const int* ray_list;
  const int* ray_count;
  int* ray_list_w;
  int* ray_count_w;
#ifdef RM_BLOCK_TRACE
  unsigned long long* btrace;  // measurement build: per-wave timing records (rm_ray_kernel)
#endif
};
#ifdef RM_BLOCK_TRACE
constexpr int kTraceWords = 12;
// measurement build: word w of this wave's record (lane 0 writes)
__device__ __forceinline__ void trace_word(const KArgs& a, int w, unsigned long long v) {
  if (a.btrace != nullptr && (threadIdx.x & 63) == 0)
    a.btrace[kTraceWords * ((unsigned long long)blockIdx.x * kWaves + (threadIdx.x >> 6)) + w] = v;
}
#define RM_TRACE(w, v) trace_word(a, (w), (v))
#else
#define RM_TRACE(w, v) ((void)0)
#endif

// ---- sphere records: pair-interleaved, in global memory, read through scalar loads ----------
// rm_prep_kernel writes them once per call. Pair i holds spheres (2i, 2i+1) so every sweep runs
// two spheres per v_pk_* instruction:
//   P0 = {-2cx0, -2cx1, -2cy0, -2cy1}   P1 = {-2cz0, -2cz1, |c0|^2, |c1|^2}
//   P2 = {k r0, k r1, r0, r1}           P3 = {red0, red1, green0, green1}   P4 = {blue0, blue1}
//   S0, S1 = P0, P1 scaled by k^2       W  = {2^(k r0), 2^(k r1), 2^(k (r0 - r_first)), 2^(k (r1 - r_first))}
// (k = smooth_k log2 e). Every lane of a wave reads the same record at the same time, so the
// kernel reads them through the constant address space: s_load into SGPRs that feed the
// packed VALU ops as scalar operands -- no LDS staging, no LDS broadcast traffic, and no limit
// on M (the records stream through the scalar cache / L2).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(4))) f4v* cf4_ptr;
typedef const __attribute__((address_space(4))) f2v* cf2_ptr;
typedef const __attribute__((address_space(4))) float* cf1_ptr;

// Header after the records: {r_min, r_max, max |c_j - c_0|, 0, c_x, c_y, c_z, R} of the real
// spheres ((c, R): bounding sphere, scene_bound), followed by one partial header per
// rm_prep_kernel block when that kernel ran on more than one block.
constexpr int kRecHeader = 8;

// Then, 16-byte aligned, the matrix-core tiles of the march (lse_mfma): per row block of 16
// spheres 64 lanes x 16 B of A fragments, then per row block 32 floats {w(16), w_fixed(16)}.
__host__ __device__ inline size_t tiles_offset(int npairs, int nprep) {
  return ((size_t)npairs * (7 * 16 + 8) + (size_t)(nprep + 1) * kRecHeader * sizeof(float) + 15) & ~(size_t)15;
}
// Then the escape thresholds of the march: kEscTab floats (see write_bound).
constexpr int kEscTab = 64;
#ifdef RM_RAY_STATS
constexpr int kStatsWords = 8;  // + [6] / [7]: lane-steps after the cap, run and compacted (measurement)
#ifndef RM_RAY_STATS_CAP
#define RM_RAY_STATS_CAP 16
#endif
#else
constexpr int kStatsWords = 6;  // rm_stats device counters (KArgs::stats)
#endif
[[maybe_unused]] constexpr int kDeadCountSlot = 44;  // Lds::misc int: the hand-off's count of waves that ended early
__host__ __device__ inline size_t esc_offset(int npairs, int nprep) {
  const size_t nrb = (size_t)npairs / 8;
  return tiles_offset(npairs, nprep) + nrb * 64 * 16 + nrb * 32 * sizeof(float);
}
// Then the per-view origin steps of camera mode (write_origins): RM_MAX_VIEWS_PER_CALL floats,
// then per view a lower bound on the eye's distance to the nearest sphere centre (the march's
// clamp-free proof, rho_lb in rm_ray_kernel): RM_MAX_VIEWS_PER_CALL floats.
__host__ __device__ inline size_t origin_offset(int npairs, int nprep) {
  return esc_offset(npairs, nprep) + kEscTab * sizeof(float);
}
__host__ __device__ inline size_t rec_bytes(int npairs, int nprep) {
  return origin_offset(npairs, nprep) + 2 * RM_MAX_VIEWS_PER_CALL * sizeof(float);
}

struct Lds {  // the sphere records (global, scalar-loaded) plus the kernel's LDS scratch
  cf4_ptr P0, P1, P2, P3, S0, S1, W;
  cf2_ptr P4;
  const uint4* At;  // lse_mfma sphere fragments (global)
  const float* Wt;  // lse_mfma weights (global)
  float* slots;  // backward wave partials, 2 buffers (LDS); lse_mfma's ray exchange in the march
  float* misc;   // small LDS scratch
  __device__ __forceinline__ static float4 v4(f4v v) { return make_float4(v.x, v.y, v.z, v.w); }
  __device__ __forceinline__ float4 p0(int i) const { return v4(P0[i]); }
  __device__ __forceinline__ float4 p1(int i) const { return v4(P1[i]); }
  __device__ __forceinline__ float4 p2(int i) const { return v4(P2[i]); }
  __device__ __forceinline__ float4 p3(int i) const { return v4(P3[i]); }
  __device__ __forceinline__ float2 p4(int i) const {
    const f2v v = P4[i];
    return make_float2(v.x, v.y);
  }
  __device__ __forceinline__ float2 kr(int i) const {
    const f4v v = P2[i];
    return make_float2(v.x, v.y);
  }
  // the same records from pair `off` on (a split block's quarter of the vector sweeps)
  __device__ __forceinline__ Lds from_pair(int off) const {
    Lds q = *this;
    q.P0 += off;
    q.P1 += off;
    q.P2 += off;
    q.P3 += off;
    q.S0 += off;
    q.S1 += off;
    q.W += off;
    q.P4 += off;
    return q;
  }
};

// LDS: the backward's two partial buffers, or (during the march) lse_mfma's per-wave ray
// exchange (64 x (16 + 16 + 4) B per wave); then 256 B of misc scratch.
// The transposed backward (RM_BWD_TRANSPOSED) uses 15 x 64 ray-data floats (field-major) per wave
// and kWaves x 64 g_t shares per wave (19.3 KB). The LDS of a block decides how many blocks a CU
// holds once waves leave the march early (their registers free up, the block's LDS stays until its
// last wave ends): 19.3 KB -> 8 blocks per CU (24.3 KB -> 6, 32.3 KB -> 4).
constexpr int kBwdFields = 15;  // ray-image fields of the transposed backward
constexpr size_t kSlotBwdT = ((size_t)kWaves * 64 * kBwdFields + (size_t)kWaves * kWaves * 64) * sizeof(float);
constexpr size_t kSlotBytes0 = (size_t)2 * kWaves * kChunkBwd * 8 * sizeof(float) > (size_t)kWaves * 64 * 36
                                   ? (size_t)2 * kWaves * kChunkBwd * 8 * sizeof(float)
                                   : (size_t)kWaves * 64 * 36;
constexpr size_t kSlotBytes = RM_BWD_TRANSPOSED && kSlotBwdT > kSlotBytes0 ? kSlotBwdT : kSlotBytes0;
__host__ __device__ constexpr size_t lds_bytes() { return kSlotBytes + 256; }
// the split march's two combine buffers (kWaves x 64 floats each) after the march exchange
constexpr int kSplitCombOff = kWaves * 64 * 9;  // floats: xa, xb (64 uint4 per wave each), xs
static_assert((kSplitCombOff + 2 * kWaves * 64) * sizeof(float) <= kSlotBytes, "split combine buffers fit the slots");

// three-value block reduction (min, max, max) for the record header (blockDim.x / 64 <= 16 waves)
__device__ __forceinline__ void header_reduce(float& rmin, float& rmax, float& spread, float* dst) {
  __shared__ float red[3][16];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    rmin = fminf(rmin, __shfl_xor(rmin, off));
    rmax = fmaxf(rmax, __shfl_xor(rmax, off));
    spread = fmaxf(spread, __shfl_xor(spread, off));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = rmin;
    red[1][wave] = rmax;
    red[2][wave] = spread;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w2 = 1; w2 < (int)(blockDim.x >> 6); ++w2) {
      red[0][0] = fminf(red[0][0], red[0][w2]);
      red[1][0] = fmaxf(red[1][0], red[1][w2]);
      red[2][0] = fmaxf(red[2][0], red[2][w2]);
    }
    dst[0] = red[0][0];
    dst[1] = red[1][0];
    dst[2] = red[2][0];
    dst[3] = 0.0f;
  }
}

// Bounding sphere of the scene, block-wide: c0 = centre of the centres' bounding box,
// R >= |c_j - c0| + r_j for every sphere (rounded up). scratch: >= 8 floats of LDS per wave of
// the block.
__device__ __forceinline__ void scene_bound(const KArgs& a, float* scratch, int tid, float c0[3], float& R) {
  const int lane = tid & 63, wave = tid >> 6, nt = (int)blockDim.x, nw = nt >> 6;
  float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int j = tid; j < a.M; j += nt)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float c = a.centers[3 * j + k];
      v[k] = fminf(v[k], c);
      v[3 + k] = fmaxf(v[3 + k], c);
    }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[k] = fminf(v[k], __shfl_xor(v[k], off));
      v[3 + k] = fmaxf(v[3 + k], __shfl_xor(v[3 + k], off));
    }
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < 6; ++k) scratch[8 * wave + k] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float lo = scratch[k], hi = scratch[3 + k];
    for (int w = 1; w < nw; ++w) {
      lo = fminf(lo, scratch[8 * w + k]);
      hi = fmaxf(hi, scratch[8 * w + 3 + k]);
    }
    c0[k] = 0.5f * (lo + hi);
  }
  float r = 0.0f;
  for (int j = tid; j < a.M; j += nt) {
    const float dx = a.centers[3 * j] - c0[0], dy = a.centers[3 * j + 1] - c0[1], dz = a.centers[3 * j + 2] - c0[2];
    r = fmaxf(r, fsqrt(dx * dx + dy * dy + dz * dz) + a.radius[j]);  // 1 ulp: inside the round-up below
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) r = fmaxf(r, __shfl_xor(r, off));
  __syncthreads();  // everyone has read the box
  if (lane == 0) scratch[8 * wave] = r;
  __syncthreads();
  R = scratch[0];
  for (int w = 1; w < nw; ++w) R = fmaxf(R, scratch[8 * w]);
  R = R * (1.0f + 1e-5f) + 1e-6f;  // cover the f32 rounding of |c - c0| + r
  __syncthreads();  // scratch is reused by the caller
}

// ---- matrix-core march fragments (see lse_mfma) ----------------------------------------------
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// exact three-part bf16 split of x (bit patterns in the low 16 bits)
__device__ __forceinline__ void split3(float x, unsigned& h1, unsigned& h2, unsigned& h3) {
  const unsigned a = __float_as_uint(x) & 0xFFFF0000u;
  const float r1 = x - __uint_as_float(a);
  const unsigned b = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(b);
  const unsigned c = __float_as_uint(r2) & 0xFFFF0000u;
  h1 = a >> 16;
  h2 = b >> 16;
  h3 = c >> 16;
}
__device__ __forceinline__ unsigned pack2(unsigned lo16, unsigned hi16) { return lo16 | (hi16 << 16); }
constexpr unsigned kBf16One = 0x3F80u;

// sphere-side fragment: K slice g (8 bf16) of sphere j (rm_prep_kernel)
__device__ __forceinline__ uint4 mfma_a_slice(const KArgs& a, int j, int g) {
  const float kappa = a.k * kLog2e, k2 = kappa * kappa;
  float cx, cy, cz;
  if (j < a.M) {
    cx = a.centers[3 * j];
    cy = a.centers[3 * j + 1];
    cz = a.centers[3 * j + 2];
  } else {  // padding sphere (see rm_prep_kernel)
    cx = kPadCenter;
    cy = cz = 0.0f;
  }
  unsigned x[3], y[3], z[3], C[3];
  split3(-2.0f * k2 * cx, x[0], x[1], x[2]);
  split3(-2.0f * k2 * cy, y[0], y[1], y[2]);
  split3(-2.0f * k2 * cz, z[0], z[1], z[2]);
  split3(k2 * (cx * cx + cy * cy + cz * cz), C[0], C[1], C[2]);
  if (g < 2)
    return make_uint4(pack2(x[g], x[g]), pack2(x[g], y[g]), pack2(y[g], y[g]), pack2(z[g], z[g]));
  if (g == 2) return make_uint4(pack2(x[2], x[2]), pack2(0u, y[2]), pack2(y[2], 0u), pack2(z[2], z[2]));
  return make_uint4(pack2(z[0], z[1]), pack2(kBf16One, kBf16One), pack2(kBf16One, C[0]), pack2(C[1], C[2]));
}
// Element e of the tile array: v_mfma_f32_16x16x32_bf16 -- row block rb = e / 64 of 16 spheres,
// lane l = e % 64 holds sphere 16 rb + (l & 15), slice l >> 4; RM_MFMA32 (v_mfma_f32_32x32x16_bf16,
// two per 32 spheres: K halves m = 0, 1) -- block e / 128 of 32 spheres, m = (e / 64) & 1, lane l
// holds sphere 32 rb + (l & 31), slice 2 m + (l >> 5). The same bytes per sphere either way.
__device__ __forceinline__ uint4 mfma_a_frag(const KArgs& a, int e) {
  const int l = e & 63;
#if RM_MFMA32
  return mfma_a_slice(a, 32 * (e >> 7) + (l & 31), 2 * ((e >> 6) & 1) + (l >> 5));
#else
  return mfma_a_slice(a, 16 * (e >> 6) + (l & 15), l >> 4);
#endif
}
// Sphere of weight slot e (per 16 spheres 32 slots: 16 unshifted | 16 fixed-shift weights in sphere
// order; RM_MFMA32: per 32 spheres 64 slots, 32 | 32, slot h * 16 + 4 i + v of a half is sphere
// 8 i + 4 h + v of the block -- the 32x32 result rows of lane half h)
__device__ __forceinline__ int mfma_w_sphere(int e) {
#if RM_MFMA32
  const int x = e & 31;
  return 32 * (e >> 6) + 8 * ((x >> 2) & 3) + 4 * (x >> 4) + (x & 3);
#else
  return 16 * (e >> 5) + (e & 15);
#endif
}
__device__ __forceinline__ bool mfma_w_fixed(int e) { return (e & (RM_MFMA32 ? 32 : 16)) != 0; }

// hdr[4..7] = the bounding sphere (c, R) of scene_bound, for the march's escape test, and its
// distance thresholds T(n), n < kEscTab: a receding ray at distance d from c with n march steps
// left ends them at distance >= gone_d + R' from c if (1 - 1e-5) d >= T(n). Every step is at
// least g = d - R' long (R' = R + ln(M)/k + 1e-3: the soft-min is >= the hard min - ln(M)/k,
// 1e-3 covers the fp32 march) and keeps the ray receding, so one step takes d to at least
// F(d) = (1 - 1e-5) sqrt(d^2 + (d - R')^2); T(0) = gone_d + R' and T(n) = F^-1(T(n - 1)) =
// (R' + sqrt(2 y^2 - R'^2)) / 2 with y = T(n - 1) / (1 - 1e-5), rounded up. For n >= kEscTab the
// march uses T(kEscTab - 1) >= T(n).
__device__ void write_bound(const KArgs& a, float* hdr, float* esc) {
  __shared__ float scratch[8 * 16];
  float c[3], R;
  scene_bound(a, scratch, threadIdx.x, c, R);
  if (threadIdx.x == 0) {
    hdr[4] = c[0];
    hdr[5] = c[1];
    hdr[6] = c[2];
    hdr[7] = R;
  }
  if (threadIdx.x < kEscTab) {
    // f32 with a 1e-5 relative + 1e-6 absolute round-up per iteration (the f32 rounding of one
    // iteration is a few 1e-7): every T(n) stays above the exact inverse iterate. (R' rounded up
    // is conservative too: F^-1 grows with R' for y > R', which holds along the table.)
    float tv = INFINITY;
    if (a.gone_d > 0.0f) {
      const float rp = (R + a.lse_slack + 1e-3f) * (1.0f + 1e-6f);
      const float inv_shrink = 1.0000101f;  // y = T / (1 - 1e-5) <= T inv_shrink
      float T = (a.gone_d + rp) * (1.0f + 1e-6f);
      // four dependent instructions per step (v_sqrt_f32: 1 ulp, inside the round-up)
      const float two_c2 = 2.0f * inv_shrink * inv_shrink * (1.0f + 1e-6f), nrp2 = -rp * rp,
                  half_up = 0.5f * (1.0f + 1e-5f);
      // the march reads T(n) for n <= a.steps only: entries past it repeat T(a.steps) (>= T(n)),
      // which shortens the longest dependent chain at S < kEscTab
      const int nmax = min((int)threadIdx.x, a.steps);
      for (int n = 1; n <= nmax; ++n) T = fmaf(rp + fsqrt(fmaf(two_c2 * T, T, nrp2)), half_up, 1e-6f);
      tv = T * (1.0f + 1e-6f);
    }
    esc[threadIdx.x] = tv;
  }
}

// Records of the call (see Lds), one thread per sphere pair. Each block reduces its pairs'
// {r_min, r_max, spread} into the header (one block) or its partial (several blocks, then
// rm_prep_finish); the final header also gets the scene's bounding sphere (scene_bound).
constexpr int kPrepStageMax = 512;  // one-block prep: parameters staged in LDS up to this M

template <bool PAR>
__device__ void write_origins(const KArgs& a, const float4& S00, const float4& S10, float rmax, float spread,
                              const uint4* At, const float* Wt, float* orig, unsigned char* xch, int v);

__global__ __launch_bounds__(256) void rm_prep_kernel(const KArgs a0, float4* __restrict__ rec) {
  // One-block case: stage the parameters in LDS once (one load round instead of one per phase:
  // records, MFMA tiles, header, bounding sphere); the phases below read them through `a`.
  __shared__ float stage[7 * kPrepStageMax];
  const int nt = (int)blockDim.x;
  KArgs a = a0;
  if (gridDim.x == 1 && a0.M <= kPrepStageMax) {
    const int M = a0.M;
    for (int e = threadIdx.x; e < 3 * M; e += nt) {
      stage[e] = a0.centers[e];
      stage[3 * M + e] = a0.colors_h != nullptr ? (float)a0.colors_h[e] : a0.colors[e];
    }
    for (int e = threadIdx.x; e < M; e += nt) stage[6 * M + e] = a0.radius[e];
    __syncthreads();
    a.centers = stage;
    a.colors = stage + 3 * M;
    a.colors_h = nullptr;
    a.radius = stage + 6 * M;
  }
  const int np = a.Mpad / 2;
  float4* P0 = rec;
  float4* P1 = P0 + np;
  float4* P2 = P1 + np;
  float4* P3 = P2 + np;
  float4* S0 = P3 + np;
  float4* S1 = S0 + np;
  float4* W = S1 + np;
  float2* P4 = reinterpret_cast<float2*>(W + np);
  float* hdr = reinterpret_cast<float*>(P4 + np);
  const float kappa = a.k * kLog2e, k2 = kappa * kappa;
  const float kr_first = kappa * a.radius[0];
  const float c0x = a.centers[0], c0y = a.centers[1], c0z = a.centers[2];
  float rmin = INFINITY, rmax = 0.0f, spread = 0.0f;
  const int ip = blockIdx.x * nt + threadIdx.x;
  if (ip < np) {
    float gx[2], gy[2], gz[2], cc[2], kr[2], rr[2], cr[2], cg[2], cb[2], w[2], wf[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * ip + h;
      if (j < a.M) {
        const float cx = a.centers[3 * j], cy = a.centers[3 * j + 1], cz = a.centers[3 * j + 2];
        const float r = a.radius[j];
        gx[h] = -2.0f * cx;
        gy[h] = -2.0f * cy;
        gz[h] = -2.0f * cz;
        cc[h] = cx * cx + cy * cy + cz * cz;
        kr[h] = kappa * r;
        rr[h] = r;
        if (a.colors_h != nullptr) {  // fp16 colours: widened exactly, blended in fp32
          cr[h] = (float)a.colors_h[3 * j];
          cg[h] = (float)a.colors_h[3 * j + 1];
          cb[h] = (float)a.colors_h[3 * j + 2];
        } else {
          cr[h] = a.colors[3 * j];
          cg[h] = a.colors[3 * j + 1];
          cb[h] = a.colors[3 * j + 2];
        }
        w[h] = fexp2(kr[h]);
        wf[h] = fexp2(kr[h] - kr_first);
        rmin = fminf(rmin, r);
        rmax = fmaxf(rmax, r);
        const float ex = cx - c0x, ey = cy - c0y, ez = cz - c0z;
        spread = fmaxf(spread, sqrtf(ex * ex + ey * ey + ez * ez));
      } else {
        // padding sphere at c = (kPadCenter, 0, 0): the expansion form (|c|^2) and the direct
        // form of the normal taps (p - c) both see distance ~1e15, so every exp() of its terms
        // underflows to exactly 0 (its weights are 0) and all of its gradient terms are 0.
        gx[h] = -2.0f * kPadCenter;
        gy[h] = gz[h] = 0.0f;
        cc[h] = kPadCenter * kPadCenter;
        kr[h] = rr[h] = cr[h] = cg[h] = cb[h] = w[h] = wf[h] = 0.0f;
      }
    }
    P0[ip] = make_float4(gx[0], gx[1], gy[0], gy[1]);
    P1[ip] = make_float4(gz[0], gz[1], cc[0], cc[1]);
    P2[ip] = make_float4(kr[0], kr[1], rr[0], rr[1]);
    P3[ip] = make_float4(cr[0], cr[1], cg[0], cg[1]);
    P4[ip] = make_float2(cb[0], cb[1]);
    S0[ip] = make_float4(k2 * gx[0], k2 * gx[1], k2 * gy[0], k2 * gy[1]);
    S1[ip] = make_float4(k2 * gz[0], k2 * gz[1], k2 * cc[0], k2 * cc[1]);
    W[ip] = make_float4(w[0], w[1], wf[0], wf[1]);
  }
  // matrix-core tiles of the march (lse_mfma)
  const int nrb = np / 8;
  char* tiles = reinterpret_cast<char*>(rec) + tiles_offset(np, gridDim.x);
  uint4* At = reinterpret_cast<uint4*>(tiles);
  float* Wt = reinterpret_cast<float*>(At + (size_t)nrb * 64);
#ifndef RM_DBG_NO_TILES
  for (int e = blockIdx.x * nt + threadIdx.x; e < nrb * 64; e += gridDim.x * nt) At[e] = mfma_a_frag(a, e);
#endif
  for (int e = blockIdx.x * nt + threadIdx.x; e < nrb * 32; e += gridDim.x * nt) {
    const int j = mfma_w_sphere(e);
    const float krj = j < a.M ? kappa * a.radius[j] : 0.0f;
    Wt[e] = j >= a.M ? 0.0f : (mfma_w_fixed(e) ? fexp2(krj - kr_first) : fexp2(krj));
  }
  header_reduce(rmin, rmax, spread, gridDim.x == 1 ? hdr : hdr + (size_t)(1 + blockIdx.x) * kRecHeader);
#ifndef RM_DBG_NO_BOUND
  if (gridDim.x == 1) write_bound(a, hdr, reinterpret_cast<float*>(reinterpret_cast<char*>(rec) + esc_offset(np, 1)));
#endif
}

__global__ __launch_bounds__(256) void rm_prep_finish(const KArgs a, float* __restrict__ hdr, float* __restrict__ esc,
                                                      int nprep) {
  float rmin = INFINITY, rmax = 0.0f, spread = 0.0f;
  for (int b = threadIdx.x; b < nprep; b += 256) {
    const float* h = hdr + (size_t)(1 + b) * kRecHeader;
    rmin = fminf(rmin, h[0]);
    rmax = fmaxf(rmax, h[1]);
    spread = fmaxf(spread, h[2]);
  }
  header_reduce(rmin, rmax, spread, hdr);
  write_bound(a, hdr, esc);
}

// The per-view origin steps (write_origins), one 64-thread block (one wave) per view, after the
// records are complete: the views run on separate CUs side by side.
// A split launch's origin step runs its four quarters on four waves of the block (the split
// march's own combine: the same bits).
constexpr int kOriginXch = 64 * 36;  // bytes of march exchange per wave
template <bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 64 * kSplitWaves : 64) void rm_origin_kernel(const KArgs a,
                                                                                 const float4* __restrict__ rec,
                                                                                 int nprep) {
  __shared__ __attribute__((aligned(16))) unsigned char xch[SPLIT ? kSplitWaves * kOriginXch + kSplitWaves * 64 * 4
                                                                  : kOriginXch];
  const int np = a.Mpad / 2;
  const uint4* At = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(rec) + tiles_offset(np, nprep));
  const float* Wt = reinterpret_cast<const float*>(At + (size_t)(np / 8) * 64);
  const float* hdr = reinterpret_cast<const float*>(reinterpret_cast<const float2*>(rec + 7 * (size_t)np) + np);
  write_origins<SPLIT>(a, rec[4 * np], rec[5 * np], hdr[1], hdr[2], At, Wt, a.origin, xch, blockIdx.x);
}

// ---- packed helpers --------------------------------------------------------------------------
__device__ __forceinline__ f2 sp(float x) { return f2{x, x}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 sqrt2(f2 q) { return f2{fsqrt(q.x), fsqrt(q.y)}; }
__device__ __forceinline__ f2 exp2v(f2 x) { return f2{fexp2(x.x), fexp2(x.y)}; }
__device__ __forceinline__ f2 rcp2(f2 x) { return f2{frcp(x.x), frcp(x.y)}; }
__device__ __forceinline__ f2 rsq2(f2 x) { return f2{frsq(x.x), frsq(x.y)}; }
// max(q, qmin) for qmin > 0 as one integer max on the bit patterns (non-negative floats order
// like their bits, negative ones have negative bit patterns): fmaxf in the kernels' IEEE mode
// costs a canonicalising v_max before the v_max. Equal to fmaxf for every non-NaN q.
__device__ __forceinline__ float qclamp(float q, float qmin) {
  return __int_as_float(max(__float_as_int(q), __float_as_int(qmin)));
}
__device__ __forceinline__ f2 clamp_q(f2 q) { return f2{qclamp(q.x, 1e-6f), qclamp(q.y, 1e-6f)}; }
__device__ __forceinline__ f2 lo(const float4& v) { return f2{v.x, v.y}; }
__device__ __forceinline__ f2 hi(const float4& v) { return f2{v.z, v.w}; }

// q = |p|^2 + |c|^2 - 2 p.c for a sphere pair (expansion form, scene.rs:66-71). Every sweep that
// must reproduce another sweep's distances bit for bit uses this one expression.
__device__ __forceinline__ f2 qpair(const f2& PX, const f2& PY, const f2& PZ, const f2& PP, const float4& A,
                                    const float4& B) {
  return fma2(PZ, lo(B), fma2(PY, hi(A), fma2(PX, lo(A), PP + hi(B))));
}
__device__ __forceinline__ float psq(const float p[3]) { return fmaf(p[2], p[2], fmaf(p[1], p[1], p[0] * p[0])); }

// The light direction ld / |ld| (renderer_diff.rs:49-50) and the Jacobian of that normalisation
// applied to summed per-ray terms r: component k of (r - ldn (ldn . r)) / |ld|. Contraction off in
// both: every kernel (general and small, forward and final blocks) forms them with the same fp32
// operations whatever code surrounds the call, so their bits cannot follow unrelated edits.
__device__ __forceinline__ float light_unit(const float* light_dir, float (&ln)[3]) {
#pragma clang fp contract(off)
  const float l0 = light_dir[0], l1 = light_dir[1], l2 = light_dir[2];
  const float len = sqrtf(l0 * l0 + l1 * l1 + l2 * l2);
  ln[0] = l0 / len;
  ln[1] = l1 / len;
  ln[2] = l2 / len;
  return len;
}
__device__ __forceinline__ float light_grad(const float (&r)[3], const float* light_dir, int k) {
#pragma clang fp contract(off)
  float ln[3];
  const float len = light_unit(light_dir, ln);
  const float proj = ln[0] * r[0] + ln[1] * r[1] + ln[2] * r[2];
  const float rk = k == 0 ? r[0] : (k == 1 ? r[1] : r[2]), lk = k == 0 ? ln[0] : (k == 1 ? ln[1] : ln[2]);
  return (rk - lk * proj) / len;
}

// A wave's 64 spheres' 8 record columns (lane = sphere, v[7] = 0) stored as two contiguous 1 KB
// runs: store h covers spheres 32 h .. 32 h + 31, lane l writing half (l & 1) of sphere
// 32 h + (l >> 1) (two half-line stores per lane would touch every line twice). Every lane of
// the wave calls it; nsph = the group's spheres below Mpad.
__device__ __forceinline__ void store_group_cols(float* rec_grp, const float (&v)[8], int lane, int nsph) {
  const int s = lane >> 1, hf = lane & 1;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float lo = __shfl(v[c], 32 * h + s), hi = __shfl(v[4 + c], 32 * h + s);
      o[c] = hf ? hi : lo;
    }
    const int sph = 32 * h + s;
    if (sph < nsph) reinterpret_cast<float4*>(rec_grp)[2 * sph + hf] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

// ---- forward sweeps -----------------------------------------------------------------
// Base-2 log-sum-exp of v_j = kappa*(r_j - rho_j) over a tile (sdf.rs:36-40), running max m and
// shifted sum s carried across tiles; chunks of 16 spheres, one rescale exp per chunk.
// CLAMP=false drops max(q, 1e-6): only used when the caller proved every rho_j >= kSafeRho.
// Shift of the exponents: kShiftMax = chunked running max (always safe); kShiftFixed = m set
// once from the first sphere (safe when kappa * (r_max + max |c_j - c_0|) <= 100 and the point
// is near enough that fp32 rounding of rho stays small, so every exponent lies within +-100 of
// it); kShiftNone = m = 0 (safe when the hard maximum is known to lie in [-100, 100]). All three
// give the same log-sum-exp up to fp32 rounding.
enum LseShift { kShiftMax = 0, kShiftFixed = 1, kShiftNone = 2 };

template <bool CLAMP, int SHIFT>
__device__ __forceinline__ void lse_point(const float p[3], const Lds& L, int npairs, float nkappa, float& m,
                                          float& s) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), NK = sp(nkappa);
  for (int i0 = 0; i0 < npairs; i0 += 8) {
    f2 v[8];
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
      const float4 A = L.p0(i0 + ii), B = L.p1(i0 + ii);
      const float2 K = L.kr(i0 + ii);
      f2 q = qpair(PX, PY, PZ, PP, A, B);
      if constexpr (CLAMP) q = clamp_q(q);
      v[ii] = fma2(q * rsq2(q), NK, f2{K.x, K.y});  // rho = q rsq(q), as backward sweep 2
    }
    if constexpr (SHIFT != kShiftMax) {
      if constexpr (SHIFT == kShiftFixed) {
        if (m == -INFINITY) m = v[0].x;
      }
      const f2 MN = sp(m);
      f2 acc = f2{s, 0.0f};
#pragma unroll
      for (int ii = 0; ii < 8; ++ii) acc += exp2v(SHIFT == kShiftNone ? v[ii] : v[ii] - MN);
      s = acc.x + acc.y;
      continue;
    }
    float cm = fmaxf(v[0].x, v[0].y);
#pragma unroll
    for (int ii = 1; ii < 8; ++ii) cm = fmaxf(cm, fmaxf(v[ii].x, v[ii].y));
    const float mn = fmaxf(m, cm);
    const f2 MN = sp(mn);
    f2 acc = f2{s * fexp2(m - mn), 0.0f};
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) acc += exp2v(v[ii] - MN);
    s = acc.x + acc.y;
    m = mn;
  }
}

// ---- the march's log-sum-exp on the matrix cores ---------------------------------------------
// q'_jn = k^2 |p_n - c_j|^2 for 16 spheres x 16 rays is one v_mfma_f32_16x16x32_bf16: every f32
// operand is split exactly into three bf16 parts (x = x1 + x2 + x3, truncation: each part keeps
// the next 8 significant bits), and the K = 32 products are the 30 split-part products that
// matter (a3 x3 is below 2^-30 of a x), all exact in fp32:
//   K slice 0: A = [a1x a1x a1x a1y a1y a1y a1z a1z]   B = Sa = [x1 x2 x3 y1 y2 y3 z1 z2]
//   K slice 1: A = [a2x a2x a2x a2y a2y a2y a2z a2z]   B = Sa
//   K slice 2: A = [a3x a3x 0   a3y a3y 0   a3z a3z]   B = Sa
//   K slice 3: A = [a1z a2z 1 1 1 C1 C2 C3]             B = Sb = [z3 z3 P1 P2 P3 1 1 1]
// with a = -2 k^2 c, C = k^2 |c|^2 (sphere side, rm_prep_kernel) and P = k^2 |p|^2 (ray side):
// sum = k^2 (|p|^2 - 2 p.c + |c|^2), the expansion form of scene.rs:66-71. The lanes then run
// only sqrt, exp2 and the weighted accumulate (lse_weighted's four packed ops per sphere pair
// go to the matrix pipe). Lane (n, g) = (l & 15, l >> 4) holds rays 16cb + n of the wave and
// spheres 16rb + 4g + v; the rays' Sa / Sb / shift go through a per-wave LDS exchange.
// Sum over the spheres of w_j 2^(-rho'_j) (FIXED = false; w = 2^(k r)) or w_j 2^(sh - rho'_j)
// (FIXED; w = 2^(k (r - r_0)), sh = the ray's own shift) for the lane's own ray -- the same sum
// as lse_weighted up to fp32 rounding. xa / xb / xs: this wave's LDS exchange (64 uint4, 64
// uint4, 64 floats).
// NCB < 4 (the split march's smaller ray groups, kSplitRays): the wave's lanes hold 16 NCB rays,
// lane l the ray of lane l mod 16 NCB; only the first NCB column blocks are multiplied and summed,
// and the reduction takes the missing blocks as copies of the present ones. A ray's sum is the
// same chain of the same terms as with NCB = 4 (the same bits; IEEE addition is commutative).
template <bool CLAMP, bool FIXED, bool BUF = (RM_MARCH_BUFLOAD != 0), int NCB = 4>
__device__ __forceinline__ float lse_mfma(const float p[3], float k2, float sh, const uint4* __restrict__ At,
                                          const float* __restrict__ Wt, int nrb, uint4* xa, uint4* xb, float* xs,
                                          int lane) {
  // no fp contraction: the record kernel's origin step (write_origins) runs this code in another
  // kernel and must reproduce it bit for bit
#pragma clang fp contract(off)
  static_assert(NCB == 1 || NCB == 2 || NCB == 4, "column blocks per wave");
  {  // the lane's own ray: Sa, Sb and the shift into the exchange
    unsigned x[3], y[3], z[3], P[3];
    split3(p[0], x[0], x[1], x[2]);
    split3(p[1], y[0], y[1], y[2]);
    split3(p[2], z[0], z[1], z[2]);
    split3(k2 * psq(p), P[0], P[1], P[2]);
    xa[lane] = make_uint4(pack2(x[0], x[1]), pack2(x[2], y[0]), pack2(y[1], y[2]), pack2(z[0], z[1]));
    xb[lane] = make_uint4(pack2(z[2], z[2]), pack2(P[0], P[1]), pack2(P[2], kBf16One), pack2(kBf16One, kBf16One));
    if constexpr (FIXED) xs[lane] = sh;
  }
  __builtin_amdgcn_wave_barrier();
  const int n = lane & 15, g = lane >> 4;
  const uint4* src = g < 3 ? xa : xb;
  bf16x8 B[NCB];
  float S[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) {
    B[cb] = __builtin_bit_cast(bf16x8, src[16 * cb + n]);
    S[cb] = FIXED ? xs[16 * cb + n] : 0.0f;
  }
  const float QMIN = k2 * 1e-6f;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
  if (nrb == 0) {  // an empty quarter of a split block
    __builtin_amdgcn_wave_barrier();
    return 0.0f;
  }
  // BUF: buffer loads -- the row block's byte offset in a scalar register, the lane's offset
  // fixed in a vector register, no per-load 64-bit address arithmetic on the vector units (the
  // unsplit march +3 %, the split march +2 % once its quarter bounds are scalar); else global loads
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)At, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Wt + (FIXED ? 16 : 0)), (short)0, 0x7fffffff, 0x00020000);
  const int va = lane * 16, vw = g * 16;
  const float* wsrc = Wt + (FIXED ? 16 : 0) + 4 * g;
  auto load_a = [&](int rb) {
    if constexpr (BUF) return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, va, rb * 1024, 0));
    else return __builtin_bit_cast(bf16x8, At[rb * 64 + lane]);
  };
  auto load_w = [&](int rb) {
    if constexpr (BUF) return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw, vw, rb * 128, 0));
    else return *reinterpret_cast<const float4*>(wsrc + rb * 32);
  };
  auto tile = [&](const bf16x8& A, f32x4 (&D)[NCB]) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) D[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[cb], zero, 0, 0, 0);
  };
#if RM_MARCH_PK  // packed accumulate: two chains per ray (v even / odd), one v_pk_fma_f32 per two terms
  f2 acc2[NCB];
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc2[cb] = sp(0.0f);
#endif
  auto consume = [&](const f32x4 (&D)[NCB], const float4& w) {
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      float q[4] = {D[cb].x, D[cb].y, D[cb].z, D[cb].w};
      const float wv[4] = {w.x, w.y, w.z, w.w};
#if RM_MARCH_PK
      float rho[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if constexpr (CLAMP) q[v] = qclamp(q[v], QMIN);
        rho[v] = fsqrt(q[v]);
      }
#pragma unroll
      for (int v = 0; v < 4; v += 2) {
        // FIXED: the shifted exponents two at a time (v_pk_add_f32: the same bits as two v_sub_f32)
        const f2 x = FIXED ? sp(S[cb]) - f2{rho[v], rho[v + 1]} : f2{-rho[v], -rho[v + 1]};
        acc2[cb] = fma2(f2{wv[v], wv[v + 1]}, f2{fexp2(x.x), fexp2(x.y)}, acc2[cb]);
      }
#else
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if constexpr (CLAMP) q[v] = qclamp(q[v], QMIN);
        const float rho = fsqrt(q[v]);
        acc[cb] = fmaf(wv[v], fexp2(FIXED ? S[cb] - rho : -rho), acc[cb]);
      }
#endif
    }
  };
  // one tile at a time (registers: the march must not spill at 128 VGPRs); the fragments of the
  // next row block load while the lanes work on this one (nrb is even: Mpad % 32 == 0)
  f32x4 D[NCB];
  bf16x8 A = load_a(0);
  float4 w = load_w(0);
  for (int rb = 0; rb < nrb; rb += 2) {
    tile(A, D);
    const bf16x8 A1 = load_a(rb + 1);
    const float4 w1 = load_w(rb + 1);
    RM_SCHED_BARRIER();  // keep the loads a tile ahead of their use
    consume(D, w);
    RM_SCHED_BARRIER();
    tile(A1, D);
    const int rn = min(rb + 2, nrb - 1);
    A = load_a(rn);
    w = load_w(rn);
    RM_SCHED_BARRIER();
    consume(D, w1);
    RM_SCHED_BARRIER();
  }
  // partial sums of ray 16cb + n sit in the four lane groups: one transposing reduction (two
  // v_permlane32_swap and one v_permlane16_swap, no LDS) leaves lane (n, g) with the total of
  // its own ray 16g + n: rows 0/2 keep the column blocks 0/2 summed over lane bit 5, rows 1/3
  // the blocks 1/3, then each row adds its bit-4 partner
#if RM_MARCH_PK
#pragma unroll
  for (int cb = 0; cb < NCB; ++cb) acc[cb] = acc2[cb].x + acc2[cb].y;
#endif
  // NCB < 4: column block cb + NCB is a copy of block cb (the lanes' rays repeat every 16 NCB)
#pragma unroll
  for (int cb = NCB; cb < 4; ++cb) acc[cb] = acc[cb - NCB];
  const float own = swap16_sum(swap32_sum(acc[0], acc[2]), swap32_sum(acc[1], acc[3]));
  __builtin_amdgcn_wave_barrier();  // the exchange is rewritten by the next step
  return own;
}

#if RM_MFMA32
typedef float f32x16 __attribute__((ext_vector_type(16)));
// lse_mfma with v_mfma_f32_32x32x16_bf16: per 32 spheres and 32 rays two MFMAs (K halves: slices
// 0-1 with B = Sa, slices 2-3 with B = Sa / Sb by lane half), half the matrix-core instructions
// of 16x16x32 per evaluation (each holds the SIMD's vector issue for 8 cycles). Lane (r, h) =
// (l & 31, l >> 5) gets, per column block cb, 16 results of ray 32 cb + r: rows (i & 3) + 8 (i >> 2)
// + 4 h (mfma_w_sphere's slot order); the two halves of a ray meet in one v_permlane32_swap.
// Registers: one column block's tile at a time, the weights loaded as they are used, the ray side
// re-read from the exchange (measured: Appendix A; 2 spilled VGPRs in the train kernel).
template <bool CLAMP, bool FIXED, bool BUF = (RM_MARCH_BUFLOAD != 0)>
__device__ __forceinline__ float lse_mfma32(const float p[3], float k2, float sh, const uint4* __restrict__ At,
                                            const float* __restrict__ Wt, int nrb, uint4* xa, uint4* xb, float* xs,
                                            int lane) {
#pragma clang fp contract(off)
  {
    unsigned x[3], y[3], z[3], P[3];
    split3(p[0], x[0], x[1], x[2]);
    split3(p[1], y[0], y[1], y[2]);
    split3(p[2], z[0], z[1], z[2]);
    split3(k2 * psq(p), P[0], P[1], P[2]);
    xa[lane] = make_uint4(pack2(x[0], x[1]), pack2(x[2], y[0]), pack2(y[1], y[2]), pack2(z[0], z[1]));
    xb[lane] = make_uint4(pack2(z[2], z[2]), pack2(P[0], P[1]), pack2(P[2], kBf16One), pack2(kBf16One, kBf16One));
    if constexpr (FIXED) xs[lane] = sh;
  }
  __builtin_amdgcn_wave_barrier();
  const int r = lane & 31, h = lane >> 5;
  float S[2];
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) S[cb] = FIXED ? xs[32 * cb + r] : 0.0f;
  const float QMIN = k2 * 1e-6f;
  float acc[2] = {0.0f, 0.0f};
  if (nrb == 0) {
    __builtin_amdgcn_wave_barrier();
    return 0.0f;
  }
  const int n32 = nrb >> 1;  // nrb (16-sphere blocks) is even
  const f32x16 zero = {};
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)At, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Wt + (FIXED ? 32 : 0)), (short)0, 0x7fffffff, 0x00020000);
  const int va = lane * 16, vw = h * 64;
  auto load_a = [&](int rb, int m) {
    if constexpr (BUF) return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, va, (2 * rb + m) * 1024, 0));
    else return __builtin_bit_cast(bf16x8, At[(2 * rb + m) * 64 + lane]);
  };
  auto load_w = [&](int rb, int i) {
    if constexpr (BUF) return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rw, vw + 16 * i, rb * 256, 0));
    else return *reinterpret_cast<const float4*>(Wt + (FIXED ? 32 : 0) + rb * 64 + h * 16 + 4 * i);
  };
  auto consume = [&](const f32x16& D, int rb, int cb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float4 wi = load_w(rb, i);
      const float wv[4] = {wi.x, wi.y, wi.z, wi.w};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float q = D[4 * i + v];
        if constexpr (CLAMP) q = qclamp(q, QMIN);
        const float rho = fsqrt(q);
        acc[cb] = fmaf(wv[v], fexp2(FIXED ? S[cb] - rho : -rho), acc[cb]);
      }
    }
  };
  bf16x8 A0 = load_a(0, 0), A1 = load_a(0, 1);
  for (int rb = 0; rb < n32; ++rb) {
    int z = 0;  // opaque 0: the ray-side reads stay in the loop (hoisted they hold 16 VGPRs)
    asm volatile("" : "+s"(z));
    const uint4* xah = xa + z;
    const uint4* xbh = (h ? xb : xa) + z;
    f32x16 D = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, __builtin_bit_cast(bf16x8, xah[r]), zero, 0, 0, 0);
    D = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, __builtin_bit_cast(bf16x8, xbh[r]), D, 0, 0, 0);
    RM_SCHED_BARRIER();
    consume(D, rb, 0);
    RM_SCHED_BARRIER();
    D = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, __builtin_bit_cast(bf16x8, xah[32 + r]), zero, 0, 0, 0);
    D = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, __builtin_bit_cast(bf16x8, xbh[32 + r]), D, 0, 0, 0);
    const int rn = min(rb + 1, n32 - 1);
    A0 = load_a(rn, 0);
    A1 = load_a(rn, 1);
    RM_SCHED_BARRIER();
    consume(D, rb, 1);
    RM_SCHED_BARRIER();
  }
  // lanes < 32 end with column block 0 (rays 0-31), lanes >= 32 with block 1: ray l either way
  const float own = swap32_sum(acc[0], acc[1]);
  __builtin_amdgcn_wave_barrier();
  return own;
}
#endif

// Split march (RM_MARCH_SPLIT): the kSplitWaves waves of a block hold the same 64 rays; wave w
// sums the row blocks [part_rb(w), part_rb(w + 1)) (even bounds: lse_mfma runs pairs) and the
// partial sums are added in wave order, so every wave gets the same total. comb: 64 floats per
// wave of LDS.
__device__ __forceinline__ int part_rb(int nrb, int w) { return ((nrb * w) / kSplitWaves) & ~1; }
__device__ __forceinline__ float split_combine(float part, float* comb, int wave, int lane) {
  comb[wave * 64 + lane] = part;
  __syncthreads();
  float s = comb[lane];
#pragma unroll
  for (int w = 1; w < kSplitWaves; ++w) s += comb[w * 64 + lane];
  return s;
}
// A march step's soft-min D at p on the matrix cores without a shift (soft_min_march's
// unshifted step; shared with write_origins like march_d_fixed). comb != nullptr: a split
// block's wave, At / Wt / nrb its quarter (split_combine).
template <bool CLAMP, bool BUF = (RM_MARCH_BUFLOAD != 0), int NCB = 4>
__device__ __forceinline__ float march_d_none(const float p[3], float kappa, float inv_kappa,
                                              const uint4* __restrict__ At, const float* __restrict__ Wt, int nrb,
                                              uint4* xa, uint4* xb, float* xs, int lane, float* comb = nullptr,
                                              int wave = 0) {
#pragma clang fp contract(off)
#if RM_MFMA32
  float s = lse_mfma32<CLAMP, false, BUF>(p, kappa * kappa, 0.0f, At, Wt, nrb, xa, xb, xs, lane);
#else
  float s = lse_mfma<CLAMP, false, BUF, NCB>(p, kappa * kappa, 0.0f, At, Wt, nrb, xa, xb, xs, lane);
#endif
  if (comb != nullptr) s = split_combine(s, comb, wave, lane);
  return -flog2(fmaxf(s, 1e-30f)) * inv_kappa;
}

// rho'_0 = k |p - c_0| (k = smooth_k log2 e) of sphere 0 from its records S00 / S1[0] = S10: the
// fixed shift of the march, and (rho'_0 - k r_0 >= k d_min) the unshifted form's admission test.
__device__ __forceinline__ float fixed_shift(const float p[3], float k2, const float4& S00, const float4& S10) {
#pragma clang fp contract(off)
  const float q0 = fmaf(p[2], S10.x, fmaf(p[1], S00.z, fmaf(p[0], S00.x, fmaf(k2, psq(p), S10.z))));
  return fsqrt(qclamp(q0, k2 * 1e-6f));
}

// A march step's soft-min D at p on the matrix cores with the fixed shift sh = rho'_0 (sphere 0;
// S00 / S10 = its records S0[0] / S1[0]) -- soft_min_march's fixed-shift step, shared with the
// per-view origin step (write_origins) so that both give the same bits.
template <bool CLAMP, bool BUF = (RM_MARCH_BUFLOAD != 0), int NCB = 4>
__device__ __forceinline__ float march_d_fixed(const float p[3], float kappa, float inv_kappa, float kr_first,
                                               const float4& S00, const float4& S10, const uint4* __restrict__ At,
                                               const float* __restrict__ Wt, int nrb, uint4* xa, uint4* xb,
                                               float* xs, int lane, float* comb = nullptr, int wave = 0) {
#pragma clang fp contract(off)
  const float k2 = kappa * kappa;
  const float sh = fixed_shift(p, k2, S00, S10);
#if RM_MFMA32
  float s = lse_mfma32<CLAMP, true, BUF>(p, k2, sh, At, Wt, nrb, xa, xb, xs, lane);
#else
  float s = lse_mfma<CLAMP, true, BUF, NCB>(p, k2, sh, At, Wt, nrb, xa, xb, xs, lane);
#endif
  if (comb != nullptr) s = split_combine(s, comb, wave, lane);
  const float m = kr_first - sh;
  return -(flog2(fmaxf(s, 1e-30f)) + m) * inv_kappa;
}

// Camera mode: every ray of view v starts its march at the eye (camera.rs:83-85), so the first
// step's soft-min D(eye) is one number per view. Evaluated here once per view (one wave each) by
// the march's own code path for that step -- none = false (no previous step), the clamped
// sweep (no distance bound yet), fixed shift on the matrix cores -- it stands in for the step of
// every ray bit for bit (rm_ray_kernel). NaN where the first step would take another path
// (vector-only march, or the fixed shift not provably safe): those rays march it themselves.
// rec / hdr: this call's complete records and header; At / Wt: its march tiles; xch: 64 x 36 B
// of LDS. One wave computes view v.
template <bool PAR>
__device__ void write_origins(const KArgs& a, const float4& S00, const float4& S10, float rmax, float spread,
                              const uint4* At, const float* Wt, float* orig, unsigned char* xch, int v) {
  const int lane = threadIdx.x & 63;
  const int np = a.Mpad / 2;
  const float kappa = a.k * kLog2e, inv_kappa = 1.0f / kappa;
  const bool shift_fixed_ok = kappa * (rmax + spread) * 1.001f <= 100.0f;
  const bool shift_none_ok = kappa * rmax * 1.001f <= 30.0f;
  const float kr_first = kappa * a.radius[0];
  // PAR (a split launch, a block of kSplitWaves waves): wave w sums quarter w, combined in wave
  // order (split_combine) -- the split march's own sum; else one wave sums every row block
  const int wave = PAR ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  uint4* xa = reinterpret_cast<uint4*>(xch + wave * kOriginXch);
  uint4* xb = xa + 64;
  float* xs = reinterpret_cast<float*>(xa) + 64 * 8;
  float* comb = PAR ? reinterpret_cast<float*>(xch + kSplitWaves * kOriginXch) : nullptr;
  const int nrb = np / 8;
  const uint4* Aq = At;
  const float* Wq = Wt;
  int nq = nrb;
  if constexpr (PAR) {
    const int r0 = part_rb(nrb, wave);
    nq = part_rb(nrb, wave + 1) - r0;
    Aq += (size_t)r0 * 64;
    Wq += (size_t)r0 * 32;
  }
  {
    const CamBasis& cb = a.cams_dev != nullptr ? a.cams_dev[v] : a.cams[v];
    const float p[3] = {cb.eye[0], cb.eye[1], cb.eye[2]};
    float D = __builtin_nanf("");
    // the first step's choice in soft_min_march: unshifted when sphere 0 proves it safe, else
    // the fixed shift (else the vector path: not shared); block-uniform
    const bool none = a.mfma && shift_none_ok && fixed_shift(p, kappa * kappa, S00, S10) - kr_first <= 90.0f;
    // (a split launch's first step adds the four quarters' sums: the same here)
    if (none)
      D = march_d_none<true>(p, kappa, inv_kappa, Aq, Wq, nq, xa, xb, xs, lane, comb, wave);
    else if (a.mfma && shift_fixed_ok && psq(p) <= 1e10f)
      D = march_d_fixed<true>(p, kappa, inv_kappa, kr_first, S00, S10, Aq, Wq, nq, xa, xb, xs, lane, comb, wave);
    if (lane == 0 && wave == 0) orig[v] = D;
    // the eye's distance to the nearest sphere centre (direct form), rounded down by a relative
    // 1e-6 and 1e-6 (1 + |eye|) against the fp32 rounding of the eye and of the centres' offsets
    float m2 = INFINITY;
    for (int j = (int)threadIdx.x; j < a.M; j += (int)blockDim.x) {
      const float dx = p[0] - a.centers[3 * j], dy = p[1] - a.centers[3 * j + 1], dz = p[2] - a.centers[3 * j + 2];
      m2 = fminf(m2, fmaf(dz, dz, fmaf(dy, dy, dx * dx)));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m2 = fminf(m2, __shfl_xor(m2, off));
    if constexpr (PAR) {
      __shared__ float wmin[kSplitWaves];
      if (lane == 0) wmin[wave] = m2;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < kSplitWaves; ++w) m2 = fminf(m2, wmin[w]);
    }
    if (lane == 0 && wave == 0)
      orig[RM_MAX_VIEWS_PER_CALL + v] =
          sqrtf(m2) * (1.0f - 1e-6f) - 1e-6f * (1.0f + fabsf(p[0]) + fabsf(p[1]) + fabsf(p[2]));
  }
}

// The march's log-sum-exp in weighted form: rho' = sqrt(k^2 q) = k rho straight from the scaled
// geometry, term = 2^(k r_j) 2^(-rho'_j) (FIXED = false: shift 0) or 2^(k (r_j - r_0))
// 2^(rho'_0 - rho'_j) (FIXED: shift v_0 = k r_0 - rho'_0) -- one packed fma per sphere pair
// instead of the fma + subtract + add of lse_point. Returns the sum; *sh receives rho'_0.
template <bool CLAMP, bool FIXED>
__device__ __forceinline__ float lse_weighted(const float p[3], const Lds& L, int npairs, float k2, float& sh) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(k2 * psq(p)), QMIN = sp(k2 * 1e-6f);
  f2 acc[2] = {sp(0.0f), sp(0.0f)}, SH = sp(0.0f);  // two chains keep the fma latency hidden
  for (int i0 = 0; i0 < npairs; i0 += 8) {
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
      const float4 A = Lds::v4(L.S0[i0 + ii]), B = Lds::v4(L.S1[i0 + ii]), Wt = Lds::v4(L.W[i0 + ii]);
      f2 q = qpair(PX, PY, PZ, PP, A, B);
      if constexpr (CLAMP) q = f2{qclamp(q.x, QMIN.x), qclamp(q.y, QMIN.y)};
      const f2 rho = sqrt2(q);
      if constexpr (FIXED) {
        if (i0 == 0 && ii == 0) SH = sp(rho.x);
        acc[ii & 1] = fma2(hi(Wt), exp2v(SH - rho), acc[ii & 1]);
      } else {
        acc[ii & 1] = fma2(lo(Wt), exp2v(-rho), acc[ii & 1]);
      }
    }
  }
  sh = SH.x;
  const f2 t = acc[0] + acc[1];
  return t.x + t.y;
}

// The six normal taps p +- eps*e_a (scene.rs:93-111) in one pass over the spheres. q at a tap
// is formed from e = p - c in direct form, |e +- eps e_a|^2 = |e|^2 + eps^2 +- 2 eps e_a, which
// keeps the fp32 error of the finite difference ~10x below the reference's expansion form.
template <bool CLAMP>
__device__ __forceinline__ void lse_taps(const float p[3], const Lds& L, int npairs, float nkappa, float two_eps,
                                         float eps2, float (&m)[6], float (&s)[6]) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), NK = sp(nkappa), HALF = sp(0.5f), E2 = sp(eps2),
           TE = sp(two_eps), NTE = sp(-two_eps);
  for (int i0 = 0; i0 < npairs; i0 += 4) {
    f2 v[6][4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const float4 A = L.p0(i0 + ii), B = L.p1(i0 + ii);
      const float2 K = L.kr(i0 + ii);
      const f2 ex = fma2(HALF, lo(A), PX), ey = fma2(HALF, hi(A), PY), ez = fma2(HALF, lo(B), PZ);
      const f2 Q = fma2(ez, ez, fma2(ey, ey, fma2(ex, ex, E2)));
      f2 q[6] = {fma2(ex, TE, Q), fma2(ex, NTE, Q), fma2(ey, TE, Q), fma2(ey, NTE, Q), fma2(ez, TE, Q),
                 fma2(ez, NTE, Q)};
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        if constexpr (CLAMP) q[t] = clamp_q(q[t]);
        v[t][ii] = fma2(sqrt2(q[t]), NK, f2{K.x, K.y});
      }
    }
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      float cm = fmaxf(v[t][0].x, v[t][0].y);
#pragma unroll
      for (int ii = 1; ii < 4; ++ii) cm = fmaxf(cm, fmaxf(v[t][ii].x, v[t][ii].y));
      const float mn = fmaxf(m[t], cm);
      const f2 MN = sp(mn);
      f2 acc = f2{s[t] * fexp2(m[t] - mn), 0.0f};
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) acc += exp2v(v[t][ii] - MN);
      s[t] = acc.x + acc.y;
      m[t] = mn;
    }
  }
}

// The six taps in weighted form (no shift, see lse_weighted): e' = k (p - c) from the unscaled
// records, q'_tap = |e'|^2 + (k eps)^2 +- 2 (k eps) e'_a = k^2 q_tap, term = 2^(k r) 2^(-sqrt(q')),
// one packed fma per tap and pair instead of fma + subtract + add + running max.
template <bool CLAMP>
__device__ __forceinline__ void lse_taps_w(const float p[3], const Lds& L, int npairs, float kappa, float eps,
                                           float (&s)[6]) {
  const f2 KPX = sp(kappa * p[0]), KPY = sp(kappa * p[1]), KPZ = sp(kappa * p[2]), HK = sp(0.5f * kappa),
           E2 = sp(kappa * kappa * eps * eps), TE = sp(2.0f * kappa * eps), NTE = sp(-2.0f * kappa * eps),
           QMIN = sp(kappa * kappa * 1e-6f);
  f2 acc[6];
#pragma unroll
  for (int t = 0; t < 6; ++t) acc[t] = sp(0.0f);
  for (int i0 = 0; i0 < npairs; i0 += 4) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const float4 A = L.p0(i0 + ii), B = L.p1(i0 + ii);
      const f4v Wt = L.W[i0 + ii];
      const f2 W = f2{Wt.x, Wt.y};
      const f2 ex = fma2(HK, lo(A), KPX), ey = fma2(HK, hi(A), KPY), ez = fma2(HK, lo(B), KPZ);
      const f2 Q = fma2(ez, ez, fma2(ey, ey, fma2(ex, ex, E2)));
      f2 q[6] = {fma2(ex, TE, Q), fma2(ex, NTE, Q), fma2(ey, TE, Q), fma2(ey, NTE, Q), fma2(ez, TE, Q),
                 fma2(ez, NTE, Q)};
#pragma unroll
      for (int t = 0; t < 6; ++t) {
        if constexpr (CLAMP) q[t] = f2{qclamp(q[t].x, QMIN.x), qclamp(q[t].y, QMIN.y)};
        acc[t] = fma2(W, exp2v(-sqrt2(q[t])), acc[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 6; ++t) s[t] = acc[t].x + acc[t].y;
}

// Distances delta_j = rho_j - r_j at p_final for a pair (shade sweep and backward sweep 1 share it).
template <bool CLAMP>
__device__ __forceinline__ f2 delta_pair(const f2& PX, const f2& PY, const f2& PZ, const f2& PP, const float4& A,
                                         const float4& B, const float4& R, f2& q_out, f2& rho_out) {
  f2 q = qpair(PX, PY, PZ, PP, A, B);
  q_out = q;
  if constexpr (CLAMP) q = clamp_q(q);
  rho_out = sqrt2(q);
  return rho_out - hi(R);
}
// The same with rho = q rsq(q): one transcendental gives rho and 1/rho (r_out). The differentiable
// modes' shade sweep and backward sweep 1 both use this form, so their delta agree bit for bit.
template <bool CLAMP>
__device__ __forceinline__ f2 delta_pair_rsq(const f2& PX, const f2& PY, const f2& PZ, const f2& PP, const float4& A,
                                             const float4& B, const float4& R, f2& q_out, f2& r_out) {
  f2 q = qpair(PX, PY, PZ, PP, A, B);
  q_out = q;
  if constexpr (CLAMP) q = clamp_q(q);
  r_out = rsq2(q);
  return q * r_out - hi(R);
}

// Shared sweep at p_final: colour softmax over -csharp*delta (renderer_diff.rs:74-82) and the mask
// soft-min over -k*delta (renderer_diff.rs:86). Both maxima sit at min delta, so one running
// minimum dmin shifts both sums; exponents are (dmin - delta) <= 0 exactly (never overflow).
template <bool CLAMP>
__device__ __forceinline__ void shade_sweep(const float p[3], const Lds& L, int npairs, float c10l, float kappa,
                                            float& dmin, f2& Zw, f2 (&C)[3], f2& Zb) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), CL = sp(c10l), KA = sp(kappa);
  for (int i0 = 0; i0 < npairs; i0 += 4) {
    f2 dl[4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      f2 q, rho;
      dl[ii] = delta_pair<CLAMP>(PX, PY, PZ, PP, L.p0(i0 + ii), L.p1(i0 + ii), L.p2(i0 + ii), q, rho);
    }
    float cmin = fminf(dl[0].x, dl[0].y);
#pragma unroll
    for (int ii = 1; ii < 4; ++ii) cmin = fminf(cmin, fminf(dl[ii].x, dl[ii].y));
    const float dn = fminf(dmin, cmin);
    const f2 sw = sp(fexp2((dn - dmin) * c10l)), sb = sp(fexp2((dn - dmin) * kappa));
    Zw *= sw;
    C[0] *= sw;
    C[1] *= sw;
    C[2] *= sw;
    Zb *= sb;
    dmin = dn;
    const f2 DN = sp(dn);
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const f2 dd = DN - dl[ii];
      const f2 ew = exp2v(dd * CL), eb = exp2v(dd * KA);
      const float4 c3 = L.p3(i0 + ii);
      const float2 c4 = L.p4(i0 + ii);
      Zw += ew;
      C[0] = fma2(ew, lo(c3), C[0]);
      C[1] = fma2(ew, hi(c3), C[1]);
      C[2] = fma2(ew, f2{c4.x, c4.y}, C[2]);
      Zb += eb;
    }
  }
}

// The differentiable modes' sweep at p_final: shade_sweep's sums plus the detached normal
// (scene.rs:81-128, as its eps -> 0 limit f = 2 eps grad D) in the same pass. grad D =
// sum_j beta_j (p - c_j) / rho_j with beta = softmax(-k delta) -- the mask soft-min's own
// weights 2^(kappa (dmin - delta_j)) / Zb -- so G accumulates eb (p - c_j) rsq(q_j) next to Zb,
// rescaled with it when dmin moves (f = 2 eps G / Zb). One rsq per sphere gives rho and 1/rho.
template <bool CLAMP>
__device__ __forceinline__ void shade_normal_sweep(const float p[3], const Lds& L, int npairs, float c10l,
                                                   float kappa, float& dmin, f2& Zw, f2 (&C)[3], f2& Zb,
                                                   f2 (&G)[3]) {
  const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), CL = sp(c10l), KA = sp(kappa),
           HALF = sp(0.5f);
  for (int i0 = 0; i0 < npairs; i0 += 4) {
    f2 dl[4], r[4];
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      f2 q;
      dl[ii] = delta_pair_rsq<CLAMP>(PX, PY, PZ, PP, L.p0(i0 + ii), L.p1(i0 + ii), L.p2(i0 + ii), q, r[ii]);
      if constexpr (CLAMP) {  // clamp_min(1e-6): that distance is constant, no gradient
        r[ii].x = q.x >= 1e-6f ? r[ii].x : 0.0f;
        r[ii].y = q.y >= 1e-6f ? r[ii].y : 0.0f;
      }
    }
    float cmin = fminf(dl[0].x, dl[0].y);
#pragma unroll
    for (int ii = 1; ii < 4; ++ii) cmin = fminf(cmin, fminf(dl[ii].x, dl[ii].y));
    const float dn = fminf(dmin, cmin);
    const f2 sw = sp(fexp2((dn - dmin) * c10l)), sb = sp(fexp2((dn - dmin) * kappa));
    Zw *= sw;
    C[0] *= sw;
    C[1] *= sw;
    C[2] *= sw;
    Zb *= sb;
    G[0] *= sb;
    G[1] *= sb;
    G[2] *= sb;
    dmin = dn;
    const f2 DN = sp(dn);
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const f2 dd = DN - dl[ii];
      const f2 ew = exp2v(dd * CL), eb = exp2v(dd * KA);
      const float4 c3 = L.p3(i0 + ii), A = L.p0(i0 + ii), B = L.p1(i0 + ii);
      const float2 c4 = L.p4(i0 + ii);
      Zw += ew;
      C[0] = fma2(ew, lo(c3), C[0]);
      C[1] = fma2(ew, hi(c3), C[1]);
      C[2] = fma2(ew, f2{c4.x, c4.y}, C[2]);
      Zb += eb;
      const f2 wr = eb * r[ii];  // p - c = 0.5 (-2c) + p, exactly as the backward's
      G[0] = fma2(wr, fma2(HALF, lo(A), PX), G[0]);
      G[1] = fma2(wr, fma2(HALF, hi(A), PY), G[1]);
      G[2] = fma2(wr, fma2(HALF, lo(B), PZ), G[2]);
    }
  }
}

// ---- the fused per-ray kernel ----------------------------------------------------------
// Does the ray provably end (after `steps` march steps, or at the given march t) at scene
// distance >= min_d, beyond its closest approach to the scene's bounding sphere (c0, R)?
//  * Every sphere distance is >= |p - c0| - R, and the soft-min is >= the hard min minus
//    ln(M)/k (sdf.rs:30-44), so g(t) = |o + d t - c0| - R - ln(M)/k never exceeds the march
//    step D(t). Shrinking g by a relative 1e-5 and an absolute 1e-5 (R + |c0| + 1) covers the
//    f32 rounding of the march (expansion-form distances err by ~6e-8 |p|).
//  * t + g(t) is non-decreasing (g is (1 - 1e-5)-Lipschitz), so the f64 march of g alone,
//    tau <- tau + g(tau), stays below the real t at every step (induction from t = tau = 0).
//  * Past the closest approach g only grows; so tau_S >= t_closest and g(tau_S) >= min_d give
//    D >= min_d at the march end, at the reconnected point t + D (renderer_diff.rs:30-39) and
//    hence for the mask, which is then exactly 0 -- as are out and every gradient term.
__device__ __forceinline__ bool escapes(const float o[3], const float d[3], float t_given, bool have_t, int steps,
                                     const float c0[3], float R, float slack, float min_d) {
  const double eps = 1e-5;
  const double ox = (double)o[0] - c0[0], oy = (double)o[1] - c0[1], oz = (double)o[2] - c0[2];
  const double dx = d[0], dy = d[1], dz = d[2];
  const double Rs = (double)R + (double)slack;
  const double K = eps * (Rs + sqrt((double)c0[0] * c0[0] + (double)c0[1] * c0[1] + (double)c0[2] * c0[2]) + 1.0);
  auto g = [&](double tt) {
    const double x = fma(dx, tt, ox), y = fma(dy, tt, oy), z = fma(dz, tt, oz);
    return (1.0 - eps) * (sqrt(x * x + y * y + z * z) - Rs) - K;
  };
  const double tc = -(ox * dx + oy * dy + oz * dz) / (dx * dx + dy * dy + dz * dz);
  double tau = 0.0;
  if (have_t) {
    tau = t_given;
  } else {
    for (int s = 0; s < steps; ++s) tau += g(tau);
  }
  return tau >= tc && g(tau) >= (double)min_d;
}

// The cost-ordered dispatch's list sets of this launch: with a.oturn the pointers of KArgs are
// set 0's and the sets follow the device turn word w: read (w + 2) % 3, append w, clear (w + 1) % 3.
struct OrderSets {
  const int* list_r;
  const int* cnt_r;
  int* list_w;
  int* cnt_w;
  int* cnt_z;
};
__device__ __forceinline__ OrderSets order_sets(const KArgs& a) {
  OrderSets o{a.olist_r, a.ocnt_r, a.olist_w, a.ocnt_w, a.ocnt_z};
  if (a.oturn != nullptr) {
    const int w = __builtin_amdgcn_readfirstlane(*a.oturn);
    const int r = (w + 2) % 3, z = (w + 1) % 3;
    constexpr long long kSet = (long long)RM_ORDER_CLASSES * kMaxBlocksPerLaunch;
    if (o.list_r != nullptr) {
      o.list_r += r * kSet;
      o.cnt_r += r * RM_ORDER_CNT_STRIDE;
    }
    if (o.list_w != nullptr) {
      o.list_w += w * kSet;
      o.cnt_w += w * RM_ORDER_CNT_STRIDE;
    }
    if (o.cnt_z != nullptr) o.cnt_z += z * RM_ORDER_CNT_STRIDE;
  }
  return o;
}

// Launch position -> logical ray block. With block_order (whole 16x16-tiled views per launch) the
// blocks are dispatched tile rank by tile rank, the views interleaved, in the order of
// block_order: the tiles nearest the image centre -- where the scene usually is, and so the
// rays that march all their steps -- first, the cheap border tiles last, where they fill the
// machine while the heavy blocks finish. Partials stay indexed by the logical block, so the
// gradient sums (and every result) do not depend on the order.
__device__ __forceinline__ long long ray_block(const KArgs& a, int* cls = nullptr) {
  int b = blockIdx.x;
  if (a.block_order == nullptr) return b;
  // The dispatcher hands block i to XCD i % 8. With the views interleaved (b = rank * V + v),
  // V = 2 or 4 would pin each view to a fixed subset of XCDs, and views differ in cost (how much
  // of the scene they see): the XCDs of the dearest view finish last. Rotating the positions
  // inside every full round of 8 blocks by the round number makes each XCD cycle through all
  // views (rank order is kept up to 8 positions, so heavy tiles still start first).
#ifndef RM_XCD_ROTATE
#define RM_XCD_ROTATE 1
#endif
#if RM_XCD_ROTATE
  const int g = b >> 3;
  if ((g + 1) * 8 <= (int)gridDim.x) b = (g << 3) + (((b & 7) + g) & 7);
#endif
  const OrderSets os = order_sets(a);
  if (os.cnt_r != nullptr) {
    // position b of the class-major concatenation of the previous launch's lists; every block
    // reads the same counts, so a short total (never expected) sends all blocks to the static order
    int tot = 0, cb = -1, base = 0;
#pragma unroll
    for (int c = 0; c < RM_ORDER_CLASSES; ++c) {
      const int n = os.cnt_r[c * RM_ORDER_CLS_STRIDE];
      if (cb < 0 && b < tot + n) {
        cb = c;
        base = tot;
      }
      tot += n;
    }
    if (tot == (int)gridDim.x && cb >= 0) {
      if (cls != nullptr) *cls = cb;
      return os.list_r[cb * kMaxBlocksPerLaunch + (b - base)];
    }
  }
  const int r = b / a.order_views, v = b - r * a.order_views;
  return (long long)v * a.order_tiles + a.block_order[r];
}

// Appends the block to its cost class's list for the next launch's dispatch order (class 0: the
// dearest blocks; cost in march-step units, see the hand-off in rm_ray_kernel).
__device__ __forceinline__ void order_append(const KArgs& a, long long blk, int cost) {
  constexpr int kCls = RM_ORDER_CLASSES;
  const float cls_scale = (float)kCls / (float)((a.split ? 1 : kWaves) * (a.steps + kPostCost) + 1);
  const int c = kCls - 1 - (int)fminf((float)cost * cls_scale, (float)(kCls - 1));
  const OrderSets os = order_sets(a);
  const int idx = atomicAdd(os.cnt_w + c * RM_ORDER_CLS_STRIDE, 1);
  // counts left uncleared (a failed launch in the rotation) overrun the total, and ray_block
  // then falls back to the static order: never write past the list
  if (idx < kMaxBlocksPerLaunch) os.list_w[c * kMaxBlocksPerLaunch + idx] = (int)blk;
}

// compute_loss's progress (training.rs:17-34 weights): the call's argument, or with device step
// scalars bound (rm_bind_step_scalars) index / total in fp32 as train.rs:171-172 forms it.
__device__ __forceinline__ float progress_of(const KArgs& a) {
  if (a.sdev == nullptr) return a.progress;
  return fminf((float)a.sdev->index / (float)a.sdev->total, 1.0f);
}

// A block of escaping rays: out = 0 (requested outputs), zero gradient partials, and for the
// train step the L1 loss of out = 0, reduced exactly as in the full path.
template <int MODE>
__device__ __forceinline__ void escaped_block(const KArgs& a, const Lds& L, long long blk, long long ri, bool valid,
                                           int tid, int lane, int wave) {
  if (MODE != kBwd && a.out != nullptr && valid) {
    a.out[3 * ri] = 0.0f;
    a.out[3 * ri + 1] = 0.0f;
    a.out[3 * ri + 2] = 0.0f;
  }
  if constexpr (MODE == kFwd || MODE == kRender) return;
  float* rec = a.partials + blk * a.rec;  // per-sphere columns stay unwritten: live flag 0
  float loss = 0.0f;
  if (MODE == kTrain && valid) {  // training.rs:17-34 with out = 0
    const float t0 = a.targets[3 * ri], t1 = a.targets[3 * ri + 1], t2 = a.targets[3 * ri + 2];
    const float W = (t0 + t1 + t2) > 0.01f ? 10.0f : fmaf(progress_of(a), 4.0f, 1.0f);
    const float tg[3] = {t0, t1, t2};
#pragma unroll
    for (int c = 0; c < 3; ++c) loss = fmaf(fabsf(0.0f - tg[c]), W, loss);
  }
  const float vals[8] = {0.0f, 0.0f, 0.0f, 0.0f, loss, 0.0f, 0.0f, 0.0f};
  const float red = wave_reduce8(vals, lane);
  if ((lane & 7) == 7) L.slots[wave * 8 + (lane >> 3)] = red;
  __syncthreads();
  if (tid < 8) {
    float acc = L.slots[tid];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) acc += L.slots[w * 8 + tid];
    rec[(long long)a.Mpad * 8 + tid] = acc;
  }
}

// Ray of thread row ri (camera.rs:58-87 in camera mode). In camera mode ri is remapped from
// the launch order (16x16 pixel tiles per block, 8x8 per wave) to the pixel's row of the
// [N,3] tensors.
template <bool CAM>
__device__ __forceinline__ void setup_ray(const KArgs& a, long long& ri, float o[3], float d[3], int& view) {
  view = 0;
  if constexpr (CAM) {
    const long long npix = (long long)a.width * a.height;
    const int v = (int)(ri / npix);
    view = v;
    const long long pix = ri - (long long)v * npix;
    int x, y;
    if (a.tiling == 2) {
      // a block takes a 16x16 tile, each wave an 8x8 quadrant: compact ray bundles keep the
      // wave-uniform fast paths on and let whole blocks pass the escape test
      const long long tl = pix >> 8;
      const int w = (int)(pix & 255), tiles_x = a.width >> 4;
      const int ty = (int)(tl / tiles_x), tx = (int)(tl - (long long)ty * tiles_x);
      const int qd = w >> 6, l = w & 63;
      y = (ty << 4) + ((qd >> 1) << 3) + (l >> 3);
      x = (tx << 4) + ((qd & 1) << 3) + (l & 7);
    } else {
      y = (int)(pix / a.width);
      x = (int)(pix - (long long)y * a.width);
    }
    ri = (long long)v * npix + (long long)y * a.width + x;
    if (a.cams_dev != nullptr) camera_ray(a.cams_dev[v], x, y, a.width, a.height, o, d);
    else camera_ray(a.cams[v], x, y, a.width, a.height, o, d);
  } else {
    o[0] = a.org[3 * ri];
    o[1] = a.org[3 * ri + 1];
    o[2] = a.org[3 * ri + 2];
    d[0] = a.dir[3 * ri];
    d[1] = a.dir[3 * ri + 1];
    d[2] = a.dir[3 * ri + 2];
  }
}

// Escape pre-pass (RM_MARCH_SKIP_ESCAPED): one thread per ray of the coming per-ray launch
// (same blocks, same rays); flags[b] = 1 when every ray of block b escapes. Kept out of the
// per-ray kernel so its f64 arithmetic costs that kernel no registers.
template <int MODE, bool CAM>
__global__ __launch_bounds__(kBlock) void rm_escape_kernel(const KArgs a, int* __restrict__ flags) {
  __shared__ float scratch[8 * kWaves];
  const int tid = threadIdx.x;
  const long long blk = ray_block(a);
  const long long li = blk * kBlock + tid;
  const bool valid = li < a.n_rays;
  long long ri = a.ray_begin + (valid ? li : 0);
  float o[3], d[3];
  int view;
  setup_ray<CAM>(a, ri, o, d, view);
  float c0[3], R;
  scene_bound(a, scratch, tid, c0, R);
  const bool have_t = MODE == kBwd && a.t_in != nullptr;
  const bool esc = !valid || escapes(o, d, have_t ? a.t_in[ri] : -1.0f, have_t, a.steps, c0, R, a.lse_slack,
                                     a.cull_min_d);
  const int all = __syncthreads_and(esc);
  if (tid == 0) flags[blk] = all;
}

template <int MODE, bool CAM, bool SPLIT>
__device__ __forceinline__ void ray_body(const KArgs& a);

// The per-ray kernel. Measurement build (-DRM_BLOCK_TRACE): every wave also records {start, end}
// (s_memrealtime, 100 MHz), its hardware slot (HW_ID | XCC_ID << 32), {logical block, launch
// position}, the times its march and its post-march forward ended and its march steps saved into
// a.btrace[kTraceWords * (blockIdx.x * kWaves + wave) ...] (tools/block_trace.py).
// SPLIT: the split march (RM_MARCH_SPLIT, KArgs::split).
template <int MODE, bool CAM, bool SPLIT>
__device__ __forceinline__ void ray_entry(const KArgs& a) {
#ifdef RM_BLOCK_TRACE
  const unsigned long long t_begin = __builtin_amdgcn_s_memrealtime();
  ray_body<MODE, CAM, SPLIT>(a);
  const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
  if (a.btrace != nullptr && (threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    unsigned long long* r = a.btrace + kTraceWords * ((unsigned long long)blockIdx.x * kWaves + (threadIdx.x >> 6));
    r[0] = t_begin;
    r[1] = t_end;
    r[2] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    r[3] = (unsigned long long)ray_block(a) | ((unsigned long long)blockIdx.x << 32);
  }
#else
  ray_body<MODE, CAM, SPLIT>(a);
#endif
}
template <int MODE, bool CAM, bool SPLIT>
__global__ __launch_bounds__(kBlock, SPLIT ? RM_SPLIT_MIN_WAVES : kMinWavesPerSimd) void rm_ray_kernel(const KArgs a) {
  ray_entry<MODE, CAM, SPLIT>(a);
}
// The split continuation launch (KArgs::cont_resume > 0) as its own kernel: the same code at the
// register budget RM_CONT_MIN_WAVES (waves per SIMD), so that more of its blocks are resident at once.
template <int MODE, bool CAM>
__global__ __launch_bounds__(kBlock, RM_CONT_MIN_WAVES) void rm_cont_kernel(const KArgs a) {
  ray_entry<MODE, CAM, true>(a);
}

// Split march (SPLIT): a block takes 64 rays (one 8x8 quadrant of a 16x16 tile in camera mode)
// and all four of its waves hold them; every march step each wave sums a quarter of the sphere
// row blocks on the matrix cores and the quarters are added in wave order (split_combine), so
// the four waves march in lockstep through identical decisions (shift, clamp, exit). After the
// march only wave 0 goes on (post-march forward, backward); the others end as escaped waves
// with zero contributions. A ray that marches every step then occupies four SIMDs instead of one.
template <int MODE, bool CAM, bool SPLIT>
__device__ __forceinline__ void ray_body(const KArgs& a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
#ifdef RM_RAY_STATS
  __shared__ unsigned rs_w[3];  // measurement build (see the march)
#endif
  Lds L;
  {
    const int np = a.Mpad / 2;
    L.P0 = (cf4_ptr)a.rec_buf;
    L.P1 = L.P0 + np;
    L.P2 = L.P1 + np;
    L.P3 = L.P2 + np;
    L.S0 = L.P3 + np;
    L.S1 = L.S0 + np;
    L.W = L.S1 + np;
    L.P4 = (cf2_ptr)(L.W + np);
    L.At = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.rec_buf) + tiles_offset(np, (np + 255) / 256));
    L.Wt = reinterpret_cast<const float*>(L.At + (size_t)(np / 8) * 64);
  }
  L.slots = reinterpret_cast<float*>(smem);
  L.misc = L.slots + kSlotBytes / sizeof(float);

  // wave: the wave's index, made scalar (readfirstlane) so that everything derived from it -- a
  // split wave's quarter of the row blocks, its loop bounds and fragment addresses, LDS slots --
  // stays wave-uniform for the compiler (threadIdx-derived values are otherwise vector values)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int cls = -1;  // the block's cost class in the previous launch (cost-ordered dispatch), else -1
  long long blk;
  // ray_cont (ray mode): this block marches listed rays [32 b, 32 b + 32) of ray_list, one per lane
  // (lanes l and l + 32 the same ray); lanes past the list's end are invalid copies of its first
  long long li_listed = -1;
  bool listed = true;
  if (SPLIT && a.cont_resume > 0 && a.ray_cont) {
    const int n = *a.ray_count;
    const int i0 = (int)blockIdx.x * kSplitRays;
    if (i0 >= n) return;
    const int i = i0 + (lane & (kSplitRays - 1));
    listed = i < n;
    li_listed = a.ray_list[listed ? i : i0];
    blk = -1;  // no group of its own
  } else if (SPLIT && a.cont_resume > 0) {  // continuation launch: the blocks the first launch deferred
    // position blockIdx.x of the class-major concatenation of the class lists
    int b = (int)blockIdx.x, c = 0;
    for (; c < kContClasses; ++c) {
      const int n = a.cont_count[c];
      if (b < n) break;
      b -= n;
    }
    if (c == kContClasses) return;
    blk = a.cont_list[(long long)c * a.cont_stride + b];
  } else {
    blk = ray_block(a, &cls);
  }
  // SPLIT: lane l holds ray l mod kSplitRays of the group (kSplitRays < 64: copies, see kSplitRays)
  const long long li = li_listed >= 0 ? li_listed
                                      : (SPLIT ? blk * kSplitRays + (lane & (kSplitRays - 1)) : blk * kBlock + tid);
#if RM_HEAVY_PRIO
  // the dearest class's waves first at the SIMD's issue arbiter: they set the launch's critical
  // path, the cheaper waves fill the issue slots they leave
  if (cls >= 0 && cls < RM_HEAVY_PRIO) __builtin_amdgcn_s_setprio(2);
#endif
  const bool valid = listed && li < a.n_rays;
  long long ri = a.ray_begin + (valid ? li : 0);  // becomes the ray's row in the [N,3] tensors
  // the wave that writes this ray's outputs; SPLIT: all four waves run the post-march forward
  // (each over a quarter of the spheres, merged) and wave w seeds the backward of the group's rays
  // [w R / 4, (w + 1) R / 4) (R = kSplitRays; lanes past R carry copies and seed nothing)
  const bool own_rays = !SPLIT || (wave == 0 && lane < kSplitRays);
  const bool seed_lane = !SPLIT || (wave == 0 && lane < kSplitRays);

  const float kappa = a.k * kLog2e, nkappa = -kappa, inv_kappa = 1.0f / kappa;

  // ray (camera.rs:58-87 in camera mode)
  float o[3], d[3];
  int view;
  setup_ray<CAM>(a, ri, o, d, view);

  // ---- escape skip (RM_MARCH_SKIP_ESCAPED): a block whose rays all provably leave the scene
  // (rm_escape_kernel) gets out = 0 and zero gradients without marching -- exactly what the full
  // computation yields for them, since their silhouette mask is 0 in f32 (see escapes()).
  if (a.ocnt_z != nullptr && blockIdx.x == 0 && tid < RM_ORDER_CLASSES) order_sets(a).cnt_z[tid * RM_ORDER_CLS_STRIDE] = 0;
  if (a.esc_flags != nullptr && blk >= 0 && a.esc_flags[blk]) {
    if (a.stats != nullptr && tid == 0) atomicAdd(a.stats, 1ull);
    if (a.ocnt_w != nullptr && tid == 0) order_append(a, blk, 0);
    escaped_block<MODE>(a, L, blk, ri, valid, tid, lane, wave);
    return;
  }
#if RM_DEAD_EARLY
  if constexpr (!SPLIT && (MODE == kBwd || MODE == kTrain)) {
    // the hand-off's count of the waves that end early: zero before any wave can reach it
    if (tid == 0) reinterpret_cast<int*>(L.misc)[kDeadCountSlot] = 0;
    __syncthreads();
  }
#endif

  // Scene radius bounds from the record header: with r_min, a lower bound on the scene distance
  // proves rho_j = dist_j + r_j >= kSafeRho for every sphere, so max(q, 1e-6) cannot bind and
  // the sweeps may skip it (exactly the same results).
  const cf1_ptr hdr = (cf1_ptr)(L.P4 + a.Mpad / 2);
  const float rmin = hdr[0], rmax = hdr[1], spread = hdr[2];
  // Block-uniform permissions for the cheaper log-sum-exp shifts of the march:
  // |v_j - v_0| = kappa |r_j - r_0 - (rho_j - rho_0)| <= kappa (r_max + |c_j - c_0|); v <= kappa r_max;
  // the weighted form 2^(k r) 2^(-k rho) also needs 2^(-k rho) of the nearest sphere normal:
  // k rho <= 90 + k r_max <= 120
  // (RM_MARCH_FORCE_MAX_SHIFT: neither, every step takes the running maximum -- tests)
  const bool shift_fixed_ok = !a.shift_max && kappa * (rmax + spread) * 1.001f <= 100.0f;
  const bool shift_none_ok = !a.shift_max && kappa * rmax * 1.001f <= 30.0f;
  const float kr_first = kappa * a.radius[0];
  // Wave-uniform choice of the clamp-free path from a per-lane lower bound on the distance.
  // Rays proven to escape (`gone`, see the march) no longer take part in the wave-uniform
  // choices: their outputs and gradient terms are exactly 0 whatever they compute.
  bool gone = false;
  // Ray mode: the ray's state repeats with period 2; its t is final (see the march)
  bool retired = false;
  // A second proof per ray (camera mode): rho_lb, a lower bound on the distance to the nearest
  // sphere CENTRE -- the eye's (write_origins), less the path marched since (every centre distance
  // is 1-Lipschitz along the ray). Where the soft-min runs far below the hard min (small k: at
  // k = 5 by up to ln(M)/k = 1.1) the scene-distance bound above fails inside the scene long
  // before any centre comes near; either proof skips the clamp, with the same bits.
  float rho_lb = -INFINITY;
  const float onorm = fabsf(o[0]) + fabsf(o[1]) + fabsf(o[2]);
  // rho_lb after the ray moved from march distance t0 to t1 (|d| <= 1 + 1e-6; the fp32 rounding of
  // both points p = o + d t, ~1.1e-7 (|o|_1 + 1.74 t) each, inside the absolute 1e-6 (1 + |o|_1 + t))
  auto rho_moved = [&](float rl, float t0, float t1) {
    return rl - (fabsf(t1 - t0) * 1.000001f + 1e-6f * (1.0f + onorm + fmaxf(t0, t1)));
  };
  auto all_safe = [&](float dist_lb, float rlb) {
    return __all(dist_lb + rmin >= kSafeRho || rlb >= kSafeRho || gone) != 0;
  };
  int split_par = 0;  // SPLIT: which of the two combine buffers the next step uses

  // every sweep visits all sphere pairs in one pass (records are not staged)
  auto for_tiles = [&](auto&& body) { body(0, a.Mpad); };
  // soft-min scene SDF at one point (scene.rs:60-79 + sdf.rs:30-44); returns D, keeps (m, s)
  auto soft_min = [&](const float p[3], bool fast, float& m, float& s) {
    m = -INFINITY;
    s = 0.0f;
    if (fast)
      for_tiles([&](int, int tn) { lse_point<false, kShiftMax>(p, L, tn / 2, nkappa, m, s); });
    else
      for_tiles([&](int, int tn) { lse_point<true, kShiftMax>(p, L, tn / 2, nkappa, m, s); });
    return -(flog2(fmaxf(s, 1e-8f)) + m) * inv_kappa;
  };
  // SPLIT: the post-march vector sweeps of a 64-ray block run on its four waves, wave w over the
  // pairs [split_pair(w), split_pair(w + 1)) (multiples of 8), and the partial states are merged
  // through LDS in wave order (every wave then holds the same totals).
  auto split_pair = [&](int w) { return (((a.Mpad / 2) * w) / kSplitWaves) & ~7; };
  auto soft_min_split = [&](const float p[3], bool fast, float& m, float& s) {
    const int b0 = split_pair(wave), b1 = split_pair(wave + 1);
    const Lds Lq = L.from_pair(b0);
    m = -INFINITY;
    s = 0.0f;
    if (fast) lse_point<false, kShiftMax>(p, Lq, b1 - b0, nkappa, m, s);
    else lse_point<true, kShiftMax>(p, Lq, b1 - b0, nkappa, m, s);
    float* xm = L.slots;
    float* xs = L.slots + kSplitWaves * 64;
    __syncthreads();  // the march's last exchange is read
    xm[wave * 64 + lane] = m;
    xs[wave * 64 + lane] = s;
    __syncthreads();
    float mm = xm[lane];
#pragma unroll
    for (int w = 1; w < kSplitWaves; ++w) mm = fmaxf(mm, xm[w * 64 + lane]);
    float ss = 0.0f;
#pragma unroll
    for (int w = 0; w < kSplitWaves; ++w) ss += xs[w * 64 + lane] * fexp2(xm[w * 64 + lane] - mm);
    m = mm;
    s = ss;
    return -(flog2(fmaxf(s, 1e-8f)) + m) * inv_kappa;
  };
  // shade_normal_sweep's state (dmin; colour sums at c10l, mask and normal sums at kappa, each
  // relative to dmin) merged over the four waves; the totals come back in the .x lanes
  auto shade_merge = [&](float c10l, float& dmin, f2& Zw, f2 (&C)[3], f2& Zb, f2 (&G)[3]) {
    constexpr int kF = 9;
    float* xb = L.slots + 2 * kSplitWaves * 64;  // [kF][wave][64], after soft_min_split's buffers
    const float v[kF] = {dmin, Zw.x + Zw.y, C[0].x + C[0].y, C[1].x + C[1].y, C[2].x + C[2].y,
                         Zb.x + Zb.y, G[0].x + G[0].y, G[1].x + G[1].y, G[2].x + G[2].y};
#pragma unroll
    for (int f = 0; f < kF; ++f) xb[(f * kSplitWaves + wave) * 64 + lane] = v[f];
    __syncthreads();
    float dm = xb[lane];
#pragma unroll
    for (int w = 1; w < kSplitWaves; ++w) dm = fminf(dm, xb[w * 64 + lane]);
    float acc[kF - 1] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int w = 0; w < kSplitWaves; ++w) {
      const float dw = xb[w * 64 + lane];
      const float sw = fexp2((dm - dw) * c10l), sb = fexp2((dm - dw) * kappa);
#pragma unroll
      for (int f = 1; f < kF; ++f) acc[f - 1] = fmaf(xb[(f * kSplitWaves + w) * 64 + lane], f < 5 ? sw : sb, acc[f - 1]);
    }
    dmin = dm;
    Zw = f2{acc[0], 0.0f};
    C[0] = f2{acc[1], 0.0f};
    C[1] = f2{acc[2], 0.0f};
    C[2] = f2{acc[3], 0.0f};
    Zb = f2{acc[4], 0.0f};
    G[0] = f2{acc[5], 0.0f};
    G[1] = f2{acc[6], 0.0f};
    G[2] = f2{acc[7], 0.0f};
  };
  // The march's soft-min with the cheapest safe shift (the result differs only by fp32 rounding).
  // kShiftNone needs the hard maximum -kappa d_min >= -100 at the new point: d_min(new) <=
  // d_min(old) + |D| <= D + ln(M)/k + |D| (the soft-min is within ln(M)/k below the hard min).
#ifdef RM_BLOCK_TRACE
  // measurement build: march steps per path (16 bits each: none fast, none clamped, fixed fast,
  // fixed clamped), shader cycles inside the matrix-core steps, vector-path steps
  unsigned long long tr_paths = 0, tr_lse_cyc = 0, tr_vec = 0;
#endif
  // choice: the step's wave-uniform choices, bit 0 unshifted, bit 1 fixed shift, bit 2 clamp-free
  // force: 0 the cheapest safe shift for the wave (above); 1 the fixed shift, 2 the running maximum,
  // 3 unshifted (ray mode: see soft_min_march)
  auto soft_min_core = [&](const float p[3], bool fast, float Dprev, int& choice, int force) {
    bool none = force == 3 || (force == 0 && shift_none_ok &&
                __all(2.0f * fmaxf(Dprev, 0.0f) + a.lse_slack <= 90.0f * inv_kappa || gone));
    // or: the nearest sphere is no farther than sphere 0, k (rho_0 - r_0) = rho'_0 - k r_0 <= 90
    // bounds k d_min just as well (the first steps after the eye, where the 2 D bound is loose)
    if (!none && force == 0 && shift_none_ok && a.mfma)
      none = __all(fixed_shift(p, kappa * kappa, Lds::v4(L.S0[0]), Lds::v4(L.S1[0])) - kr_first <= 90.0f || gone);
    float m = none ? 0.0f : -INFINITY, s = 0.0f;
    const bool fixed = force == 1 || (force == 0 && !none && shift_fixed_ok && __all(psq(p) <= 1e10f || gone));
    choice = (none ? 1 : 0) | (fixed ? 2 : 0) | (fast ? 4 : 0);
    if ((none || fixed) && a.mfma) {
      const float k2 = kappa * kappa;
      // opaque per step: the row-block count's derived guards are formed here, not hoisted out
      // of the march loop as long-lived lane masks (SGPR pressure: spills to v_writelane)
      int nrb = a.Mpad / 16;
      asm volatile("" : "+s"(nrb));
      uint4* xa = reinterpret_cast<uint4*>(L.slots) + wave * 64;
      uint4* xb = reinterpret_cast<uint4*>(L.slots) + kWaves * 64 + wave * 64;
      float* xs = L.slots + kWaves * 64 * 8 + wave * 64;
#ifdef RM_BLOCK_TRACE
      const unsigned long long tq0 = __builtin_readcyclecounter();
      tr_paths += 1ull << (16 * ((fixed ? 2 : 0) + (fast ? 0 : 1)));
#endif
      float Dm;
      constexpr bool kBuf = RM_MARCH_BUFLOAD != 0;
      const uint4* At = L.At;
      const float* Wt = L.Wt;
      int nq = nrb;
      float* comb = nullptr;
      if constexpr (SPLIT) {  // this wave's quarter of the row blocks; combine buffers alternate
        const int r0 = part_rb(nrb, wave);
        nq = part_rb(nrb, wave + 1) - r0;
        At += (size_t)r0 * 64;
        Wt += (size_t)r0 * 32;
        comb = L.slots + kSplitCombOff + (split_par ^= 1) * (kWaves * 64);
      }
      constexpr int kNcb = SPLIT ? kSplitCB : 4;  // column blocks of this wave's rays
      if (fixed) {  // the ray's shift: rho'_0 of sphere 0 (any value near it keeps +-100 headroom)
        const float4 A = Lds::v4(L.S0[0]), B = Lds::v4(L.S1[0]);
        Dm = fast ? march_d_fixed<false, kBuf, kNcb>(p, kappa, inv_kappa, kr_first, A, B, At, Wt, nq, xa, xb, xs, lane, comb, wave)
                  : march_d_fixed<true, kBuf, kNcb>(p, kappa, inv_kappa, kr_first, A, B, At, Wt, nq, xa, xb, xs, lane, comb, wave);
      } else {
        Dm = fast ? march_d_none<false, kBuf, kNcb>(p, kappa, inv_kappa, At, Wt, nq, xa, xb, xs, lane, comb, wave)
                  : march_d_none<true, kBuf, kNcb>(p, kappa, inv_kappa, At, Wt, nq, xa, xb, xs, lane, comb, wave);
      }
      (void)k2;
#ifdef RM_BLOCK_TRACE
      tr_lse_cyc += __builtin_readcyclecounter() - tq0;
#endif
      return Dm;
    }
#ifdef RM_BLOCK_TRACE
    ++tr_vec;
#endif
    if (none || fixed) {
      const float k2 = kappa * kappa;
      const int np = a.Mpad / 2;
      float sh;
      if (none) {
        s = fast ? lse_weighted<false, false>(p, L, np, k2, sh) : lse_weighted<true, false>(p, L, np, k2, sh);
      } else {
        s = fast ? lse_weighted<false, true>(p, L, np, k2, sh) : lse_weighted<true, true>(p, L, np, k2, sh);
        m = kr_first - sh;
      }
      return -(flog2(fmaxf(s, 1e-30f)) + m) * inv_kappa;
    }
    if (none) {
      if (fast) for_tiles([&](int, int tn) { lse_point<false, kShiftNone>(p, L, tn / 2, nkappa, m, s); });
      else for_tiles([&](int, int tn) { lse_point<true, kShiftNone>(p, L, tn / 2, nkappa, m, s); });
    } else if (fixed) {
      // |p| <= 1e5: the expansion-form rounding of rho (~1.5 ulp(|p|)) moves the exponents by
      // < 0.5; far out it can exceed the +-100 headroom, so distant points keep the running max
      if (fast) for_tiles([&](int, int tn) { lse_point<false, kShiftFixed>(p, L, tn / 2, nkappa, m, s); });
      else for_tiles([&](int, int tn) { lse_point<true, kShiftFixed>(p, L, tn / 2, nkappa, m, s); });
    } else {
      if (fast) for_tiles([&](int, int tn) { lse_point<false, kShiftMax>(p, L, tn / 2, nkappa, m, s); });
      else for_tiles([&](int, int tn) { lse_point<true, kShiftMax>(p, L, tn / 2, nkappa, m, s); });
    }
    return -(flog2(fmaxf(s, 1e-30f)) + m) * inv_kappa;
  };
  // The march's soft-min. Ray mode (the split kernels): each ray's own choice, so that its step is
  // a function of its own state (its p and previous D) -- unshifted when the ray's own bound admits
  // it (the tests of soft_min_core, per ray), else the scene-uniform fixed shift when its |p| admits
  // it (|p| <= 1e5, the fixed form's fp32 headroom), else the running maximum (a vector sweep over
  // all spheres, lane by lane); a wave runs each form only when one of its live rays takes it
  // (two forms in the waves whose rays disagree).
  auto soft_min_march = [&](const float p[3], bool fast, float Dprev, int& choice) {
    if constexpr (SPLIT) {
      const bool live = !gone && !retired;
      bool nr = live && shift_none_ok && 2.0f * fmaxf(Dprev, 0.0f) + a.lse_slack <= 90.0f * inv_kappa;
      if (live && !nr && shift_none_ok && a.mfma)
        nr = fixed_shift(p, kappa * kappa, Lds::v4(L.S0[0]), Lds::v4(L.S1[0])) - kr_first <= 90.0f;
      const bool far = live && !nr && !(psq(p) <= 1e10f);
      const bool use_fixed = !nr && shift_fixed_ok && !far;
      unsigned long long bn = __ballot(nr);
      const unsigned long long bf = __ballot(live && use_fixed), bx = __ballot(live && !nr && !use_fixed);
      // exit off (the capability measurement: every ray does every step's work): a wave whose
      // rays are all gone still runs a sweep, as the wave-uniform march does (results unused)
      if (!a.early_exit && (bn | bf | bx) == 0ull) bn = 1ull;
      int cm = 0;
      float Dn = 0.0f, Dm = 0.0f, Dx = 0.0f;
      if (bn != 0ull) Dn = soft_min_core(p, fast, Dprev, cm, 3);
      if (bf != 0ull) Dm = soft_min_core(p, fast, Dprev, cm, 1);
      if (bx != 0ull) Dx = soft_min_core(p, fast, Dprev, cm, 2);
      choice = (nr ? 1 : 0) | (use_fixed ? 2 : 0) | (fast ? 4 : 0);
      return nr ? Dn : (use_fixed ? Dm : Dx);
    } else {
      return soft_min_core(p, fast, Dprev, choice, 0);
    }
  };

  // ---- march: t <- (t + sdf(o + d t)).detach(), S times (renderer_diff.rs:20-26)
  // The fast path needs a distance lower bound: the previous point's hard minimum (>= its
  // soft-min D) minus the step just taken (every dist_j is 1-Lipschitz and |d| = 1).
  float t = 0.0f;
  float lb = -INFINITY;  // lower bound on the scene distance at the current point
  float Dprev = INFINITY;  // previous march step (none yet)
  bool dead = false;       // wave-uniform: every ray of the wave has escaped (see below)
  int steps_saved = 0;     // wave-uniform: march steps this wave did not run (work statistics)
  // the scene's bounding sphere (c, R) (scene_bound, in the record header); R' = R + soft-min
  // slack + 1e-3 (fp32 margin of the march)
  const float c0x = hdr[4], c0y = hdr[5], c0z = hdr[6];
  const cf1_ptr esc_tab = (cf1_ptr)(reinterpret_cast<const char*>(a.rec_buf) + esc_offset(a.Mpad / 2, (a.Mpad / 2 + 255) / 256));
  if (MODE == kBwd && a.t_in != nullptr) {
    t = a.t_in[ri];
  } else {
#if RM_PRIO_RAMP
    // Equalise progress of the waves sharing a SIMD: VALU issue is arbitrated by priority,
    // then age, so without this the oldest wave races ahead and the youngest finishes last
    // (alone, latency-bound) -- a ~14% tail when one launch fills the GPU exactly once.
    // A wave lowers its priority as it passes checkpoints (march halves, post-march forward,
    // backward), so laggards win the arbitration.
    __builtin_amdgcn_s_setprio(3);
    const int half = max(a.steps / 2, 1);
#endif
    // Escaped rays: receding from the scene's bounding sphere (c_0, R) with every later
    // soft-min >= |p - c_0| - R - ln(M)/k >= gone_d (the distance only grows along a
    // receding ray, so t keeps increasing); the reconnected point and the mask argument
    // are then >= gone_d too, where sigmoid(-msharp D) (or exp(-10 D^2)) is exactly 0 in
    // fp32: out = 0 and every gradient term is 0, whatever the remaining steps would give.
    // Margins: 1e-5 relative + 1e-3 cover the fp32 rounding of the march at any |p|.
    // Each remaining step is >= dist - R' long and keeps the ray receding, so the distance
    // grows step by step (write_bound): with n steps left the ray is gone once
    // (1 - 1e-5) dist >= T(n) -- proven long before the ray gets there.
    // A gone ray (sticky) steps by that bound, dist - R', instead of its soft-min: the proof
    // holds for any steps >= the bound, so its outputs stay exactly 0, and it leaves the
    // wave's shift / clamp choices (far points would force the running-max vector sweep on
    // the whole wave: 48 % of the march steps at 4096 spheres / 128 steps). A wave whose
    // rays are all gone stops (a.early_exit). The same in every mode that builds the table,
    // exit on or off, so both give the same bits.
    const float rprime = (hdr[7] + a.lse_slack + 1e-3f) * (1.0f + 1e-6f);  // R' as in write_bound
#ifdef RM_LANE_STATS  // measurement build: lane-steps of escaped (or invalid) rays in marching waves
    unsigned long long lane_gone_steps = 0;
    int lanes_gone_last = 0;
#endif
    float gone_step = 0.0f;  // dist - R' of a gone ray at the current point
    auto wave_escaped = [&](int st, const float p[3]) {
      if (!(a.gone_d > 0.0f)) return false;
      const float ex = p[0] - c0x, ey = p[1] - c0y, ez = p[2] - c0z;
      const float Tn = esc_tab[min(a.steps - st, kEscTab - 1)];
      const float dist = fsqrt(fmaf(ez, ez, fmaf(ey, ey, ex * ex)));
      gone = gone || (!retired && fmaf(ez, d[2], fmaf(ey, d[1], ex * d[0])) >= 0.0f && dist * (1.0f - 1e-5f) >= Tn);
      gone_step = dist - rprime;
      if (a.early_exit && __all(gone || !valid)) {
        steps_saved += a.steps - st;
        return true;
      }
#ifdef RM_LANE_STATS
      lane_gone_steps += __popcll(__ballot(gone || !valid));
      lanes_gone_last = __popcll(__ballot(gone || !valid));
#endif
      return false;
    };
    // A gone ray's remaining bound steps from step `from` to the end (what the march would do):
    // where the march of its wave stops early but its rays' final states are used later (ray mode:
    // the continuation caps and the listed rays' write-back) -- a gone ray's mask is exactly 0
    // only where the bound steps end, not where it was proven
    auto gone_finish = [&](int from) {
      if (gone && !retired)
        for (int k = from; k < a.steps; ++k) {
          const float q[3] = {fmaf(d[0], t, o[0]) - c0x, fmaf(d[1], t, o[1]) - c0y, fmaf(d[2], t, o[2]) - c0z};
          t = fminf(t + (fsqrt(fmaf(q[2], q[2], fmaf(q[1], q[1], q[0] * q[0]))) - rprime), kTMax);
        }
    };
    int st_stop = -1;  // the step at which the march found every ray of the wave gone (not taken)
    int st0 = 0;
#ifdef RM_BLOCK_TRACE
    const unsigned long long tr_c_begin = __builtin_readcyclecounter();
    unsigned long long tr_cyc = 0;  // period | step << 8 of the cycle exit
#endif
    if constexpr (CAM) {
      // Camera mode: step 0 from the soft-min at the eye, evaluated once per view by the same
      // code path (write_origins), when every lane of the wave has it (not NaN). Taken before
      // the loop so that D0 holds no register through the march.
      if (a.origin != nullptr && a.steps > 0 && !(SPLIT && a.cont_resume > 0)) {
        const float D0 = a.origin[view];
        rho_lb = a.origin[RM_MAX_VIEWS_PER_CALL + view];  // at the eye
        if (__all((__float_as_uint(D0) & 0x7fffffffu) <= 0x7f800000u)) {
          const float p[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
          if (wave_escaped(0, p)) {
            dead = true;
          } else {  // == soft_min_march(p, all_safe(-inf) = false, inf) at p = o = the eye
            t = fminf(t + (gone ? gone_step : D0), kTMax);
            rho_lb = rho_moved(rho_lb, 0.0f, t);
            lb = D0 - fabsf(D0);
            Dprev = D0;
            st0 = 1;
            steps_saved = 1;  // a step this wave did not run
          }
        }
      }
    }
    // the cycle exit's history: t one to four steps back, and the choices (3 bits per step,
    // the latest in the low bits; 7 is no valid choice)
    float cyc_t1 = __builtin_nanf(""), cyc_t2 = __builtin_nanf("");
#if RM_CYCLE_MAX >= 3
    float cyc_t3 = __builtin_nanf("");
#endif
#if RM_CYCLE_MAX >= 4
    float cyc_t4 = __builtin_nanf("");
#endif
    int chist = 0xFFF;
    int rhist = 0xFFF;  // ray mode: the ray's own choice history (per lane: listed rays come from many groups)
    static_assert(RM_CYCLE_MAX == 2 || !SPLIT, "the continuation saves two steps of history");
    if (SPLIT && a.cont_resume > 0) {  // the state the first launch saved at step cont_resume
      const float* cs = a.cont_state;
      const long long R = a.cont_rays;
      const long long G = (SPLIT ? 8 : 7) * R;  // the per-group words after the per-ray rows
      t = cs[li];
      lb = cs[R + li];
      Dprev = cs[2 * R + li];
      cyc_t1 = cs[3 * R + li];
      cyc_t2 = cs[4 * R + li];
      const float gflag = cs[5 * R + li];  // ray mode: 1 gone, 2 retired; else non-zero = gone
      gone = SPLIT ? gflag == 1.0f : gflag != 0.0f;
      retired = SPLIT && gflag == 2.0f;
      rho_lb = cs[6 * R + li];
      if (SPLIT) rhist = __float_as_int(cs[7 * R + li]);
      if (!a.ray_cont) {
        chist = __float_as_int(cs[G + 2 * blk]);
        steps_saved = __float_as_int(cs[G + 2 * blk + 1]);
      }
      st0 = a.cont_resume;
    }
    const unsigned long long below = (1ull << lane) - 1ull;
#ifdef RM_RAY_STATS  // measurement build: the march steps each ray needs (until gone or period 2)
    int ray_need = st0;
    // and what packing a block's rays still marching at step RM_RAY_STATS_CAP into the fewest
    // waves would leave of its waves' steps after it (unsplit): live rays, summed steps, max steps
    if (tid < 3) rs_w[tid] = 0u;
    __syncthreads();
    bool rs_at = false;
    int rs_last = st0 - 1;
#endif
    for (int st = st0; !dead && st < a.steps; ++st) {
      if (SPLIT && a.cont_cap > 0 && st == a.cont_cap) {
        // ray mode, defer at the top of this step: every ray's state, the marching rays to the
        // ray list; a group (not a ray_cont block) also to the resume list, its not-run steps
        // counted as saved now (the ray_cont blocks subtract the steps they run)
        float* cs = a.cont_state;
        const long long R = a.cont_rays;
        const bool act = valid && !gone && !retired && lane < kSplitRays;
        gone_finish(st);
        if (wave == 0 && lane < kSplitRays && valid) {
          cs[li] = t;
          cs[R + li] = lb;
          cs[2 * R + li] = Dprev;
          cs[3 * R + li] = cyc_t1;
          cs[4 * R + li] = cyc_t2;
          cs[5 * R + li] = gone ? 1.0f : (retired ? 2.0f : 0.0f);
          cs[6 * R + li] = rho_lb;
          cs[7 * R + li] = __int_as_float(rhist);
        }
        if (wave == 0) {
          const unsigned long long am = __ballot(act);
          const int na = __popcll(am);
          int base = 0;
          if (lane == 0 && na > 0) base = atomicAdd(a.ray_count_w, na);
          base = __shfl(base, 0);
          if (act) a.ray_list_w[base + __popcll(am & below)] = (int)li;
          if (lane == 0) {
            if (!a.ray_cont) {
              cs[8 * R + 2 * blk] = __int_as_float(chist);
              cs[8 * R + 2 * blk + 1] = __int_as_float(steps_saved + (a.steps - st));
              a.cont_list_w[atomicAdd(a.cont_count_w, 1)] = (int)blk;
            } else if (a.stats != nullptr && st > st0) {
              atomicAdd(a.stats + 2, (unsigned long long)(-(long long)(st - st0)));
            }
          }
        }
        return;
      }
#if RM_PRIO_RAMP
      if (st == half) __builtin_amdgcn_s_setprio(2);
#endif
      const float p[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
      if (wave_escaped(st, p)) {
        dead = true;
        st_stop = st;
        break;
      }
#ifdef RM_RAY_STATS
      if (!SPLIT && st == RM_RAY_STATS_CAP) {
        const int lv = __popcll(__ballot(valid && !gone && ray_need >= st));
        if (lane == 0) atomicAdd(&rs_w[0], (unsigned)lv);
        rs_at = true;
      }
      rs_last = st;
#endif
      int choice;
      const float D = soft_min_march(p, all_safe(lb, rho_lb), Dprev, choice);
      const float t_step = t;  // this step's state: (t_step, choice)
#ifdef RM_RAY_STATS
      if (valid && !gone && !(t_step == cyc_t2 && choice == ((chist >> 3) & 7))) ray_need = st + 1;
#endif
      if constexpr (SPLIT) {
        // Ray mode: a ray's step is a function of its own t (the shift is scene-uniform; the clamp
        // choice changes no bit), so a ray whose t repeats with period 2 (t_step == t two steps
        // back, under the same shift choice) keeps repeating: it retires with the state the march
        // would end in -- this step's when an even number of steps is left, the next one's
        // otherwise -- and keeps it (its lanes still run, their results unused). Gone rays
        // (sticky) and retired rays leave the wave-uniform choices.
        const float rl0 = rho_lb;
        if (!retired) {
          t = fminf(t + (gone ? gone_step : D), kTMax);
          rho_lb = rho_moved(rl0, t_step, t);
          lb = D - fabsf(D);
          Dprev = D;
        }
        if (a.early_exit && MODE != kRender) {
          if (!retired && !gone && valid && t_step == cyc_t2 && (choice & 3) == ((rhist >> 3) & 3)) {
            retired = true;
            if (((a.steps - st) & 1) == 0) {  // the state after the last step is this step's
              t = t_step;
              rho_lb = rl0;
            }
          }
          if (!retired) {
            cyc_t2 = cyc_t1;
            cyc_t1 = t_step;
          }
          rhist = ((rhist << 3) | choice) & 0xFFF;
          if (__all(gone || !valid || retired)) {  // every ray final or gone: gone rays take their bound steps
            if (gone) {
              for (int k = st + 1; k < a.steps; ++k) {
                const float q[3] = {fmaf(d[0], t, o[0]) - c0x, fmaf(d[1], t, o[1]) - c0y, fmaf(d[2], t, o[2]) - c0z};
                t = fminf(t + (fsqrt(fmaf(q[2], q[2], fmaf(q[1], q[1], q[0] * q[0]))) - rprime), kTMax);
              }
            }
            steps_saved += a.steps - 1 - st;
            break;
          }
        }
        continue;
      }
      t = fminf(t + (gone ? gone_step : D), kTMax);
      rho_lb = rho_moved(rho_lb, t_step, t);
      // next point: hard min >= soft-min D here, moved by |D|
      lb = D - fabsf(D);
      Dprev = D;
      // Cycle exit (exact). A march step is a deterministic function of the wave's state: the t
      // of every ray that is not gone and the step's wave-uniform choice (which carries all the
      // previous step's D decides). When this step's state equals the state P steps back (P = 2,
      // or up to RM_CYCLE_MAX) the march repeats with period P from there, so the state after
      // the last step is the one (steps left) mod P steps after that earlier state. A ray cycling
      // between fixed points cannot become gone later (its thresholds only grow); gone rays take
      // their remaining bound steps here, as the march would. Of the last step's D the post-march
      // needs only the clamp-free choice of the reconnect: the final state's choice bit 2.
      if (a.early_exit && MODE != kRender) {
        int P = 0;
        if (choice == ((chist >> 3) & 7) && __all(gone || t_step == cyc_t2)) P = 2;
#if RM_CYCLE_MAX >= 3
        else if (choice == ((chist >> 6) & 7) && __all(gone || t_step == cyc_t3)) P = 3;
#endif
#if RM_CYCLE_MAX >= 4
        else if (choice == ((chist >> 9) & 7) && __all(gone || t_step == cyc_t4)) P = 4;
#endif
        if (P != 0) {
          // the state after the last step (step a.steps) is this step's state or the one `back`
          // steps before it; `left` steps remain after this one
          const int left = a.steps - 1 - st, m = a.steps - st, back = (P - m % P) % P;
          const int cf = back == 0 ? choice : (chist >> (3 * (back - 1))) & 7;
          if (!gone) {
            if (back == 0) t = t_step;
            else if (back == 1) t = cyc_t1;
#if RM_CYCLE_MAX >= 3
            else if (back == 2) t = cyc_t2;
#endif
#if RM_CYCLE_MAX >= 4
            else if (back == 3) t = cyc_t3;
#endif
            lb = (cf & 4) ? INFINITY : -INFINITY;  // all_safe(lb, rho_lb) of the final state = its bit 2
            rho_lb = -INFINITY;
          } else {
            for (int k = st + 1; k < a.steps; ++k) {
              const float q[3] = {fmaf(d[0], t, o[0]) - c0x, fmaf(d[1], t, o[1]) - c0y, fmaf(d[2], t, o[2]) - c0z};
              t = fminf(t + (fsqrt(fmaf(q[2], q[2], fmaf(q[1], q[1], q[0] * q[0]))) - rprime), kTMax);
            }
          }
          steps_saved += left;
#ifdef RM_BLOCK_TRACE
          tr_cyc = (unsigned long long)P | ((unsigned long long)st << 8);
#endif
          break;
        }
#if RM_CYCLE_MAX >= 4
        cyc_t4 = cyc_t3;
#endif
#if RM_CYCLE_MAX >= 3
        cyc_t3 = cyc_t2;
#endif
        cyc_t2 = cyc_t1;
        cyc_t1 = t_step;
        chist = ((chist << 3) | choice) & 0xFFF;
      }
    }
#ifdef RM_RAY_STATS
    if (!SPLIT && a.stats != nullptr) {  // stats[3]: the needed lane-steps, summed
      unsigned long long v = valid ? (unsigned long long)ray_need : 0ull;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0) atomicAdd(a.stats + 3, v);
      if (rs_at && lane == 0) {
        atomicAdd(&rs_w[1], (unsigned)(rs_last + 1 - RM_RAY_STATS_CAP));
        atomicMax(&rs_w[2], (unsigned)(rs_last + 1 - RM_RAY_STATS_CAP));
      }
    }
#endif
    if (SPLIT && a.ray_cont) {
      // ray mode: the listed rays' final states back into their groups' rows (the resume launch
      // runs the groups' post-march forward and backward); the steps this block ran uncounted
      // from the saved steps its groups booked at the cap
      float* cs = a.cont_state;
      const long long R = a.cont_rays;
      if (st_stop >= 0) gone_finish(st_stop);
      if (wave == 0 && lane < kSplitRays && valid) {
        cs[li] = t;
        cs[R + li] = lb;
        cs[5 * R + li] = gone ? 1.0f : (retired ? 2.0f : 0.0f);
        cs[6 * R + li] = rho_lb;
      }
      const long long run = (long long)(a.steps - st0) - steps_saved;
      if (wave == 0 && lane == 0 && a.stats != nullptr && run > 0) atomicAdd(a.stats + 2, (unsigned long long)(-run));
      return;
    }
  RM_TRACE(4, __builtin_amdgcn_s_memrealtime());
  RM_TRACE(6, (unsigned long long)steps_saved);
#ifdef RM_BLOCK_TRACE
  RM_TRACE(7, tr_paths);
  RM_TRACE(8, tr_lse_cyc);
  RM_TRACE(9, tr_vec);
  RM_TRACE(10, __builtin_readcyclecounter() - tr_c_begin);
  RM_TRACE(11, tr_cyc);
#endif
#ifdef RM_LANE_STATS  // stats[3] += escaped lane-steps of the march + 5 sweeps per escaped lane of a live wave
    if (a.stats != nullptr && lane == 0)
      atomicAdd(a.stats + 3, lane_gone_steps + (dead ? 0ull : 5ull * (unsigned long long)lanes_gone_last));
#endif
  }
#if RM_PRIO_RAMP
  __builtin_amdgcn_s_setprio(1);
#endif
  if ((MODE == kFwd || MODE == kRender) && a.t_out != nullptr && valid && own_rays) a.t_out[ri] = t;
  // work statistics: per wave here in the forward modes; per block at the hand-off barrier in the
  // backward modes (one pair of atomics per block, not per wave)
  if constexpr (MODE == kFwd || MODE == kRender) {
    if (a.stats != nullptr && lane == 0 && own_rays) {
      if (dead) atomicAdd(a.stats + 1, 1ull);
      if (steps_saved != 0) atomicAdd(a.stats + 2, (unsigned long long)steps_saved);
    }
  }

  // Post-march forward state. A wave whose rays have all escaped (see the march loop) keeps
  // the defaults: out = mix L mu = 0 with mu = 0, and every backward seed is 0.
  const float c10l = a.csharp * kLog2e;
  float pa[3] = {fmaf(d[0], t, o[0]), fmaf(d[1], t, o[1]), fmaf(d[2], t, o[2])};
  float p[3] = {pa[0], pa[1], pa[2]};
  float mA = 0.0f, sA = 1.0f, Da = 0.0f, tf = t;
  bool fast_a = false, fast_f = false;
  float nrm[3] = {0.0f, 0.0f, 0.0f}, D6[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  float amb = 0.0f, sdot = 0.0f, dif = 0.0f, Lgt = 0.0f;
  float dmin = 0.0f, Zw = 1.0f, Zb = 1.0f, Df = 0.0f, mix[3] = {0.0f, 0.0f, 0.0f}, mu = 0.0f;
  if (!dead) {
    // ---- reconnect: t_final = t + sdf(p_approx) (renderer_diff.rs:30-39); renderer.rs has none
    fast_a = all_safe(lb, rho_lb);
    if constexpr (MODE != kRender) {
      if constexpr (SPLIT) Da = soft_min_split(pa, fast_a, mA, sA);
      else Da = soft_min(pa, fast_a, mA, sA);
    }
    tf = t + Da;
    p[0] = fmaf(d[0], tf, o[0]);
    p[1] = fmaf(d[1], tf, o[1]);
    p[2] = fmaf(d[2], tf, o[2]);
    // p_final is |Da| from p_approx; the taps another eps away
    fast_f = MODE == kRender ? all_safe(lb - a.eps, rho_lb - a.eps)
                             : all_safe(-mA * inv_kappa - fabsf(Da) - a.eps, rho_moved(rho_lb, t, tf) - a.eps);

    // ---- detached normal (scene.rs:81-128): n = f / sqrt(|f|^2 + 1e-6) with f the central
    // differences (D(p + eps e_a) - D(p - eps e_a))_a; the 1e-6 keeps |n| ~ 0.2 at eps = 1e-4.
    // ---- colour softmax + mask (renderer_diff.rs:64-90)
    dmin = INFINITY;
    f2 Zw2 = sp(0.0f), Zb2 = sp(0.0f), C2[3] = {sp(0.0f), sp(0.0f), sp(0.0f)};
    if constexpr (MODE != kRender) {
      // one sweep for both: f = 2 eps grad D (its eps -> 0 limit) with grad D = G / Zb
      f2 G2[3] = {sp(0.0f), sp(0.0f), sp(0.0f)};
      if constexpr (SPLIT) {  // this wave's quarter of the pairs, then the four partial states merged
        const int b0 = split_pair(wave), b1 = split_pair(wave + 1);
        const Lds Lq = L.from_pair(b0);
        if (fast_f) shade_normal_sweep<false>(p, Lq, b1 - b0, c10l, kappa, dmin, Zw2, C2, Zb2, G2);
        else shade_normal_sweep<true>(p, Lq, b1 - b0, c10l, kappa, dmin, Zw2, C2, Zb2, G2);
        shade_merge(c10l, dmin, Zw2, C2, Zb2, G2);
      } else {
        if (fast_f) shade_normal_sweep<false>(p, L, a.Mpad / 2, c10l, kappa, dmin, Zw2, C2, Zb2, G2);
        else shade_normal_sweep<true>(p, L, a.Mpad / 2, c10l, kappa, dmin, Zw2, C2, Zb2, G2);
      }
      const float te = 2.0f * a.eps * frcp(Zb2.x + Zb2.y);
      const float nx = te * (G2[0].x + G2[0].y), ny = te * (G2[1].x + G2[1].y), nz = te * (G2[2].x + G2[2].y);
      const float inv_len = frsq(fmaf(nz, nz, fmaf(ny, ny, fmaf(nx, nx, 1e-6f))));
      nrm[0] = nx * inv_len;
      nrm[1] = ny * inv_len;
      nrm[2] = nz * inv_len;
    } else {  // renderer.rs: the six taps themselves, then the shade sums
      float m6[6], s6[6];
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        m6[q] = -INFINITY;
        s6[q] = 0.0f;
      }
      const float eps = a.eps;
      // weighted (unshifted) taps when the hard maximum at every tap is provably >= -90:
      // d_min(tap) <= d_min(p_a) + |Da| + eps <= 2 max(Da, 0) + ln(M)/k + eps (as in the march)
      const bool none = shift_none_ok && __all(2.0f * fmaxf(Da, 0.0f) + a.lse_slack + eps <= 90.0f * inv_kappa);
      if (none) {
        if (fast_f) lse_taps_w<false>(p, L, a.Mpad / 2, kappa, eps, s6);
        else lse_taps_w<true>(p, L, a.Mpad / 2, kappa, eps, s6);
#pragma unroll
        for (int q = 0; q < 6; ++q) m6[q] = 0.0f;
      } else if (fast_f) {
        for_tiles([&](int, int tn) { lse_taps<false>(p, L, tn / 2, nkappa, 2.0f * eps, eps * eps, m6, s6); });
      } else {
        for_tiles([&](int, int tn) { lse_taps<true>(p, L, tn / 2, nkappa, 2.0f * eps, eps * eps, m6, s6); });
      }
#pragma unroll
      for (int q = 0; q < 6; ++q) D6[q] = -(flog2(fmaxf(s6[q], 1e-30f)) + m6[q]) * inv_kappa;
      const float nx = D6[0] - D6[1], ny = D6[2] - D6[3], nz = D6[4] - D6[5];
      const float inv_len = frsq(fmaf(nz, nz, fmaf(ny, ny, fmaf(nx, nx, 1e-6f))));
      nrm[0] = nx * inv_len;
      nrm[1] = ny * inv_len;
      nrm[2] = nz * inv_len;
      if (fast_f)
        for_tiles([&](int, int tn) { shade_sweep<false>(p, L, tn / 2, c10l, kappa, dmin, Zw2, C2, Zb2); });
      else
        for_tiles([&](int, int tn) { shade_sweep<true>(p, L, tn / 2, c10l, kappa, dmin, Zw2, C2, Zb2); });
    }

    // ---- lighting (renderer_diff.rs:48-62; renderer.rs:27-40 in kRender)
    float ldn[3];
    if constexpr (MODE == kRender) {
      ldn[0] = a.light_fixed[0];
      ldn[1] = a.light_fixed[1];
      ldn[2] = a.light_fixed[2];
    } else {
      amb = a.ambient[0];
      light_unit(a.light_dir, ldn);
    }
    sdot = fmaf(nrm[2], ldn[2], fmaf(nrm[1], ldn[1], nrm[0] * ldn[0]));
    dif = fmaxf(sdot, 0.0f);
    Lgt = MODE == kRender ? dif + 0.1f : fmaf(dif, 1.0f - amb, amb);

    Zw = Zw2.x + Zw2.y;
    Zb = Zb2.x + Zb2.y;
    Df = dmin - flog2(fmaxf(Zb, 1e-8f)) * inv_kappa;
    if constexpr (MODE == kRender) {
      // renderer.rs:52-71: raw exp(-10 d) weights, mixed = sum(col w) / (sum(w) + 1e-5); the sums
      // above are shifted by exp(10 dmin), undone here; mask = exp(-10 D^2) (renderer.rs:77)
      const float e = fexp2(-c10l * dmin);
      const float den = Zw * e + 1e-5f;
      mix[0] = (C2[0].x + C2[0].y) * e / den;
      mix[1] = (C2[1].x + C2[1].y) * e / den;
      mix[2] = (C2[2].x + C2[2].y) * e / den;
      mu = fexp2(-10.0f * kLog2e * Df * Df);
    } else {
      const float invZw0 = frcp(Zw);
      mix[0] = (C2[0].x + C2[0].y) * invZw0;
      mix[1] = (C2[1].x + C2[1].y) * invZw0;
      mix[2] = (C2[2].x + C2[2].y) * invZw0;
      mu = frcp(1.0f + fexp2(a.msharp * kLog2e * Df));  // sigmoid(-msharp * D)
    }
  }
  const float invZw = frcp(Zw);
  const float scale = Lgt * mu;
  const float outv[3] = {mix[0] * scale, mix[1] * scale, mix[2] * scale};

  if (MODE == kFwd && a.dbg != nullptr && valid && own_rays) {
    float* q = a.dbg + 24 * ri;
    const float vals[24] = {t, tf, nrm[0], nrm[1], nrm[2], Lgt, mix[0], mix[1], mix[2], Df, mu, sdot, dmin,
                            Zw, Zb, 0.0f, D6[0], D6[1], D6[2], D6[3], D6[4], D6[5], 0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 24; ++c) q[c] = vals[c];
  }
  const bool write_out = MODE != kBwd && a.out != nullptr && valid && own_rays;
  if (write_out) {
    a.out[3 * ri] = outv[0];
    a.out[3 * ri + 1] = outv[1];
    a.out[3 * ri + 2] = outv[2];
  }
  RM_TRACE(5, __builtin_amdgcn_s_memrealtime());
  if constexpr (MODE == kFwd || MODE == kRender) return;
#if RM_PRIO_RAMP
  __builtin_amdgcn_s_setprio(0);
#endif

  // ---- seed g = dL/dout
  float g[3] = {0.0f, 0.0f, 0.0f};
  float loss = 0.0f;
  if (valid && seed_lane) {
    if constexpr (MODE == kBwd) {
      g[0] = a.gout[3 * ri];
      g[1] = a.gout[3 * ri + 1];
      g[2] = a.gout[3 * ri + 2];
    } else {  // training.rs:17-34
      const float t0 = a.targets[3 * ri], t1 = a.targets[3 * ri + 1], t2 = a.targets[3 * ri + 2];
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

  float* rec = a.partials + blk * a.rec;
  float* slots = L.slots;
  int chunk_ctr = 0;

  // ---- per-ray scalars (light before the projection, ambient, loss) and the early-exit
  // hand-off: every wave publishes its scalar sums and whether it left the march early; after
  // this barrier such waves end (an ended wave no longer counts in s_barrier) and the others
  // run the backward sweeps and combine only their own partials. The escaped waves' terms are
  // exactly 0, so the record is the one the full computation would write.
  static_assert(2 * kWaves <= 8, "misc layout: flags before the scalars");
  int* wflag = reinterpret_cast<int*>(L.misc);  // [kWaves] dead flags, [kWaves] steps saved
  float* wscal = L.misc + 8;                     // [kWaves][8]
  {
    const float vals[8] = {gell[0], gell[1], gell[2], gamb, loss, 0.0f, 0.0f, 0.0f};
    const float red = wave_reduce8(vals, lane);
    if ((lane & 7) == 7) wscal[wave * 8 + (lane >> 3)] = red;
    if (lane == 0) {
      wflag[wave] = dead ? 1 : 0;
      wflag[kWaves + wave] = steps_saved;
    }
  }
  // the block's hand-off work, by one wave once every wave has published: the cost in march-step
  // units (steps its waves ran, + kPostCost per wave that runs the post-march forward and the
  // backward: the next call's cost-ordered dispatch) and the work statistics
  auto handoff_work = [&]() {
    if (a.ocnt_w != nullptr) {
      int cost = 0;
#pragma unroll
      for (int w = 0; w < (SPLIT ? 1 : kWaves); ++w) cost += a.steps - wflag[kWaves + w] + (wflag[w] ? 0 : kPostCost);
      order_append(a, blk, cost);
    }
    if (a.stats != nullptr) {
      int ex = 0, sv = 0;
#pragma unroll
      for (int w = 0; w < (SPLIT ? 1 : kWaves); ++w) {
        ex += wflag[w];
        sv += wflag[kWaves + w];
      }
      if (ex != 0) atomicAdd(a.stats + 1, (unsigned long long)ex);
      if (sv != 0) atomicAdd(a.stats + 2, (unsigned long long)sv);
    }
  };
  // the whole block escaped: scalar totals, live flag 0 (the reduction skips the per-sphere
  // columns, all zero)
  auto escaped_record = [&]() {
    if (lane < 8) {
      float acc = wscal[lane];
#pragma unroll
      for (int w = 1; w < (SPLIT ? kSplitWaves : kWaves); ++w) acc += wscal[w * 8 + lane];
      rec[(long long)a.Mpad * 8 + lane] = acc;
    }
  };
#if RM_DEAD_EARLY
  if constexpr (!SPLIT) {
    if (dead) {
      // This wave's rays all escaped and its sums are published: it ends here rather than at the
      // barrier below (an ended wave no longer counts in s_barrier), so its slot is free while the
      // block's other waves march on. The count of such waves says which one was last; when every
      // wave of the block left early, that one does the block's hand-off work (the others'
      // publications precede their adds to the count: LDS operations of a wave run in order).
      int* dcnt = reinterpret_cast<int*>(L.misc) + kDeadCountSlot;
      int prev = 0;
      if (lane == 0) prev = __hip_atomic_fetch_add(dcnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
      prev = __shfl(prev, 0);
      if (prev != kWaves - 1) return;
      if (lane == 0) handoff_work();
      escaped_record();
      return;
    }
  }
#endif
  __syncthreads();
#ifdef RM_RAY_STATS
  if (!SPLIT && tid == 0 && a.stats != nullptr && rs_w[1] != 0u) {
    atomicAdd(a.stats + 6, 64ull * rs_w[1]);
    atomicAdd(a.stats + 7, 64ull * ((rs_w[0] + 63u) / 64u) * rs_w[2]);
  }
#endif
  int alive = 0;
#pragma unroll
  for (int w = 0; w < (SPLIT ? kSplitWaves : kWaves); ++w) alive |= wflag[w] ? 0 : (1 << w);
  alive = __builtin_amdgcn_readfirstlane(alive);  // block-uniform: scalar for the compiler
  // the hand-off work: the block's first live wave (wave 0 when every wave escaped)
  if (lane == 0 && wave == (alive != 0 ? __builtin_ctz(alive) : 0)) handoff_work();
  if (dead) {
    if (alive == 0 && wave == 0) escaped_record();
    return;
  }
  const int arank = __popc(alive & ((1 << wave) - 1));
  const int atid = arank * 64 + lane, astride = __popc(alive) * 64;
  // sum of the live waves' slots, in wave order (the order the all-alive case uses)
  auto live_sum = [&](const float* s0, int stride) {
    float acc = 0.0f;
    bool first = true;
#pragma unroll
    for (int w = 0; w < (SPLIT ? kSplitWaves : kWaves); ++w)
      if (alive & (1 << w)) {
        acc = first ? s0[w * stride] : acc + s0[w * stride];
        first = false;
      }
    return acc;
  };

#if RM_BWD_TRANSPOSED
  // ---- backward sweeps with one sphere per lane (transposed), the work shared out over the
  // block's live waves. Each live wave publishes its rays with non-zero seeds (a source) as a
  // compacted field-major LDS image. The work units are (64-sphere group, source wave) pairs in
  // group-major order; live wave r of n takes the units [r U / n, (r + 1) U / n) (U = groups x
  // sources). For each sphere of its lane a wave sums the terms of the rays of its units (sources
  // in wave order, their rays two per packed instruction) in registers, and writes the group's
  // record columns itself when it holds every source of the group; a group whose sources span
  // waves is added up from the waves' partials in LDS, in source order, by the wave that holds its
  // first unit. So each sphere group is loaded by one wave (two at a split), and there is no
  // combine of wave partials and no barrier per group. A split block's waves hold the same rays:
  // wave 0 is its one source (it seeds every lane) and the waves share the groups.
  // Only the position gradient g_p of sweep 1 is a per-ray sum over spheres, and only g_t = g_p . d
  // (the ray direction) is needed (t_final = t + D(p_a), p = o + d t_final): each computing wave
  // reduces its share across the lanes for batches of 8 rays (one transposing reduction) into an
  // LDS slot per (computing wave, source wave, ray), and the ray's owner adds the computing waves'
  // shares in wave order. Rays whose seeds are zero contribute exact zeros and are not listed
  // (sweep 1: gm = 0 and b_scale = 0; sweep 2: g_t = 0) -- in practice the escaped rays of live
  // waves; an odd count is padded with a copy of the last ray whose seeds are zero (exact zero
  // terms). Distances are formed with the same fp32 operations and operands as the forward sweeps
  // (qpair, delta_pair_rsq), so dd = dmin - delta <= 0 and v - mA <= 0 hold exactly.
  bool any_seed = true;  // block-uniform: some ray of the block has a non-zero seed
  {
    (void)slots;
    (void)live_sum;
    (void)chunk_ctr;
    (void)atid;
    (void)astride;
    constexpr int kFields = kBwdFields;  // sweep 1: px py pz |p|^2 dmin 1/Zw b_scale mg gm.xyz d.xyz (14); sweep 2: 6
    constexpr int kWv = SPLIT ? kSplitWaves : kWaves;
    float* rayf_all = L.slots;                     // [wave][field][64 ray slots]; after a sweep: partials
    float* rayf = rayf_all + wave * 64 * kFields;  // this wave's rays
    float* gta = L.slots + kWaves * 64 * kFields;  // [computing wave][source wave][64] g_t shares
    int* nsrc = reinterpret_cast<int*>(L.misc) + 40;  // [kWaves] the sources' ray counts (sweep 1, then 2)
    const int np = a.Mpad / 2;
    const float4* R4 = reinterpret_cast<const float4*>(a.rec_buf);
    const float2* R2 = reinterpret_cast<const float2*>(R4 + 7 * (size_t)np);
    const int ngrp = (a.Mpad + 63) / 64;
    // The computing waves of a sweep: the block's source waves -- a set that does not depend on
    // which rayless waves left the march early, so the partition and every sum order are the same
    // with the early exit on and off -- or, in a split block, its waves (alive together).
    // the packed pair (slots s, s + 1) of field f of source wave sw's image
    auto pair = [&](int sw, int f, int s) {
      return *reinterpret_cast<const f2*>(rayf_all + (sw * kFields + f) * 64 + s);
    };
    const unsigned long long below = (1ull << lane) - 1ull;
    // this wave's units of a sweep with nsw sources: [u0, u1)
    auto unit_range = [&](int r, int nsw, int ncw, int& u0, int& u1) {
      const int U = ngrp * nsw;
      u0 = (r * U) / ncw;
      u1 = ((r + 1) * U) / ncw;
    };
    // the block's source waves (bits) from the published counts
    auto sources = [&]() {
      int m = 0;
#pragma unroll
      for (int sw = 0; sw < kWv; ++sw)
        if ((alive >> sw) & 1) m |= nsrc[sw] > 0 ? (1 << sw) : 0;
      return __builtin_amdgcn_readfirstlane(m);
    };
    // Partials of the groups a wave holds only in part: slot 0 its first group, slot 1 its last,
    // kept in registers through the sweep and written over the wave's own ray image after it
    // (ncomp floats x 64 per slot). The wave that holds a split group's first unit adds the
    // partials of the waves that hold its units, in order, and writes (ncomp 8) or adds to (4)
    // the record columns.
    // Does a wave boundary fall inside a group (a multiple of nsw units is a group boundary)?
    auto has_split = [&](int nsw, int ncw) {
      const int U = ngrp * nsw;
      for (int r = 1; r < ncw; ++r)
        if (((r * U) / ncw) % nsw != 0) return true;
      return false;
    };
    // (always inlined: as a call its array arguments went to scratch memory)
    auto finish_split = [&](int nsw, int ncw, int crank, bool in, int ncomp, const float (&p0)[8],
                            const float (&p1)[8]) __attribute__((always_inline)) {
      __syncthreads();  // every wave is done with the sweep's images
      // the partials indexed by live rank: slot 0 in rows [0, nst), slot 1 in [nst, 2 nst) (a
      // sweep-1 partial's column 7 is 0 and not stored: 14 rows fit a wave's 15-row image)
      const int nst = ncomp == 8 ? 7 : 4;
      float* mine = rayf_all + crank * 64 * kFields;  // by computing rank
      if (in) {
#pragma unroll
        for (int c = 0; c < 7; ++c)
          if (c < nst) {
            mine[c * 64 + lane] = p0[c];
            mine[(nst + c) * 64 + lane] = p1[c];
          }
      }
      __syncthreads();
      if (!in) return;
      int u0, u1;
      unit_range(crank, nsw, ncw, u0, u1);
      if (u1 <= u0) return;
      const int gl = (u1 - 1) / nsw;  // this wave's last group
      const int kb = max(u0, gl * nsw) - gl * nsw;
      if (kb != 0 || u1 - gl * nsw >= nsw) return;  // not the first unit of a split group
      // this wave holds units [0, u1 - gl nsw) of group gl: its last group, or its only one
      float acc[8];
      const int own_slot = (u0 / nsw == gl) ? 0 : 1;
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = c < nst ? mine[(nst * own_slot + c) * 64 + lane] : 0.0f;
      for (int rr = crank + 1; rr < ncw; ++rr) {  // the next waves hold the group's next units
        int v0, v1;
        unit_range(rr, nsw, ncw, v0, v1);
        if (v0 >= (gl + 1) * nsw) break;
        if (v1 <= v0) continue;
        const float* part = rayf_all + rr * 64 * kFields;  // its first group: slot 0
#pragma unroll
        for (int c = 0; c < 7; ++c)
          if (c < nst) acc[c] += part[c * 64 + lane];
      }
      const int j = gl * 64 + lane;
      if (ncomp == 8) {
        store_group_cols(rec + (long long)gl * 64 * 8, acc, lane, min(64, a.Mpad - gl * 64));
      } else if (j < a.Mpad) {
        float4* dst = reinterpret_cast<float4*>(rec + (long long)j * 8);
        {
          float4 v = dst[0];
          v.x += acc[0];
          v.y += acc[1];
          v.z += acc[2];
          v.w += acc[3];
          dst[0] = v;
        }
      }
    };

    // ---- sweep 1 at p_final: colour softmax + mask soft-min + p_final(t_final)
    const unsigned long long act1 = __ballot(gm[0] != 0.0f || gm[1] != 0.0f || gm[2] != 0.0f || b_scale != 0.0f);
    const int n1 = __popcll(act1), rank1 = __popcll(act1 & below);
    const bool on1 = ((act1 >> lane) & 1ull) != 0ull;
    if (on1) {
      const float vals[14] = {p[0], p[1], p[2], psq(p), dmin, invZw, b_scale, mg, gm[0], gm[1], gm[2],
                              d[0], d[1], d[2]};
#pragma unroll
      for (int f = 0; f < 14; ++f) rayf[f * 64 + rank1] = vals[f];
      if ((n1 & 1) && rank1 == n1 - 1) {  // pad: this ray again, zero seeds
        const float pad[14] = {p[0], p[1], p[2], psq(p), dmin, invZw, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f,
                               d[0], d[1], d[2]};
#pragma unroll
        for (int f = 0; f < 14; ++f) rayf[f * 64 + n1] = pad[f];
      }
    }
    if (lane == 0) nsrc[wave] = n1;
    // work statistics: the rays the backward sweeps run for (a split block's rays are wave 0's)
    if (a.stats != nullptr && lane == 0 && n1 > 0 && (!SPLIT || wave == 0))
      atomicAdd(a.stats + 4, (unsigned long long)n1);
#pragma unroll
    for (int sw = 0; sw < kWv; ++sw) gta[(wave * kWaves + sw) * 64 + lane] = 0.0f;
    __syncthreads();  // every live wave's image and count
    const int srcs1 = sources();
    const int nsw1 = __popc(srcs1);
    const int cmask1 = SPLIT ? alive : srcs1, ncw1 = __popc(cmask1), crank1 = __popc(cmask1 & ((1 << wave) - 1));
    const bool in1 = ((cmask1 >> wave) & 1) != 0;
    bool split1 = false;
    {
      const f2 CL = sp(c10l), KA = sp(kappa), NCS = sp(-a.csharp);
      float p0[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, p1[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      auto sweep1 = [&](auto clamp_tag) {
        constexpr bool CLAMP = decltype(clamp_tag)::value;
        int u0 = 0, u1 = 0;
        if (in1) unit_range(crank1, nsw1, ncw1, u0, u1);
        for (int u = u0; u < u1;) {
          const int grp = u / nsw1, kb = u - grp * nsw1, ke = min(u1 - grp * nsw1, nsw1);
          u = grp * nsw1 + ke;
          const int j = grp * 64 + lane;
          float gx = -2.0f * kPadCenter, gy = 0.0f, gz = 0.0f, cc = kPadCenter * kPadCenter, rr = 0.0f, cr = 0.0f,
                cg = 0.0f, cbl = 0.0f;
          if (j < a.Mpad) {  // sphere j of pair j/2 (records of rm_prep_kernel)
            const int i = j >> 1;
            const bool h = (j & 1) != 0;
            const float4 A = R4[i], B = R4[np + i], R = R4[2 * np + i], C3 = R4[3 * np + i];
            const float2 C4 = R2[i];
            gx = h ? A.y : A.x;
            gy = h ? A.w : A.z;
            gz = h ? B.y : B.x;
            cc = h ? B.w : B.z;
            rr = h ? R.w : R.z;
            cr = h ? C3.y : C3.x;
            cg = h ? C3.w : C3.z;
            cbl = h ? C4.y : C4.x;
          }
          const f2 GX = sp(gx), GY = sp(gy), GZ = sp(gz), CC = sp(cc), RR = sp(rr), CR = sp(cr), CG = sp(cg),
                   CB = sp(cbl), HX = sp(0.5f * gx), HY = sp(0.5f * gy), HZ = sp(0.5f * gz);
          f2 agc[3] = {sp(0.0f), sp(0.0f), sp(0.0f)}, agr = sp(0.0f), acol[3] = {sp(0.0f), sp(0.0f), sp(0.0f)};
          for (int sw = 0, k = 0; sw < kWv; ++sw) {
            if (!((srcs1 >> sw) & 1)) continue;
            const int kk = k++;
            if (kk < kb || kk >= ke) continue;
            const int ns = nsrc[sw], nps = (ns + 1) >> 1;
            float* gacc = gta + (wave * kWaves + sw) * 64;
            for (int b = 0; b < nps; b += 4) {  // batches of 4 pairs = 8 slots
              float gtv[8];
#pragma unroll
              for (int uu = 0; uu < 4; ++uu) {
                if (b + uu >= nps) {  // batch slots past the last pair
                  gtv[2 * uu] = gtv[2 * uu + 1] = 0.0f;
                  continue;
                }
                const int s0 = 2 * (b + uu);
                const f2 PX = pair(sw, 0, s0), PY = pair(sw, 1, s0), PZ = pair(sw, 2, s0);
#if RM_BWD_PSQ_REG
                const f2 PP = fma2(PZ, PZ, fma2(PY, PY, PX * PX));  // == psq(p), lane by lane
#else
                const f2 PP = pair(sw, 3, s0);
#endif
                const f2 DM = pair(sw, 4, s0), IZ = pair(sw, 5, s0), BS = pair(sw, 6, s0), MG = pair(sw, 7, s0);
                const f2 G0 = pair(sw, 8, s0), G1 = pair(sw, 9, s0), G2 = pair(sw, 10, s0);
                const f2 DX = pair(sw, 11, s0), DY = pair(sw, 12, s0), DZ = pair(sw, 13, s0);
                f2 q = fma2(PZ, GZ, fma2(PY, GY, fma2(PX, GX, PP + CC)));  // == qpair: the shade sweep's q
                const f2 qraw = q;
                if constexpr (CLAMP) q = clamp_q(q);
                const f2 ir = rsq2(q);  // == delta_pair_rsq: the shade sweep's delta, and 1/rho
                const f2 dl = q * ir - RR;
                const f2 dd = DM - dl;  // <= 0 exactly
                const f2 w = exp2v(dd * CL) * IZ;
                const f2 bt = exp2v(dd * KA) * BS;
                const f2 cgm = fma2(CB, G2, fma2(CG, G1, CR * G0));
                const f2 gd = fma2(w * NCS, cgm - MG, bt);
                f2 gu = gd * ir;
                if constexpr (CLAMP) {  // clamp_min(1e-6) gate
                  gu.x = qraw.x >= 1e-6f ? gu.x : 0.0f;
                  gu.y = qraw.y >= 1e-6f ? gu.y : 0.0f;
                }
                const f2 ex = HX + PX, ey = HY + PY, ez = HZ + PZ;  // == fma2(HALF, -2c, p) = p - c
                const f2 ngu = -gu;
                agc[0] = fma2(ngu, ex, agc[0]);  // gc_j -= g_delta_j u_j
                agc[1] = fma2(ngu, ey, agc[1]);
                agc[2] = fma2(ngu, ez, agc[2]);
                const f2 gt2 = gu * fma2(ez, DZ, fma2(ey, DY, ex * DX));  // (g_delta_j u_j) . d
                gtv[2 * uu] = gt2.x;
                gtv[2 * uu + 1] = gt2.y;
                agr -= gd;
                acol[0] = fma2(w, G0, acol[0]);
                acol[1] = fma2(w, G1, acol[1]);
                acol[2] = fma2(w, G2, acol[2]);
              }
              const float r0 = wave_reduce8(gtv, lane);
              const int slot = 2 * b + (lane >> 3);
              if ((lane & 7) == 7 && slot < ns) gacc[slot] += r0;
            }
          }
          const float v[8] = {agc[0].x + agc[0].y, agc[1].x + agc[1].y, agc[2].x + agc[2].y, agr.x + agr.y,
                              acol[0].x + acol[0].y, acol[1].x + acol[1].y, acol[2].x + acol[2].y, 0.0f};
          if (kb == 0 && ke == nsw1) {  // every source: the group's columns, written by this wave alone
            store_group_cols(rec + (long long)grp * 64 * 8, v, lane, min(64, a.Mpad - grp * 64));
          } else if (grp == u0 / nsw1) {
#pragma unroll
            for (int c = 0; c < 8; ++c) p0[c] = v[c];
          } else {
#pragma unroll
            for (int c = 0; c < 8; ++c) p1[c] = v[c];
          }
        }
      };
      if (nsw1 == 0) {  // no ray of the block has a seed: its columns are zeros, not written (live flag 0)
        any_seed = false;
      } else if (fast_f) {
        sweep1(std::false_type{});
      } else {
        sweep1(std::true_type{});
      }
      split1 = nsw1 > 0 && has_split(nsw1, ncw1);
      if (split1) finish_split(nsw1, ncw1, crank1, in1, 8, p0, p1);
      else __syncthreads();  // every computing wave's g_t shares
    }

    // ---- sweep 2 at p_approx: t_final = t + D(p_approx) -> g_t * softmax(-k dist_a)
    float gt = 0.0f;
    if (on1) {
      bool first = true;
#pragma unroll
      for (int w = 0; w < kWv; ++w)
        if ((cmask1 >> w) & 1) {
          const float v = gta[(w * kWaves + wave) * 64 + rank1];
          gt = first ? v : gt + v;
          first = false;
        }
    }
    const float hs = gt * frcp(sA);
    if (split1) __syncthreads();  // every split partial read (the images hold them)
    const unsigned long long act2 = __ballot(hs != 0.0f);
    const int n2 = __popcll(act2), rank2 = __popcll(act2 & below);
    if (((act2 >> lane) & 1ull) != 0ull) {
      const float vals[6] = {pa[0], pa[1], pa[2], psq(pa), mA, hs};
#pragma unroll
      for (int f = 0; f < 6; ++f) rayf[f * 64 + rank2] = vals[f];
      if ((n2 & 1) && rank2 == n2 - 1) {  // pad: this ray again, zero seed
        const float pad[6] = {pa[0], pa[1], pa[2], psq(pa), mA, 0.0f};
#pragma unroll
        for (int f = 0; f < 6; ++f) rayf[f * 64 + n2] = pad[f];
      }
    }
    if (lane == 0) nsrc[wave] = n2;
    if (a.stats != nullptr && lane == 0 && n2 > 0 && (!SPLIT || wave == 0))
      atomicAdd(a.stats + 5, (unsigned long long)n2);
    __syncthreads();  // every live wave's sweep-2 image and count
    const int srcs2 = sources();
    const int nsw2 = __popc(srcs2);
    const int cmask2 = SPLIT ? alive : srcs2, ncw2 = __popc(cmask2), crank2 = __popc(cmask2 & ((1 << wave) - 1));
    const bool in2 = ((cmask2 >> wave) & 1) != 0;
    if (nsw2 > 0) {
      const f2 NK = sp(nkappa);
      float p0[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f}, p1[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      auto sweep2 = [&](auto clamp_tag) {
        constexpr bool CLAMP = decltype(clamp_tag)::value;
        int u0 = 0, u1 = 0;
        if (in2) unit_range(crank2, nsw2, ncw2, u0, u1);
        for (int u = u0; u < u1;) {
          const int grp = u / nsw2, kb = u - grp * nsw2, ke = min(u1 - grp * nsw2, nsw2);
          u = grp * nsw2 + ke;
          const int j = grp * 64 + lane;
          float gx = -2.0f * kPadCenter, gy = 0.0f, gz = 0.0f, cc = kPadCenter * kPadCenter, kr = 0.0f;
          if (j < a.Mpad) {
            const int i = j >> 1;
            const bool h = (j & 1) != 0;
            const float4 A = R4[i], B = R4[np + i], R = R4[2 * np + i];
            gx = h ? A.y : A.x;
            gy = h ? A.w : A.z;
            gz = h ? B.y : B.x;
            cc = h ? B.w : B.z;
            kr = h ? R.y : R.x;
          }
          const f2 GX = sp(gx), GY = sp(gy), GZ = sp(gz), CC = sp(cc), KR = sp(kr), HX = sp(0.5f * gx),
                   HY = sp(0.5f * gy), HZ = sp(0.5f * gz);
          f2 agc[3] = {sp(0.0f), sp(0.0f), sp(0.0f)}, agr = sp(0.0f);
          for (int sw = 0, k = 0; sw < kWv; ++sw) {
            if (!((srcs2 >> sw) & 1)) continue;
            const int kk = k++;
            if (kk < kb || kk >= ke) continue;
            const int nps = (nsrc[sw] + 1) >> 1;
            for (int i2 = 0; i2 < nps; ++i2) {
              const int s0 = 2 * i2;
              const f2 PX = pair(sw, 0, s0), PY = pair(sw, 1, s0), PZ = pair(sw, 2, s0);
#if RM_BWD_PSQ_REG
              const f2 PP = fma2(PZ, PZ, fma2(PY, PY, PX * PX));  // == psq(pa), lane by lane
#else
              const f2 PP = pair(sw, 3, s0);
#endif
              const f2 MA = pair(sw, 4, s0), HS = pair(sw, 5, s0);
              f2 q = fma2(PZ, GZ, fma2(PY, GY, fma2(PX, GX, PP + CC)));  // == qpair: the reconnect sweep's q
              const f2 qraw = q;
              if constexpr (CLAMP) q = clamp_q(q);
              const f2 r = rsq2(q);  // rho = q rsq(q) as in lse_point, 1/rho = rsq(q)
              const f2 h = exp2v(fma2(q * r, NK, KR) - MA) * HS;  // v - mA <= 0 exactly
              f2 hu = h * r;
              if constexpr (CLAMP) {
                hu.x = qraw.x >= 1e-6f ? hu.x : 0.0f;
                hu.y = qraw.y >= 1e-6f ? hu.y : 0.0f;
              }
              agc[0] = fma2(-hu, HX + PX, agc[0]);
              agc[1] = fma2(-hu, HY + PY, agc[1]);
              agc[2] = fma2(-hu, HZ + PZ, agc[2]);
              agr -= h;
            }
          }
          const float v[8] = {agc[0].x + agc[0].y, agc[1].x + agc[1].y, agc[2].x + agc[2].y, agr.x + agr.y,
                              0.0f, 0.0f, 0.0f, 0.0f};
          if (kb == 0 && ke == nsw2) {  // added to the group's sweep-1 columns 0-3
            if (j < a.Mpad) {
              float4* dst = reinterpret_cast<float4*>(rec + (long long)j * 8);
              float4 o = dst[0];
              o.x += v[0];
              o.y += v[1];
              o.z += v[2];
              o.w += v[3];
              dst[0] = o;
            }
          } else if (grp == u0 / nsw2) {
#pragma unroll
            for (int c = 0; c < 8; ++c) p0[c] = v[c];
          } else {
#pragma unroll
            for (int c = 0; c < 8; ++c) p1[c] = v[c];
          }
        }
      };
      if (fast_a) sweep2(std::false_type{});
      else sweep2(std::true_type{});
      if (has_split(nsw2, ncw2)) finish_split(nsw2, ncw2, crank2, in2, 4, p0, p1);
    }
  }
  __syncthreads();
#else
  // ---- backward sweep 1 at p_final: colour softmax + mask soft-min + p_final(t_final)
  f2 GP[3] = {sp(0.0f), sp(0.0f), sp(0.0f)};
  {
    const f2 PX = sp(p[0]), PY = sp(p[1]), PZ = sp(p[2]), PP = sp(psq(p)), CL = sp(c10l), KA = sp(kappa),
             DM = sp(dmin), IZ = sp(invZw), BS = sp(b_scale), G0 = sp(gm[0]), G1 = sp(gm[1]), G2 = sp(gm[2]),
             MG = sp(mg), NCS = sp(-a.csharp), HALF = sp(0.5f);
    auto sweep1 = [&](auto clamp_tag, int t0, int tn) {
      constexpr bool CLAMP = decltype(clamp_tag)::value;
      for (int jc = 0; jc < tn; jc += kChunkBwd, ++chunk_ctr) {
        float* sb = slots + (chunk_ctr & 1) * (kWaves * kChunkBwd * 8);
        for (int jj = 0; jj < kChunkBwd; jj += 4) {  // 4 spheres (2 pairs) per masked LDS write
          float red[4];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int i = (jc + jj) / 2 + u;
            const float4 A = L.p0(i), B = L.p1(i), R = L.p2(i), C3 = L.p3(i);
            const float2 C4 = L.p4(i);
            f2 q, ir;
            const f2 dl = delta_pair_rsq<CLAMP>(PX, PY, PZ, PP, A, B, R, q, ir);  // bitwise the shade sweep's
            const f2 dd = DM - dl;  // <= 0 exactly
            const f2 w = exp2v(dd * CL) * IZ;
            const f2 bt = exp2v(dd * KA) * BS;
            const f2 cg = fma2(f2{C4.x, C4.y}, G2, fma2(hi(C3), G1, lo(C3) * G0));
            const f2 gd = fma2(w * NCS, cg - MG, bt);
            f2 gu = gd * ir;
            if constexpr (CLAMP) {  // clamp_min(1e-6) gate
              gu.x = q.x >= 1e-6f ? gu.x : 0.0f;
              gu.y = q.y >= 1e-6f ? gu.y : 0.0f;
            }
            const f2 ex = fma2(HALF, lo(A), PX), ey = fma2(HALF, hi(A), PY), ez = fma2(HALF, lo(B), PZ);
            GP[0] = fma2(gu, ex, GP[0]);
            GP[1] = fma2(gu, ey, GP[1]);
            GP[2] = fma2(gu, ez, GP[2]);
            const f2 ngu = -gu;
            const f2 v0 = ngu * ex, v1 = ngu * ey, v2 = ngu * ez, v4 = w * G0, v5 = w * G1, v6 = w * G2;
            const float va[8] = {v0.x, v1.x, v2.x, -gd.x, v4.x, v5.x, v6.x, 0.0f};
            const float vb[8] = {v0.y, v1.y, v2.y, -gd.y, v4.y, v5.y, v6.y, 0.0f};
            red[2 * u] = wave_reduce8(va, lane);
            red[2 * u + 1] = wave_reduce8(vb, lane);
          }
          if ((lane & 7) == 7) {
            float* dst = sb + (wave * kChunkBwd + jj) * 8 + (lane >> 3);
#pragma unroll
            for (int k2 = 0; k2 < 4; ++k2) dst[8 * k2] = red[k2];
          }
        }
        __syncthreads();
        for (int e = atid; e < kChunkBwd * 8; e += astride) rec[(long long)(t0 + jc) * 8 + e] = live_sum(sb + e, kChunkBwd * 8);
      }
    };
    if (fast_f)
      for_tiles([&](int t0, int tn) { sweep1(std::false_type{}, t0, tn); });
    else
      for_tiles([&](int t0, int tn) { sweep1(std::true_type{}, t0, tn); });
  }
  __syncthreads();

  // ---- backward sweep 2 at p_approx: t_final = t + D(p_approx) -> g_t * softmax(-k dist_a)
  const float gp[3] = {GP[0].x + GP[0].y, GP[1].x + GP[1].y, GP[2].x + GP[2].y};
  const float gt = fmaf(gp[2], d[2], fmaf(gp[1], d[1], gp[0] * d[0]));
  {
    const f2 PX = sp(pa[0]), PY = sp(pa[1]), PZ = sp(pa[2]), PP = sp(psq(pa)), NK = sp(nkappa), MA = sp(mA),
             HS = sp(gt * frcp(sA)), HALF = sp(0.5f);
    auto sweep2 = [&](auto clamp_tag, int t0, int tn) {
      constexpr bool CLAMP = decltype(clamp_tag)::value;
      for (int jc = 0; jc < tn; jc += kChunkBwd, ++chunk_ctr) {
        float* sb = slots + (chunk_ctr & 1) * (kWaves * kChunkBwd * 8);
        for (int jj = 0; jj < kChunkBwd; jj += 4) {  // 2 pairs per masked LDS write
          float red[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int i = (jc + jj) / 2 + u;
            const float4 A = L.p0(i), B = L.p1(i);
            const float2 K = L.kr(i);
            f2 q = qpair(PX, PY, PZ, PP, A, B);  // bitwise the reconnect sweep's q
            const f2 qraw = q;
            if constexpr (CLAMP) q = clamp_q(q);
            const f2 r = rsq2(q);  // rho = q rsq(q) as in lse_point, 1/rho = rsq(q)
            const f2 h = exp2v(fma2(q * r, NK, f2{K.x, K.y}) - MA) * HS;  // v - mA <= 0 exactly
            f2 hu = h * r;
            if constexpr (CLAMP) {
              hu.x = qraw.x >= 1e-6f ? hu.x : 0.0f;
              hu.y = qraw.y >= 1e-6f ? hu.y : 0.0f;
            }
            const f2 nhu = -hu;
            const f2 v0 = nhu * fma2(HALF, lo(A), PX), v1 = nhu * fma2(HALF, hi(A), PY),
                     v2 = nhu * fma2(HALF, lo(B), PZ);
            const float vals[8] = {v0.x, v1.x, v2.x, -h.x, v0.y, v1.y, v2.y, -h.y};
            red[u] = wave_reduce8(vals, lane);
          }
          if ((lane & 7) == 7) {
            float* dst = sb + (wave * kChunkBwd + jj) * 4 + (lane >> 3);
            dst[0] = red[0];
            dst[8] = red[1];
          }
        }
        __syncthreads();
        for (int e = atid; e < kChunkBwd * 4; e += astride) {  // added to sweep 1's columns 0-3
          float* dst = rec + (long long)(t0 + jc + (e >> 2)) * 8 + (e & 3);
          *dst += live_sum(sb + e, kChunkBwd * 4);
        }
      }
    };
    if (fast_a)
      for_tiles([&](int t0, int tn) { sweep2(std::false_type{}, t0, tn); });
    else
      for_tiles([&](int t0, int tn) { sweep2(std::true_type{}, t0, tn); });
  }
  __syncthreads();

#endif  // RM_BWD_TRANSPOSED

  // ---- per-ray scalar totals of the block (published before the sweeps)
  if (arank == 0 && lane < 8) {
    float acc = wscal[lane];
#pragma unroll
    for (int w = 1; w < (SPLIT ? kSplitWaves : kWaves); ++w) acc += wscal[w * 8 + lane];
#if RM_BWD_TRANSPOSED
    const float live = any_seed ? 1.0f : 0.0f;
#else
    const float live = 1.0f;
#endif
    rec[(long long)a.Mpad * 8 + lane] = lane == 7 ? live : acc;  // scalar 7: live flag
  }
}

// ---- cross-block reduction (fixed order => deterministic) --------------------------------
// Partial record of one ray block (rec = Mpad*8 + 8 floats):
//   [Mpad][8] (gc.xyz, gr, gcol.rgb, 0) -- backward sweep 1's terms, sweep 2's (gc, gr) terms added
//   by the block itself -- | 8 scalars
// Scalar 7 is the block's live flag: 0 when every wave of the block left the march early or no ray
// of it has a non-zero backward seed (its per-sphere columns are all zero and were not written),
// 1 otherwise.
// Output columns (ncols = Mpad*8 + 8): [Mpad][8] combined per-sphere grads | 8 scalars.
//
// Pass 1, grid (column blocks x segments of ray blocks): each block sums its segment for its 256
// columns into S[seg][col] -- one addition chain per column in ray-block order, loads batched
// eight rows at a time. Rows of dead
// blocks are skipped: they only hold zeros, and adding +0 leaves a chain unchanged, so the sums
// are those of the full chain.
struct FinalArgs {
  const float* light_dir;
  float *gc, *gcol, *gr, *gld, *gamb, *loss_sum;
  int accumulate;
  int* oturn;  // nullable: the cost-order turn word the reduction advances (KArgs::oturn)
  // rm_train_step_camera_adam on a model of M <= kOptSmallMaxM spheres: the optimizer step on the
  // packed gradient (grad = gc: the packed layout) runs in the reduction's last block
  // (fused_optimizer); raw == nullptr otherwise
  float *raw, *m1, *m2, *act_out, *loss_penalty;
  _Float16* col_h;
  rm_step_scalars* sdev;
  unsigned* opt_arrival;  // the column blocks' arrival counter (zero between launches)
  int step, with_pen;
  float lr, wd;
};
__device__ void fused_optimizer(const FinalArgs& f, int M);

#ifndef RM_REDUCE_BATCH
#define RM_REDUCE_BATCH 8
#endif
constexpr int kReduceBatch = RM_REDUCE_BATCH;  // partial rows in flight per thread
#ifndef RM_FIN_U
#define RM_FIN_U 16  // finalize_block: 4 * RM_FIN_U loads in flight (32 with batch 16: no gain at C2)
#endif
static_assert((kReduceSegs / 4) % RM_FIN_U == 0, "finalize_block rounds");

__device__ void finalize_block(const float* S, int nseg, int M, int Mpad, const FinalArgs& f, float* tot);

// Segments of the reduction of nblocks ray blocks: kReduceSegs, or as many multiples of 64 as a
// launch of more than kReduceSegs * 256 blocks needs (a segment's rows fit pass 1's 256-entry list)
__host__ __device__ inline int reduce_segs(long long nblocks) {
  const long long need = (nblocks + 255) / 256;
  return need <= kReduceSegs ? kReduceSegs : (int)((need + 63) / 64 * 64);
}

__global__ __launch_bounds__(256) void rm_reduce_partials(const float* __restrict__ P, long long rec, int M, int Mpad,
                                                          int nblocks, int seg_len, float* __restrict__ S,
                                                          const FinalArgs f, unsigned* __restrict__ arrivals) {
  __shared__ int rows[256];
  __shared__ int wcount[4];
  __shared__ float tot[256];
  __shared__ int last;
  const int ncols = Mpad * 8 + 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the launch whose partials these are has finished: the cost-ordered dispatch turns one set on
  if (f.oturn != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *f.oturn = (*f.oturn + 1) % 3;
  const int col = blockIdx.x * 256 + tid;
  const bool scalars = (int)blockIdx.x * 256 >= Mpad * 8;  // the column block of the 8 scalars
  const int b0 = blockIdx.y * seg_len;
  const int b1 = min(b0 + seg_len, nblocks);
  // rows of this segment to visit, in order: every row for the scalars, live rows otherwise
  {
    const int b = b0 + tid;
    const bool take = b < b1 && (scalars || P[(long long)b * rec + (long long)Mpad * 8 + 7] != 0.0f);
    const unsigned long long m = __ballot(take);
    if (lane == 0) wcount[wave] = __popcll(m);
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wave; ++w) base += wcount[w];
    if (take) rows[base + __popcll(m & ((1ull << lane) - 1))] = b;
    __syncthreads();
  }
  const int nrows = wcount[0] + wcount[1] + wcount[2] + wcount[3];
  if (col < ncols) {
    float acc = 0.0f;  // columns map 1:1 onto the record (per-sphere block, then the scalars)
    for (int i0 = 0; i0 < nrows; i0 += kReduceBatch) {
      float v1[kReduceBatch];
#pragma unroll
      for (int u = 0; u < kReduceBatch; ++u) v1[u] = P[(long long)rows[min(i0 + u, nrows - 1)] * rec + col];
#pragma unroll
      for (int u = 0; u < kReduceBatch; ++u)
        if (i0 + u < nrows) acc += v1[u];
    }
    if (arrivals == nullptr) S[(long long)blockIdx.y * ncols + col] = acc;
    else __hip_atomic_store(S + (long long)blockIdx.y * ncols + col, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (arrivals == nullptr) return;
  // Pass 2 in the same launch: the segment block that arrives last for this column block sums
  // the segments and scatters them (finalize_block, the bits of rm_finalize_grads). Hand-off
  // (MI355X_MICROARCH.md, inter-workgroup visibility): write-through segment stores drained by
  // every wave before the block barrier, one lane's agent-scope arrival, an agent-scope acquire
  // and write-through-cache loads in the last block -- the guide's write-through variant of the
  // counter hand-off, which needs no release fence (cdna_hip_programming.md §5 split-K item 2);
  // stressed under uneven load against the two-launch reduction in tests/test_gpu_fusion.py.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(arrivals + blockIdx.x * RM_RED_ARR_STRIDE, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.y - 1 ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  finalize_block(S, (int)gridDim.y, M, Mpad, f, tot);
  if (tid == 0) __hip_atomic_store(arrivals + blockIdx.x * RM_RED_ARR_STRIDE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (f.raw == nullptr) return;
  // the optimizer step on the whole gradient, by the column block that finishes last: the same
  // write-through hand-off one level up (finalize_block stored its gradient elements write-through)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(f.opt_arrival, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.x - 1 ? 1 : 0;
  }
  __syncthreads();
  if (!last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  fused_optimizer(f, M);
  if (tid == 0) __hip_atomic_store(f.opt_arrival, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Pass 2 for the 256 columns of pass-1 column block blockIdx.x, by the block of that column block
// that arrived last: thread t sums column t's kReduceSegs segments in the four chains s mod 4 of
// rm_finalize_grads, combined (a0 + a1) + (a2 + a3) -- the same bits -- then the scatter.
// The light-direction gradient: light_grad (contraction off), the same function in both pass-2
// forms (finalize_block, rm_finalize_grads) and in the small kernel's final block.

// a gradient element of the final scatter: write-through when the fused optimizer reads it
__device__ __forceinline__ void put_grad(const FinalArgs& f, float* dst, float v) {
  const float x = f.accumulate ? *dst + v : v;
  if (f.raw != nullptr) __hip_atomic_store(dst, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *dst = x;
}
__device__ void finalize_block(const float* S, int nseg, int M, int Mpad, const FinalArgs& f, float* tot) {
  const int ncols = Mpad * 8 + 8;
  const int tid = threadIdx.x;
  const int col = blockIdx.x * 256 + tid;
  const int c = min(col, ncols - 1);
  // kU * 4 loads in flight per thread (the last block runs alone: registers are free)
  constexpr int kU = RM_FIN_U;
  float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int u0 = 0; u0 < nseg / 4; u0 += kU) {
    float v[kU][4];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v[u][k] = __hip_atomic_load(S + (long long)(4 * (u0 + u) + k) * ncols + c, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] += v[u][k];
  }
  tot[tid] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (col >= ncols) return;
  if (col < Mpad * 8) {
    const int j = col >> 3, comp = col & 7;
    if (j >= M || comp == 7) return;
    const float v = tot[tid];
    float* dst = comp < 3 ? (f.gc ? f.gc + 3 * j + comp : nullptr)
                          : (comp == 3 ? (f.gr ? f.gr + j : nullptr) : (f.gcol ? f.gcol + 3 * j + (comp - 4) : nullptr));
    if (dst) put_grad(f, dst, v);
    return;
  }
  const int sc = col - Mpad * 8;  // the scalars open their column block (Mpad * 8 % 256 == 0)
  if (sc == 0 && f.gld) {
    const float r[3] = {tot[tid], tot[tid + 1], tot[tid + 2]};
#pragma unroll
    for (int k = 0; k < 3; ++k) put_grad(f, f.gld + k, light_grad(r, f.light_dir, k));
  } else if (sc == 3 && f.gamb) {
    put_grad(f, f.gamb, tot[tid]);
  } else if (sc == 4 && f.loss_sum) {
    f.loss_sum[0] = f.accumulate ? f.loss_sum[0] + tot[tid] : tot[tid];
  }
}

// Pass 2 as its own launch (RM_REDUCE_FUSED=0): sum the segments in order and scatter into the
// caller's gradient layout.
// gld = (g_ell - ldn (ldn . g_ell)) / |ld| applies the Jacobian of ld / |ld| (renderer_diff.rs:49-50).
__global__ __launch_bounds__(256) void rm_finalize_grads(const float* __restrict__ S, int nseg, int M, int Mpad,
                                                         FinalArgs f) {
  // 64 columns per block, four threads per column: thread (chain k, column) sums the segments
  // s = k mod 4 in order -- the four chains of one thread's former loop (a[s & 3] += v[s]) --
  // and the chains are combined as before, (a0 + a1) + (a2 + a3): the same bits, the loads
  // spread over four times as many CUs
  __shared__ float part[4][64];
  const int ncols = Mpad * 8 + 8;
  const int cl = threadIdx.x & 63, chain = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + cl;
  static_assert(kReduceSegs % 64 == 0, "four chains of 16-load rounds");
  {
    // nseg (reduce_segs: a multiple of 64) segments, chain `chain` sums s = chain mod 4 in order,
    // kReduceSegs / 4 loads in flight
    constexpr int kC = kReduceSegs / 4;
    const int c = min(col, ncols - 1);
    float acc = 0.0f;
    for (int u0 = 0; u0 < nseg / 4; u0 += kC) {
      float v[kC];
#pragma unroll
      for (int u = 0; u < kC; ++u) v[u] = u0 + u < nseg / 4 ? S[(long long)(4 * (u0 + u) + chain) * ncols + c] : 0.0f;
#pragma unroll
      for (int u = 0; u < kC; ++u)
        if (u0 + u < nseg / 4) acc += v[u];
    }
    part[chain][cl] = acc;
  }
  __syncthreads();
  if (chain != 0 || col >= ncols) return;
  auto seg_sum = [&](int l) { return (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]); };
  if (col < Mpad * 8) {
    const int j = col >> 3, comp = col & 7;
    if (j >= M || comp == 7) return;
    const float v = seg_sum(cl);
    float* dst = comp < 3 ? (f.gc ? f.gc + 3 * j + comp : nullptr)
                          : (comp == 3 ? (f.gr ? f.gr + j : nullptr) : (f.gcol ? f.gcol + 3 * j + (comp - 4) : nullptr));
    if (dst) *dst = f.accumulate ? *dst + v : v;
    return;
  }
  const int sc = col - Mpad * 8;  // Mpad * 8 is a multiple of 64: the scalars open their block
  if (sc == 0 && f.gld) {
    const float r[3] = {seg_sum(cl), seg_sum(cl + 1), seg_sum(cl + 2)};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float gv = light_grad(r, f.light_dir, c);
      f.gld[c] = f.accumulate ? f.gld[c] + gv : gv;
    }
  } else if (sc == 3 && f.gamb) {
    const float v = seg_sum(cl);
    f.gamb[0] = f.accumulate ? f.gamb[0] + v : v;
  } else if (sc == 4 && f.loss_sum) {
    const float v = seg_sum(cl);
    f.loss_sum[0] = f.accumulate ? f.loss_sum[0] + v : v;
  }
}

// ---- model helpers (scene.rs:41-45, training.rs:38-82, Burn Adam) -------------------------
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
// burn::tensor::activation::softplus(x, 1) = log(1 + exp(x))
__device__ __forceinline__ float softplusf_(float x) { return logf(1.0f + expf(x)); }

// scene.rs:41-45 on packed element i (layout [centers 3M | colors 3M | radius M | light 3 | ambient 1]).
__device__ __forceinline__ float activate_elem(float x, int i, int M) {
#pragma clang fp contract(off)
  if (i < 3 * M) return x;                           // centers
  if (i < 6 * M) return sigmoidf_(x);                // colors = sigmoid(raw)        scene.rs:41
  if (i < 7 * M) return softplusf_(x) + 0.01f;       // radius = softplus(raw)+0.01  scene.rs:43
  if (i < 7 * M + 3) return x;                       // light_dir raw                scene.rs:44
  return sigmoidf_(x);                               // ambient = sigmoid(raw)       scene.rs:45
}

// dataset.rs:75-79: rows idx[i] of the ray / target arrays -> the batch (3 floats per row per
// array). An index outside [0, num_src) yields a zero row rather than an out-of-bounds read.
__global__ __launch_bounds__(256) void rm_gather_kernel(const float* __restrict__ org, const float* __restrict__ dir,
                                                        const float* __restrict__ tgt, long long num_src,
                                                        const int32_t* __restrict__ idx, long long n,
                                                        float* __restrict__ oo, float* __restrict__ od,
                                                        float* __restrict__ ot) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;  // one float of the [n,3] batch
  if (e >= 3 * n) return;
  const long long i = e / 3;
  const int c = (int)(e - 3 * i);
  const long long j = idx[i];
  const bool ok = j >= 0 && j < num_src;
  const long long s = 3 * j + c;
  if (oo) oo[e] = ok ? org[s] : 0.0f;
  if (od) od[e] = ok ? dir[s] : 0.0f;
  if (ot) ot[e] = ok ? tgt[s] : 0.0f;
}

// SceneDataset::sample_batch on the device (dataset.rs:47-82): batch row i draws its pixel from
// a counter-based generator -- splitmix64 over key + (i + 1) * golden, the key mixing (seed,
// stream, counter) -- so a draw depends only on its position, not on the launch geometry: rows
// i < n_uniform take a pixel uniformly from [0, num_src), the rest a foreground pixel uniformly
// from fg[0, num_fg) (the index is the high 64 bits of r * n: bias n / 2^64). Then the row's
// ray origin, direction and target are gathered (dataset.rs:75-79). One thread per row.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void rm_sample_kernel(const float* __restrict__ org, const float* __restrict__ dir,
                                                        const float* __restrict__ tgt, long long num_src,
                                                        const int32_t* __restrict__ fg, long long num_fg,
                                                        long long n_uniform, long long n, unsigned long long key,
                                                        float* __restrict__ oo, float* __restrict__ od,
                                                        float* __restrict__ ot, int32_t* __restrict__ idx_out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const unsigned long long r = splitmix64(key + (unsigned long long)(i + 1) * 0x9E3779B97F4A7C15ull);
  long long j;
  if (i < n_uniform) j = (long long)__umul64hi(r, (unsigned long long)num_src);
  else j = fg[__umul64hi(r, (unsigned long long)num_fg)];
  if (idx_out) idx_out[i] = (int32_t)j;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (oo) oo[3 * i + c] = org[3 * j + c];
    if (od) od[3 * i + c] = dir[3 * j + c];
    if (ot) ot[3 * i + c] = tgt[3 * j + c];
  }
}

__global__ __launch_bounds__(256) void rm_activate_kernel(const float* __restrict__ raw, int M,
                                                          float* __restrict__ act) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= 7 * M + 4) return;
  act[i] = activate_elem(raw[i], i, M);
}

// Block reduction of 4 floats over 256 threads in fixed tree order (deterministic).
__device__ __forceinline__ void block_sum4(float (&v)[4], float* red) {
#pragma unroll
  for (int c = 0; c < 4; ++c) red[c * 256 + threadIdx.x] = v[c];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
#pragma unroll
      for (int c = 0; c < 4; ++c) red[c * 256 + threadIdx.x] += red[c * 256 + threadIdx.x + w];
    }
    __syncthreads();
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) v[c] = red[c * 256];
}

// Repulsion row of sphere s (training.rs:73-82) over j = j0, j0 + stride, ... < M, added to v:
// dist_sj = sqrt(max(|c_s|^2 + |c_j|^2 - 2 c_s.c_j, 1e-6)), value (dist + 100 I + 1e-6)^-1 into
// v[3], its gradient w.r.t. c_s through both the (s, j) and (j, s) entries into v[0..2].
// c: the pre-step centres [M][3] (raw = activated).
__device__ __forceinline__ void repulsion_row(const float* c, int M, int s, int j0, int stride, float (&v)[4]) {
#pragma clang fp contract(off)
  const float cx = c[3 * s], cy = c[3 * s + 1], cz = c[3 * s + 2];
  const float csq = cx * cx + cy * cy + cz * cz;
  for (int j = j0; j < M; j += stride) {
    const float ox = c[3 * j], oy = c[3 * j + 1], oz = c[3 * j + 2];
    const float q = (csq + (ox * ox + oy * oy + oz * oz)) - (cx * ox + cy * oy + cz * oz) * 2.0f;
    const float qc = fmaxf(q, 1e-6f);
    const float rho = sqrtf(qc);
    const float den = rho + (j == s ? 100.0f : 0.0f) + 1e-6f;
    const float inv = frcp(den);  // v_rcp / v_rsq (1 ulp) instead of IEEE divisions: O(M^2) pairs
    v[3] += inv;
    if (j != s && q >= 1e-6f) {  // clamp_min(1e-6) gate (the diagonal has q ~ 0)
      const float gs = -2.0f * inv * inv * frsq(qc);
      v[0] += gs * (cx - ox);
      v[1] += gs * (cy - oy);
      v[2] += gs * (cz - oz);
    }
  }
}

// Pass A of the optimizer: block s owns sphere s. It snapshots the sphere's raw parameters
// (the update kernel reads neighbours' pre-step values) and, with penalties, sums the
// repulsion row of training.rs:73-82 over j (repulsion_row), block tree reduction.
__global__ __launch_bounds__(256) void rm_penalty_pairs(const float* __restrict__ raw, int M, int with_pen,
                                                        float* __restrict__ snap, float* __restrict__ pair) {
  __shared__ float red[4 * 256];
  const int s = blockIdx.x;
  if (threadIdx.x < 7) {
    const int idx = threadIdx.x < 3 ? 3 * s + threadIdx.x
                                    : (threadIdx.x < 6 ? 3 * M + 3 * s + (threadIdx.x - 3) : 6 * M + s);
    snap[idx] = raw[idx];
  }
  if (s == 0 && threadIdx.x >= 32 && threadIdx.x < 36) snap[7 * M + threadIdx.x - 32] = raw[7 * M + threadIdx.x - 32];
  if (!with_pen) return;
  float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  repulsion_row(raw, M, s, threadIdx.x, 256, v);
  block_sum4(v, red);
  if (threadIdx.x < 4) pair[4 * s + threadIdx.x] = v[threadIdx.x];
}

// One parameter element i of the packed layout: chain rule of the activations, the compute_loss
// penalties (training.rs:38-82), coupled weight decay and Burn's Adam; optionally the activated
// parameters of the updated model (scene.rs:41-45) for the next step's render. Contraction is off
// in these functions (explicit fmaf where a fused multiply-add is meant): the optimizer runs inside
// several kernels (its own launches, the reduction's and the small kernel's last blocks), and its
// bits must not depend on which. Split in two: the
// part that depends on the pre-step parameters only (optimizer_pre: the chain-rule factor, the
// penalties' gradient terms and loss share -- the fused iteration runs it while the gradient is
// still being summed) and the update itself (optimizer_apply).
struct ElemPre {
  float fac;         // d activation / d raw (1 for centres and light)
  float t0, t1, t2;  // penalty gradient terms, added in this order after the chain rule
  float pen;         // the element's penalty-loss share
};
// raw: the pre-step parameters (a snapshot: neighbours are read); pair: the repulsion rows.
__device__ __forceinline__ ElemPre optimizer_pre(int i, const float* raw, const float* pair, int M, int with_pen) {
#pragma clang fp contract(off)
  ElemPre e{1.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  const float x = raw[i];
  const float invM = 1.0f / (float)M;
  const float rep_scale = 1e-5f / ((float)M * (float)M);
  if (i < 3 * M) {  // centers (identity activation)
    if (with_pen) {
      const int s = i / 3, ax = i - 3 * s;
      const float cx = raw[3 * s], cy = raw[3 * s + 1], cz = raw[3 * s + 2];
      const float rs = softplusf_(raw[6 * M + s]);  // penalties use softplus without +0.01 (training.rs:41)
      e.t0 = 0.05f * 2.0f * x / (3.0f * M);         // [b] mean(c^2) over [M,3] * 0.05
      const float csq = cx * cx + cy * cy + cz * cz;
      const float dist = sqrtf(csq + 1e-6f);
      const float reach = dist + rs;                // [c] mean(mask * (|c| + r - 1.2)^2) * 5
      if (reach > 1.2f) e.t1 = 5.0f * invM * 2.0f * (reach - 1.2f) * (x / dist);
      e.t2 = rep_scale * pair[4 * s + ax];          // [d] repulsion (repulsion_row)
      if (ax == 0) {
        e.pen += 0.05f * csq / (3.0f * M);
        if (reach > 1.2f) e.pen += 5.0f * invM * (reach - 1.2f) * (reach - 1.2f);
        e.pen += rep_scale * pair[4 * s + 3];
      }
    }
  } else if (i < 6 * M) {  // colors: d sigmoid = c (1 - c)
    const float c = sigmoidf_(x);
    e.fac = c * (1.0f - c);
  } else if (i < 7 * M) {  // radius: d (softplus + 0.01) = sigmoid
    const float sg = sigmoidf_(x);
    e.fac = sg;
    if (with_pen) {
      const int s = i - 6 * M;
      const float rs = softplusf_(x);
      e.t0 = 0.002f * invM * (rs > 0.0f ? 1.0f : (rs < 0.0f ? -1.0f : 0.0f)) * sg;  // [a] L1
      e.pen += 0.002f * invM * fabsf(rs);
      if (rs > 1.0f) {  // [a] large radius
        e.t1 = 0.04f * invM * 2.0f * rs * sg;
        e.pen += 0.04f * invM * rs * rs;
      }
      const float cx = raw[3 * s], cy = raw[3 * s + 1], cz = raw[3 * s + 2];
      const float reach = sqrtf(cx * cx + cy * cy + cz * cz + 1e-6f) + rs;
      if (reach > 1.2f) e.t2 = 5.0f * invM * 2.0f * (reach - 1.2f) * sg;  // [c] w.r.t. radius
    }
  } else if (i >= 7 * M + 3) {  // ambient: d sigmoid (light_dir raw: identity)
    const float a = sigmoidf_(x);
    e.fac = a * (1.0f - a);
  }
  return e;
}

// Adam's bias corrections 1 - beta^t (Burn Adam: beta1 0.9, beta2 0.999)
struct AdamBias {
  float c1, c2;
};
__device__ __forceinline__ AdamBias adam_bias(int step) {
  return AdamBias{1.0f - powf(0.9f, (float)step), 1.0f - powf(0.999f, (float)step)};
}

// The update of element i from its gradient g w.r.t. the activated value, its pre-step raw value
// x and moments mo1 / mo2: gv = g fac + t0 + t1 + t2, Burn Adam with coupled weight decay
// (g += wd theta; moments; bias correction).
__device__ __forceinline__ void optimizer_apply(int i, const ElemPre& e, float g, float x, float mo1, float mo2,
                                                const AdamBias& bias, float lr, float wd, int M,
                                                float* __restrict__ raw_out, float* __restrict__ m1,
                                                float* __restrict__ m2, float* __restrict__ act_out,
                                                _Float16* __restrict__ col_h_out) {
#pragma clang fp contract(off)
  float gv = ((g * e.fac + e.t0) + e.t1) + e.t2;
  gv = fmaf(wd, x, gv);
  const float b1 = 0.9f, b2 = 0.999f, eps = 1e-5f;
  const float mm = fmaf(b1, mo1, (1.0f - b1) * gv);
  const float vv = fmaf(b2, mo2, (1.0f - b2) * gv * gv);
  m1[i] = mm;
  m2[i] = vv;
  const float mh = mm / bias.c1;
  const float vh = vv / bias.c2;
  const float xn = x - lr * (mh / (sqrtf(vh) + eps));
  raw_out[i] = xn;
  if (act_out) act_out[i] = activate_elem(xn, i, M);
  // fp16 colour models (RM_MARCH_COLOR_F16): the next render's colours, rounded to nearest
  if (col_h_out != nullptr && i >= 3 * M && i < 6 * M) col_h_out[i - 3 * M] = (_Float16)activate_elem(xn, i, M);
}

// Both parts for one element; returns the element's penalty-loss share.
__device__ __forceinline__ float optimizer_elem(int i, const float* raw, float* __restrict__ raw_out,
                                                const float* __restrict__ gact, const float* m1_in,
                                                const float* m2_in, float* __restrict__ m1, float* __restrict__ m2,
                                                const float* pair, int M, int step, float lr, float wd, int with_pen,
                                                float* __restrict__ act_out, _Float16* __restrict__ col_h_out) {
  const ElemPre e = optimizer_pre(i, raw, pair, M, with_pen);
  optimizer_apply(i, e, gact[i], raw[i], m1_in[i], m2_in[i], adam_bias(step), lr, wd, M, raw_out, m1, m2, act_out,
                  col_h_out);
  return e.pen;
}

// Pass B: one thread per parameter element (optimizer_elem); per-block penalty partials.
__global__ __launch_bounds__(256) void rm_optimizer_kernel(const float* __restrict__ raw, float* __restrict__ raw_out,
                                                           const float* __restrict__ gact,
                                                           float* __restrict__ m1, float* __restrict__ m2,
                                                           const float* __restrict__ pair, int M, int step,
                                                           float lr, float wd, int with_pen,
                                                           float* __restrict__ pen_parts,
                                                           float* __restrict__ act_out,
                                                           _Float16* __restrict__ col_h_out,
                                                           const rm_step_scalars* __restrict__ sdev) {
  __shared__ float red[4 * 256];
  if (sdev != nullptr) step = sdev->step;  // device step scalars (rm_bind_step_scalars)
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = 7 * M + 4;
  float pen = 0.0f;
  if (i < n)
    pen = optimizer_elem(i, raw, raw_out, gact, m1, m2, m1, m2, pair, M, step, lr, wd, with_pen, act_out, col_h_out);
  if (pen_parts != nullptr) {
    float v[4] = {pen, 0.0f, 0.0f, 0.0f};
    block_sum4(v, red);
    if (threadIdx.x == 0) pen_parts[blockIdx.x] = v[0];
  }
}

// The optimizer step of a small model (M <= kOptSmallMaxM) in one block: the pre-step parameters
// into LDS (the snapshot rm_penalty_pairs writes), the repulsion rows of training.rs:73-82 (four
// threads per sphere, their partials added in order), optimizer_pre per element and the penalty
// sum (block tree reduction) -- everything that does not need the gradient (opt_small_pre) --
// then optimizer_apply per element (opt_small_post). One launch instead of three.
// OptPrefetch: the block's loads of the parameters and moments (elements tid and tid + 256),
// issued before whatever the block does next (the fused iteration's final reduction) so that
// their latency overlaps it.
constexpr int kOptSmallMaxM = 64;
struct OptPrefetch {
  float x[2], a[2], b[2];
};
__device__ __forceinline__ OptPrefetch opt_prefetch(const float* raw, const float* m1, const float* m2, int M) {
  OptPrefetch f;
  const int n = 7 * M + 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = (int)threadIdx.x + 256 * h;
    f.x[h] = i < n ? raw[i] : 0.0f;
    f.a[h] = i < n ? m1[i] : 0.0f;
    f.b[h] = i < n ? m2[i] : 0.0f;
  }
  return f;
}
struct OptPre {
  ElemPre e[2];  // elements tid and tid + 256
  AdamBias bias;
};

// The gradient-independent part, for a 256-thread block (every thread calls it: block barriers).
__device__ __forceinline__ OptPre opt_small_pre(const OptPrefetch& pf, int M, int step, int with_pen,
                                                float* __restrict__ loss_penalty) {
  static_assert(7 * kOptSmallMaxM + 4 <= 512, "two elements per thread");
  __shared__ float snap[7 * kOptSmallMaxM + 4];
  __shared__ float part[4][kOptSmallMaxM][4];
  __shared__ float pair[kOptSmallMaxM * 4];
  __shared__ float red[4 * 256];
  const int tid = threadIdx.x;
  const int n = 7 * M + 4;
  OptPre o;
  o.bias = adam_bias(step);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = tid + 256 * h;
    if (i < n) snap[i] = pf.x[h];
  }
  __syncthreads();
  if (with_pen) {
    const int s = tid >> 2, k = tid & 3;  // sphere s, columns j = k mod 4
    if (s < M) {
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      repulsion_row(snap, M, s, k, 4, v);
#pragma unroll
      for (int c = 0; c < 4; ++c) part[k][s][c] = v[c];
    }
    __syncthreads();
    if (tid < 4 * M) {
      const int s2 = tid >> 2, c = tid & 3;
      pair[4 * s2 + c] = ((part[0][s2][c] + part[1][s2][c]) + part[2][s2][c]) + part[3][s2][c];
    }
    __syncthreads();
  }
  float pen = 0.0f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = tid + 256 * h;
    o.e[h] = i < n ? optimizer_pre(i, snap, pair, M, with_pen) : ElemPre{1.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    pen += o.e[h].pen;
  }
  if (loss_penalty != nullptr) {
    float v[4] = {pen, 0.0f, 0.0f, 0.0f};
    block_sum4(v, red);
    if (tid == 0) loss_penalty[0] = v[0];
  }
  return o;
}

// The update on the gradient g (w.r.t. the activated values) of elements tid and tid + 256.
__device__ __forceinline__ void opt_small_post(const OptPre& o, const OptPrefetch& pf, const float (&g)[2],
                                               float* __restrict__ raw, float* __restrict__ m1,
                                               float* __restrict__ m2, int M, float lr, float wd,
                                               float* __restrict__ act_out, _Float16* __restrict__ col_h_out) {
  const int n = 7 * M + 4;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = (int)threadIdx.x + 256 * h;
    if (i < n)
      optimizer_apply(i, o.e[h], g[h], pf.x[h], pf.a[h], pf.b[h], o.bias, lr, wd, M, raw, m1, m2, act_out,
                      col_h_out);
  }
}

__global__ __launch_bounds__(256) void rm_optimizer_small(float* __restrict__ raw, const float* __restrict__ gact,
                                                          float* __restrict__ m1, float* __restrict__ m2, int M,
                                                          int step, float lr, float wd, int with_pen,
                                                          float* __restrict__ loss_penalty, float* __restrict__ act_out,
                                                          _Float16* __restrict__ col_h_out,
                                                          rm_step_scalars* __restrict__ sdev) {
  const OptPrefetch pf = opt_prefetch(raw, m1, m2, M);
  if (sdev != nullptr) step = sdev->step;  // device step scalars (rm_bind_step_scalars)
  const int n = 7 * M + 4, i0 = (int)threadIdx.x;
  const float g[2] = {i0 < n ? gact[i0] : 0.0f, i0 + 256 < n ? gact[i0 + 256] : 0.0f};
  const OptPre o = opt_small_pre(pf, M, step, with_pen, loss_penalty);
  opt_small_post(o, pf, g, raw, m1, m2, M, lr, wd, act_out, col_h_out);
  if (sdev != nullptr) {  // every thread has read the step: the training step ends here
    __syncthreads();
    if (threadIdx.x == 0) {
      sdev->step += 1;
      sdev->index += 1;
    }
  }
}

// rm_optimizer_small's step inside the gradient reduction's last block (rm_reduce_partials,
// FinalArgs::raw): the same functions on the same values -- the gradient read with agent-scope
// loads after the hand-off -- so the same bits as the separate launch.
__device__ void fused_optimizer(const FinalArgs& f, int M) {
  const OptPrefetch pf = opt_prefetch(f.raw, f.m1, f.m2, M);
  const int step = f.sdev != nullptr ? f.sdev->step : f.step;
  const int n = 7 * M + 4, i0 = (int)threadIdx.x;
  float g[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int i = i0 + 256 * h;
    g[h] = i < n ? __hip_atomic_load(f.gc + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
  }
  const OptPre o = opt_small_pre(pf, M, step, f.with_pen, f.loss_penalty);
  opt_small_post(o, pf, g, f.raw, f.m1, f.m2, M, f.lr, f.wd, f.act_out, f.col_h);
  if (f.sdev != nullptr) {  // every thread has read the step: the training step ends here
    __syncthreads();
    if (threadIdx.x == 0) {
      f.sdev->step += 1;
      f.sdev->index += 1;
    }
  }
}

// The end of a training step with device step scalars bound (multi-block optimizer path).
__global__ void rm_step_advance(rm_step_scalars* sdev) {
  if (threadIdx.x == 0) {
    sdev->step += 1;
    sdev->index += 1;
  }
}

__global__ void rm_sum_small(const float* __restrict__ parts, int n, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float acc = 0.0f;
    for (int i = 0; i < n; ++i) acc += parts[i];
    out[0] = acc;
  }
}

#include "rm_small.h"

// rm_debug_stall: one wave that holds its stream until the host sets *flag (a system-scope load
// of host-mapped memory, polled with s_sleep) or max_ticks of the 100 MHz real-time counter have
// passed -- every run of it ends by itself. Tests use it to stand for a stuck collective.
__global__ __launch_bounds__(64) void rm_stall_kernel(const int* flag, unsigned long long max_ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(100);
  }
}

}  // namespace rm

// =======================================================================================
// C ABI
// =======================================================================================
struct rm_context {
  int device = 0;
  hipStream_t stream = nullptr;
  rm_step_scalars* sdev = nullptr;  // device step scalars (rm_bind_step_scalars), nullable
  std::string err;
  void* ws = nullptr;  // partials | segment sums | small scratch
  size_t ws_bytes = 0;
  bool timing = false;  // record hipEvents around every per-ray kernel launch
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  size_t events_used = 0;
  unsigned long long* stats_dev = nullptr;  // work counters (rm_stats_enable), kStatsWords words
  int* esc_flags = nullptr;                 // per-block escape flags, kMaxBlocksPerLaunch ints
  void* rec = nullptr;                      // sphere records of the current call (rm_prep_kernel)
  unsigned* arrivals = nullptr;             // rm_small_kernel's arrival counter (zero between launches)
  unsigned* red_arrivals = nullptr;         // rm_reduce_partials' per-column-block arrival counters
  rm::CamBasis* cams_dev = nullptr;         // camera bases of calls with > kInlineCams views (device)
  rm::CamBasis* cams_pin = nullptr;         // their pinned host staging, kCamRing slots
  hipEvent_t cam_ev[32] = {};               // slot k's copy has run (kCamRing slots)
  int cam_slot = 0;
  std::vector<rm::CamBasis> cams_shadow;    // what the device table holds (the last upload)
  float* batch = nullptr;                   // rm_train_iteration's unfused path: the drawn batch (9 floats/ray)
  float* opt_pre = nullptr;                 // rm_train_iteration: the optimizer part of the launch's extra block
  // rm_train_step_sampled_prepared: opt_pre holds the next rm_optimizer_step's gradient-independent
  // part for these arguments (consumed by that call, cleared by any other use of opt_pre)
  bool opt_prepared = false;
  const float* prep_raw = nullptr;
  float* prep_loss_penalty = nullptr;
  int prep_M = 0, prep_step = 0, prep_pen = 0;
  unsigned* opt_arrival = nullptr;          // rm_train_step_camera_adam: the reduction's column-block counter
  bool adam_done = false;                   // the last call's optimizer ran inside its reduction
  size_t batch_bytes = 0;
  size_t rec_bytes = 0;
  long long stats_blocks = 0;               // ray blocks launched while stats are on
  long long stats_waves = 0;                // their ray waves (a split block holds one)
  int* block_order = nullptr;               // centre-out tile order for order_tx x order_ty tiles
  int order_tx = 0, order_ty = 0, order_sub = 0;
  int* olist = nullptr;                     // cost-ordered dispatch: 3 x [class][kMaxBlocksPerLaunch] block lists
  int* ocnt = nullptr;                      // 3 x [class] list lengths (zeroed one launch ahead)
  float* cont_buf = nullptr;                // split continuation: saved march state | list | count
  int* stall_flag = nullptr;                // rm_debug_stall: host-mapped release flag (host pointer)
  size_t cont_bytes = 0;
  int* oturn = nullptr;                     // device word: the list set the next keyed launch appends to
  unsigned long long cost_key = 0;          // geometry of the last keyed launch (its lists order the next)
  bool cost_valid = false;
#ifdef RM_BLOCK_TRACE
  unsigned long long* btrace = nullptr;     // measurement build: per-wave records of the last launch
  long long btrace_waves = 0;
#endif
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

// Centre-out dispatch order of the ray blocks of a view's tx x ty 16x16 tiles (ray_block): by
// distance of the block's pixel-centre from the image centre, ties by block index. A block is a
// whole tile (256-ray blocks) or one of its four 8x8 quadrants (64-ray blocks: the split march), in
// the pixel order of setup_ray. Built once per image size.
int ensure_block_order(rm_context* ctx, int tx, int ty, int sub) {
  if (ctx->block_order && ctx->order_tx == tx && ctx->order_ty == ty && ctx->order_sub == sub) return RM_OK;
  // sub = ray blocks per 16x16 tile: 1 (256-ray blocks), 4 (8x8 quadrants: 64-ray split blocks),
  // 8 (8x4 halves of the quadrants: 32-ray split blocks) or 16 (8x2 quarters: 16-ray split blocks)
  std::vector<int> ord((size_t)tx * ty * sub);
  for (size_t i = 0; i < ord.size(); ++i) ord[i] = (int)i;
  auto key = [&](int i) {  // twice the pixel offset of the block centre from the image centre
    const int tile = i / sub, q = i % sub;
    const int per_quad = sub / 4, quad = sub == 1 ? 0 : q / per_quad, part = sub == 1 ? 0 : q % per_quad;
    const long long rows = sub == 1 ? 16 : 8 / per_quad;  // pixel rows of one block inside its quadrant
    const long long ox = sub == 1 ? 16 : 16 * (quad & 1) + 8,
                    oy = sub == 1 ? 16 : 16 * (quad >> 1) + 2 * rows * part + rows;
    const long long dx = 32LL * (tile % tx) + ox - 16LL * tx, dy = 32LL * (tile / tx) + oy - 16LL * ty;
    return dx * dx + dy * dy;
  };
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return key(x) < key(y); });
  if (const char* e = std::getenv("RM_ORDER_EXPERIMENT")) {  // A/B of dispatch orders (timing only)
    const int mode = std::atoi(e);
    if (mode == 1) std::reverse(ord.begin(), ord.end());  // border tiles first
    if (mode == 2) {  // alternate centre and border: heavy and light blocks interleaved
      std::vector<int> o2;
      size_t lo = 0, hi = ord.size();
      while (lo < hi) {
        o2.push_back(ord[lo++]);
        if (lo < hi) o2.push_back(ord[--hi]);
      }
      ord.swap(o2);
    }
  }
  if (ctx->block_order) {
    RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    RM_HIP(ctx, hipFree(ctx->block_order));
    ctx->block_order = nullptr;
  }
  RM_HIP(ctx, hipMalloc(&ctx->block_order, sizeof(int) * ord.size()));
  RM_HIP(ctx, hipMemcpy(ctx->block_order, ord.data(), sizeof(int) * ord.size(), hipMemcpyHostToDevice));
  ctx->order_tx = tx;
  ctx->order_ty = ty;
  ctx->order_sub = sub;
  return RM_OK;
}

bool env_is(const char* name, char v) {
  const char* e = std::getenv(name);
  return e && e[0] == v;
}

int pad_spheres(int M) { return (M + kSphereAlign - 1) / kSphereAlign * kSphereAlign; }
// column blocks of the reduction at the largest scene (RM_MAX_SPHERES): its arrival counters
constexpr int kRedArrivals = (RM_MAX_SPHERES * 8 + 8 + 255) / 256 * RM_RED_ARR_STRIDE;

// Ray blocks per per-ray launch: kMaxBlocksPerLaunch, or less with the environment variable
// RM_MAX_BLOCKS_PER_LAUNCH (tests use it to exercise the sub-launch split at small sizes).
long long max_blocks_per_launch() {
  const char* e = std::getenv("RM_MAX_BLOCKS_PER_LAUNCH");
  const long long v = e ? std::atoll(e) : 0;
  return (v >= 1 && v <= kMaxBlocksPerLaunch) ? v : kMaxBlocksPerLaunch;
}

long long rec_floats(int Mpad) { return (long long)Mpad * 8 + 8; }

// March steps after which a split launch hands the blocks still marching to a continuation
// launch: env RM_SPLIT_CONT_STEPS (0 = one launch), else max(32, 3 S / 8) for S >= 64 march steps
// (measured, tools/gpu_env_ab.sh: at 4096 spheres S = 128 step 48 gave -20 %, S = 64 step 32 -8 %;
// at S = 32 any step was slower).
int split_cont_steps(int steps) {
  if (const char* e = std::getenv("RM_SPLIT_CONT_STEPS")) return std::max(0, std::atoi(e));
  return steps >= 64 ? std::max(32, 3 * steps / 8) : 0;
}
// The second continuation (a third launch) from S >= 128: at 3S/4 the blocks still marching are
// dealt out again over the CUs (C5 / C5g with 32-ray groups, three rounds on one box: +2.5 % /
// +3.5 % at 96 of 128 steps, profiles/r06_ab.txt r06r). 0 = none; env RM_SPLIT_CONT2_STEPS.
int split_cont2_steps(int steps) {
  if (const char* e = std::getenv("RM_SPLIT_CONT2_STEPS")) return std::max(0, std::atoi(e));
  return steps >= 128 ? 3 * steps / 4 : 0;
}
// The continuation steps of a split launch, increasing, each < steps: caps[0..n), caps[n] = 0.
// Env RM_SPLIT_CONT_LIST="48,80,112" replaces the rule (up to kMaxCont steps).
constexpr int kMaxCont = 4;
int split_cont_caps(int steps, int (&caps)[kMaxCont + 1]) {
  int n = 0;
  if (const char* e = std::getenv("RM_SPLIT_CONT_LIST")) {
    for (const char* q = e; *q && n < kMaxCont;) {
      const int v = std::atoi(q);
      if (v > 0 && v < steps && (n == 0 || v > caps[n - 1])) caps[n++] = v;
      while (*q && *q != ',') ++q;
      if (*q == ',') ++q;
    }
  } else if (steps >= 128 && !std::getenv("RM_SPLIT_CONT_STEPS") && !std::getenv("RM_SPLIT_CONT2_STEPS")) {
    // ray mode: a continuation costs only the rays still marching, so defer earlier and more
    // often -- 3S/16, 3S/8, 3S/4 (C5g, one box: 24 / 48 / 96 of 128 steps 42.3 Mrays/s against 39.8
    // with 48 / 96 and 40.1 with 32 / 96; 16 / 32 / 64 / 96 42.3; C5 within 1 %, profiles/r07g)
    caps[n++] = 3 * steps / 16;
    caps[n++] = 3 * steps / 8;
    caps[n++] = 3 * steps / 4;
  } else {
    const int c0 = split_cont_steps(steps), c1 = split_cont2_steps(steps);
    if (c0 > 0 && c0 < steps) {
      caps[n++] = c0;
      if (c1 > c0 && c1 < steps) caps[n++] = c1;
    }
  }
  for (int i = n; i <= kMaxCont; ++i) caps[i] = 0;
  return n;
}

size_t ws_need(long long max_rays, int M, int rays_per_block = kBlock) {
  const int Mpad = pad_spheres(M);
  long long blocks = (max_rays + rays_per_block - 1) / rays_per_block;
  blocks = std::min<long long>(blocks, kMaxBlocksPerLaunch);
  const long long rec = rec_floats(Mpad);
  return (size_t)(blocks * rec + (long long)reduce_segs(blocks) * rec + 4096) * sizeof(float);
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

int check_scene(rm_context* ctx, const rm_scene* s, bool need_light) {
  if (!s) return fail(ctx, RM_ERR_INVALID_ARG, "scene is NULL");
  if (s->num_spheres < 1 || s->num_spheres > RM_MAX_SPHERES)
    return fail(ctx, RM_ERR_INVALID_ARG, "num_spheres %d out of [1, %d]", s->num_spheres, RM_MAX_SPHERES);
  if (!s->centers || !s->colors || !s->radius || (need_light && (!s->light_dir || !s->ambient)))
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
  // rm_train_iteration: org / dir / targets are the dataset arrays the kernel draws the batch
  // from, and the optimizer runs in the same launch (rm_small_kernel<kTrain, MB, true>)
  const SmallArgs* fused = nullptr;
  // rm_train_step_camera_adam: the optimizer step on the packed gradient (grads->centers), run by
  // the gradient reduction's last block where it can (rm_context::adam_done says whether it did)
  struct Adam {
    float *raw, *m1, *m2, *act_out, *loss_penalty;
    _Float16* col_h;
    int step, with_pen;
    float lr, wd;
  };
  const Adam* adam = nullptr;
};

FinalArgs final_args(const Call& c, bool first) {
  const rm_grads* gp = c.grads;
  FinalArgs fa{};
  fa.light_dir = c.scene->light_dir;
  fa.gc = gp->centers;
  fa.gcol = gp->colors;
  fa.gr = gp->radius;
  fa.gld = gp->light_dir;
  fa.gamb = gp->ambient;
  fa.loss_sum = c.mode == kTrain ? c.loss_sum : nullptr;
  fa.accumulate = first ? c.accumulate : 1;
  fa.oturn = nullptr;
  return fa;
}

// The fixed-order cross-block reduction of a launch's nb partial records (a.partials) and the
// gradient scatter into the caller's layout (rm_reduce_partials + rm_finalize_grads).
int reduce_and_finalize(rm_context* ctx, const Call& c, const KArgs& a, long long nb, bool first, bool only = false) {
  FinalArgs fa = final_args(c, first);
  fa.oturn = const_cast<int*>(a.oturn);  // a keyed launch: its reduction advances the turn
  const int nblocks = (int)nb;
  const int ncols = a.Mpad * 8 + 8;
  float* S = a.partials + (long long)std::max<long long>(nb, 1) * a.rec;
  const int segs = reduce_segs(nblocks);  // every segment is written (empty ones as 0)
  const int seg_len = (nblocks + segs - 1) / segs;
  // pass 1 compacts a segment's rows in one 256-entry list (rm_reduce_partials)
  if (seg_len > 256) return fail(ctx, RM_ERR_INVALID_ARG, "%d ray blocks in one launch", nblocks);
  const int xblocks = (ncols + 255) / 256;
  // pass 2 in the same launch (the last-arriving segment block of each column block) unless
  // RM_REDUCE_FUSED=0 (then rm_finalize_grads: the same bits)
  const bool fused = !env_is("RM_REDUCE_FUSED", '0');
  if (fused && !ctx->red_arrivals) {
    RM_HIP(ctx, hipMalloc(&ctx->red_arrivals, sizeof(unsigned) * kRedArrivals));
    RM_HIP(ctx, hipMemsetAsync(ctx->red_arrivals, 0, sizeof(unsigned) * kRedArrivals, ctx->stream));
  }
  // rm_train_step_camera_adam: the optimizer in the reduction's last block (one launch, the only
  // one of the call, M <= kOptSmallMaxM, the fused reduction)
  if (c.adam != nullptr && only && fused && a.M <= kOptSmallMaxM && !env_is("RM_OPT_SMALL", '0') &&
      !env_is("RM_FUSED_ADAM", '0')) {
    if (!ctx->opt_arrival) {
      RM_HIP(ctx, hipMalloc(&ctx->opt_arrival, 128));
      RM_HIP(ctx, hipMemsetAsync(ctx->opt_arrival, 0, 128, ctx->stream));
    }
    fa.raw = c.adam->raw;
    fa.m1 = c.adam->m1;
    fa.m2 = c.adam->m2;
    fa.act_out = c.adam->act_out;
    fa.loss_penalty = c.adam->loss_penalty;
    fa.col_h = c.adam->col_h;
    fa.sdev = ctx->sdev;
    fa.opt_arrival = ctx->opt_arrival;
    fa.step = c.adam->step;
    fa.with_pen = c.adam->with_pen;
    fa.lr = c.adam->lr;
    fa.wd = c.adam->wd;
    ctx->adam_done = true;
  }
  hipLaunchKernelGGL(rm_reduce_partials, dim3((unsigned)xblocks, (unsigned)segs), dim3(256), 0, ctx->stream, a.partials,
                     a.rec, a.M, a.Mpad, nblocks, seg_len, S, fa, fused ? ctx->red_arrivals : nullptr);
  RM_HIP(ctx, hipGetLastError());
  if (!fused) {
    hipLaunchKernelGGL(rm_finalize_grads, dim3((unsigned)((ncols + 63) / 64)), dim3(256), 0, ctx->stream, S, segs, a.M,
                       a.Mpad, final_args(c, first));
    RM_HIP(ctx, hipGetLastError());
  }
  return RM_OK;
}

// Per-launch timing events (rm_timing_enable): the next pair of the context's pool.
int next_events(rm_context* ctx, hipEvent_t& ev0, hipEvent_t& ev1) {
  ev0 = ev1 = nullptr;
  if (!ctx->timing) return RM_OK;
  if (ctx->events_used == ctx->events.size()) {
    std::pair<hipEvent_t, hipEvent_t> pr;
    RM_HIP(ctx, hipEventCreate(&pr.first));
    RM_HIP(ctx, hipEventCreate(&pr.second));
    ctx->events.push_back(pr);
  }
  ev0 = ctx->events[ctx->events_used].first;
  ev1 = ctx->events[ctx->events_used].second;
  ++ctx->events_used;
  return RM_OK;
}

// Small scenes (M <= kSmallMaxM): rm_small_kernel. Taken by default for ray-array calls (the
// reference training loop's random batches, train.rs:169-199) and for camera calls of up to
// kSmallCamMaxRays rays (64x64 / 16 steps: 13.5 vs 56 us, 256x256 / 40 steps: 25 vs 84 us;
// tools/small_batch_sweep.py -- larger camera calls keep the general kernel's exact early exits);
// env RM_SMALL=1 takes it for every eligible call, RM_SMALL=0 never. Not for the renderer.rs
// mode, the diagnostics or the flags that select the general kernel's march paths for testing.
constexpr long long kSmallCamMaxRays = 1LL << 20;
bool use_small(const Call& c, int M, long long n) {
  if (M > kSmallMaxM || n <= 0 || c.mode == kRender || c.dbg) return false;
  if ((c.march->flags & (RM_MARCH_VALU_ONLY | RM_MARCH_FORCE_MAX_SHIFT | RM_MARCH_SPLIT | RM_MARCH_PER_RAY_ORIGIN |
                         RM_MARCH_SKIP_ESCAPED)) != 0)
    return false;
  const char* e = std::getenv("RM_SMALL");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return !c.cam || n <= kSmallCamMaxRays;
}

// rm_small_kernel for M spheres: the bucket of M rounded up to a multiple of 4
template <int MODE, bool FUSED = false, int LPR = 1>
void launch_small_m(int M, dim3 grid, hipStream_t st, const KArgs& a, const SmallArgs& sa, hipEvent_t ev0,
                    hipEvent_t ev1) {
  const dim3 blk(kBlock);
  switch ((M + 3) / 4) {
#define RM_SMALL_CASE(C, MB) \
  case C: hipExtLaunchKernelGGL((rm_small_kernel<MODE, MB, FUSED, LPR>), grid, blk, 0, st, ev0, ev1, 0u, a, sa); break;
    RM_SMALL_CASE(1, 4)
    RM_SMALL_CASE(2, 8)
    RM_SMALL_CASE(3, 12)
    RM_SMALL_CASE(4, 16)
    RM_SMALL_CASE(5, 20)
    RM_SMALL_CASE(6, 24)
    RM_SMALL_CASE(7, 28)
#undef RM_SMALL_CASE
    default: hipExtLaunchKernelGGL((rm_small_kernel<MODE, 32, FUSED, LPR>), grid, blk, 0, st, ev0, ev1, 0u, a, sa); break;
  }
}

// Lanes per ray of a small-kernel call: train steps of up to 32,768 rays split each ray's march
// over two lanes (rm_small.h, LPR; 16,384 rays: 18.6 vs 19.7 us, 4,096: 15.9 vs 19.2; from
// 65,536 rays the SIMDs are full and one lane per ray is faster, 25.6 vs 28.7). Env
// RM_SMALL_LPR=1 / 2 forces one or two.
int small_lpr(const Call& c, long long n) {
  if (c.mode != kTrain || env_is("RM_SMALL_LPR", '1')) return 1;
  return env_is("RM_SMALL_LPR", '2') || n <= 32768 ? 2 : 1;
}

int run_small(rm_context* ctx, const Call& c, KArgs& a, long long n) {
  const bool has_bwd = c.mode == kBwd || c.mode == kTrain;
  const int lpr = small_lpr(c, n), rpb = kBlock / lpr;
  int rc;
  if (has_bwd && (rc = ensure_ws(ctx, ws_need(n, a.M, rpb))) != RM_OK) return rc;
  if (!ctx->arrivals) {
    RM_HIP(ctx, hipMalloc(&ctx->arrivals, 64));
    RM_HIP(ctx, hipMemsetAsync(ctx->arrivals, 0, 64, ctx->stream));
  }
  long long done = 0;
  bool first = true;
  while (done < n) {
    const long long nb = std::min<long long>((n - done + rpb - 1) / rpb, max_blocks_per_launch());
    const long long nr = std::min<long long>(n - done, nb * rpb);
    a.ray_begin = done;
    a.n_rays = nr;
    a.partials = static_cast<float*>(ctx->ws);
#ifdef RM_BLOCK_TRACE
    if (!ctx->btrace)
      RM_HIP(ctx, hipMalloc(&ctx->btrace, sizeof(unsigned long long) * kTraceWords * kWaves * (size_t)kMaxBlocksPerLaunch));
    RM_HIP(ctx, hipMemsetAsync(ctx->btrace, 0, sizeof(unsigned long long) * kTraceWords * kWaves * (size_t)(nb + 1), ctx->stream));
    a.btrace = ctx->btrace;
    ctx->btrace_waves = (nb + (c.fused && c.fused->adam ? 1 : 0)) * kWaves;
#endif
    SmallArgs sa;
    std::memset(&sa, 0, sizeof sa);
    if (c.fused) sa = *c.fused;
    if (has_bwd) sa.fin = final_args(c, first);
    sa.arrivals = ctx->arrivals;
    sa.final_in_kernel = has_bwd && nb <= kSmallFinalMaxBlocks && !env_is("RM_SMALL_FINAL", '0') ? 1 : 0;
    sa.acquire = env_is("RM_SMALL_ACQUIRE", '0') ? 0 : 1;
    if (c.fused && (!sa.final_in_kernel || nr != n))  // rm_train_iteration / _step_sampled checked this
      return fail(ctx, RM_ERR_INVALID_ARG, "fused iteration needs one launch of <= %d blocks", kSmallFinalMaxBlocks);
    const bool extra = c.fused && sa.adam;  // the launch's extra (optimizer) block
    if (ctx->stats_dev) {
      ctx->stats_blocks += nb;
      ctx->stats_waves += nb * kWaves;
    }
    if (extra) {  // the extra block's optimizer part (rm_small.h)
      if (!ctx->opt_pre) RM_HIP(ctx, hipMalloc(&ctx->opt_pre, sizeof(float) * (4 * kOptPreStride + 2)));
      sa.opt_pre = ctx->opt_pre;
      ctx->opt_prepared = false;  // a preparing call records its arguments after the launch
    }
    hipEvent_t ev0, ev1;
    if ((rc = next_events(ctx, ev0, ev1)) != RM_OK) return rc;
    const dim3 grid((unsigned)(nb + (extra ? 1 : 0)));
    if (c.fused && lpr == 2) launch_small_m<kTrain, true, 2>(a.M, grid, ctx->stream, a, sa, ev0, ev1);
    else if (c.fused) launch_small_m<kTrain, true>(a.M, grid, ctx->stream, a, sa, ev0, ev1);
    else if (c.mode == kFwd) launch_small_m<kFwd>(a.M, grid, ctx->stream, a, sa, ev0, ev1);
    else if (c.mode == kBwd) launch_small_m<kBwd>(a.M, grid, ctx->stream, a, sa, ev0, ev1);
    else if (lpr == 2) launch_small_m<kTrain, false, 2>(a.M, grid, ctx->stream, a, sa, ev0, ev1);
    else launch_small_m<kTrain>(a.M, grid, ctx->stream, a, sa, ev0, ev1);
    RM_HIP(ctx, hipGetLastError());
    if (has_bwd && !sa.final_in_kernel && (rc = reduce_and_finalize(ctx, c, a, nb, first)) != RM_OK) return rc;
    done += nr;
    first = false;
  }
  return RM_OK;
}

template <int MODE>
void launch_escape(bool cam, dim3 grid, hipStream_t st, const KArgs& a, int* flags) {
  if (cam)
    hipLaunchKernelGGL((rm_escape_kernel<MODE, true>), grid, dim3(kBlock), 0, st, a, flags);
  else
    hipLaunchKernelGGL((rm_escape_kernel<MODE, false>), grid, dim3(kBlock), 0, st, a, flags);
}

template <int MODE>
void launch_cont(bool cam, dim3 grid, size_t lds, hipStream_t st, const KArgs& a, hipEvent_t ev0, hipEvent_t ev1) {
  const dim3 blk(64 * kSplitWaves);
  if (cam) hipExtLaunchKernelGGL((rm_cont_kernel<MODE, true>), grid, blk, (uint32_t)lds, st, ev0, ev1, 0u, a);
  else hipExtLaunchKernelGGL((rm_cont_kernel<MODE, false>), grid, blk, (uint32_t)lds, st, ev0, ev1, 0u, a);
}

template <int MODE>
void launch_ray(bool cam, bool split, dim3 grid, size_t lds, hipStream_t st, const KArgs& a, hipEvent_t ev0,
                hipEvent_t ev1) {
  // With timing on, the start/stop timestamps come from the kernel's own dispatch packet
  // (hipExtLaunchKernel): no extra barrier packets or cache flushes around the launch.
  const dim3 blk(split ? 64 * kSplitWaves : kBlock);
  const uint32_t sh = (uint32_t)lds;
  if (split) {
    if (cam) hipExtLaunchKernelGGL((rm_ray_kernel<MODE, true, true>), grid, blk, sh, st, ev0, ev1, 0u, a);
    else hipExtLaunchKernelGGL((rm_ray_kernel<MODE, false, true>), grid, blk, sh, st, ev0, ev1, 0u, a);
  } else {
    if (cam) hipExtLaunchKernelGGL((rm_ray_kernel<MODE, true, false>), grid, blk, sh, st, ev0, ev1, 0u, a);
    else hipExtLaunchKernelGGL((rm_ray_kernel<MODE, false, false>), grid, blk, sh, st, ev0, ev1, 0u, a);
  }
}

// Camera bases of a call with more than kInlineCams views: built on the host (make_basis), staged
// in one of kCamRing pinned slots and copied to the context's device table on its stream (the
// copy is ordered after the previous call's kernels, so one device table serves every call; a
// pinned slot is rewritten only after its previous copy has run).
constexpr int kCamRing = 32;  // calls of > 16 views in flight before the host waits for a slot
static_assert(sizeof(rm_context::cam_ev) / sizeof(hipEvent_t) == kCamRing, "one event per staging slot");
int upload_cams(rm_context* ctx, const Call& c, KArgs& a) {
  int rc;
  if (!ctx->cams_dev) {
    if (hipMalloc(&ctx->cams_dev, sizeof(CamBasis) * RM_MAX_VIEWS_PER_CALL) != hipSuccess)
      return fail(ctx, RM_ERR_OOM, "camera table");
    if (hipHostMalloc(&ctx->cams_pin, sizeof(CamBasis) * RM_MAX_VIEWS_PER_CALL * kCamRing) != hipSuccess)
      return fail(ctx, RM_ERR_OOM, "camera staging");
    for (hipEvent_t& e : ctx->cam_ev) RM_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  RM_HIP(ctx, hipStreamIsCapturing(ctx->stream, &cap));
  if (cap != hipStreamCaptureStatusNone) {
    // under hipGraph capture nothing may wait or stage: the call must find its views in the device
    // table already -- an eager call with the same views on this context uploaded them -- and the
    // replays read that table (the caller keeps it: no call with other views on this context)
    std::vector<CamBasis> want(c.views);
    for (int v = 0; v < c.views; ++v)
      if ((rc = make_basis(ctx, c.cams[v], c.W, c.H, want[v])) != RM_OK) return rc;
    if (ctx->cams_shadow.size() != want.size() ||
        std::memcmp(ctx->cams_shadow.data(), want.data(), sizeof(CamBasis) * want.size()) != 0)
      return fail(ctx, RM_ERR_UNSUPPORTED,
                  "a captured call of %d views reads the context's camera table: run the same call once before "
                  "the capture", c.views);
    a.cams_dev = ctx->cams_dev;
    return RM_OK;
  }
  const int slot = ctx->cam_slot;
  ctx->cam_slot = (slot + 1) % kCamRing;
  RM_HIP(ctx, hipEventSynchronize(ctx->cam_ev[slot]));
  CamBasis* pin = ctx->cams_pin + (size_t)slot * RM_MAX_VIEWS_PER_CALL;
  for (int v = 0; v < c.views; ++v)
    if ((rc = make_basis(ctx, c.cams[v], c.W, c.H, pin[v])) != RM_OK) return rc;
  RM_HIP(ctx, hipMemcpyAsync(ctx->cams_dev, pin, sizeof(CamBasis) * c.views, hipMemcpyHostToDevice, ctx->stream));
  RM_HIP(ctx, hipEventRecord(ctx->cam_ev[slot], ctx->stream));
  ctx->cams_shadow.assign(pin, pin + c.views);
  a.cams_dev = ctx->cams_dev;
  return RM_OK;
}

int run(rm_context* ctx, const Call& c) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  // a prepared optimizer step is for the rm_optimizer_step right after its own sampled step: any
  // other call in between may change the parameters it was prepared on (sampled_step sets it again)
  ctx->opt_prepared = false;
  int rc;
  if ((rc = check_scene(ctx, c.scene, c.mode != kRender)) != RM_OK) return rc;
  if ((rc = check_march(ctx, c.march)) != RM_OK) return rc;
  KArgs a;
  std::memset(&a, 0, sizeof a);
  if (c.cam) {
    if (!c.cams) return fail(ctx, RM_ERR_INVALID_ARG, "cams is NULL");
    if (c.views < 1 || c.views > RM_MAX_VIEWS_PER_CALL)
      return fail(ctx, RM_ERR_INVALID_ARG, "num_views %d out of [1, %d]", c.views, RM_MAX_VIEWS_PER_CALL);
    if (c.W < 1 || c.H < 1 || (long long)c.W * c.H > (1LL << 28))
      return fail(ctx, RM_ERR_INVALID_ARG, "bad image size %dx%d", c.W, c.H);
    a.cams_dev = nullptr;
    if (c.views <= kInlineCams) {
      for (int v = 0; v < c.views; ++v)
        if ((rc = make_basis(ctx, c.cams[v], c.W, c.H, a.cams[v])) != RM_OK) return rc;
    } else if ((rc = upload_cams(ctx, c, a)) != RM_OK) {
      return rc;
    }
    a.width = c.W;
    a.height = c.H;
    // Compact 16x16 tiles per block (8x8 per wave): more waves whose rays all miss the scene
    // leave the march early (68 % vs 62 % of waves at the metric view, +3-4 %).
    a.tiling = (c.W % 16 == 0 && c.H % 16 == 0) ? 2 : 0;
    a.num_views = c.views;
  } else {
    if (c.n < 0) return fail(ctx, RM_ERR_INVALID_ARG, "num_rays %lld < 0", c.n);
    if (c.n > 0 && (!c.org || !c.dir)) return fail(ctx, RM_ERR_INVALID_ARG, "ray_org/ray_dir is NULL");
  }
  const long long n = c.cam ? (long long)c.views * c.W * c.H : c.n;
  if ((c.mode == kFwd || c.mode == kRender) && n > 0 && !c.out && !c.t_out && !c.dbg) return fail(ctx, RM_ERR_INVALID_ARG, "no output requested");
  if (c.mode == kBwd && n > 0 && !c.gout) return fail(ctx, RM_ERR_INVALID_ARG, "grad_out is NULL");
  if (c.mode == kTrain && n > 0 && !c.targets) return fail(ctx, RM_ERR_INVALID_ARG, "targets is NULL");
  const bool has_bwd = c.mode == kBwd || c.mode == kTrain;
  if (has_bwd && !c.grads) return fail(ctx, RM_ERR_INVALID_ARG, "grads is NULL");

  const int M = c.scene->num_spheres;
  const int Mpad = pad_spheres(M);
  a.org = c.org;
  a.dir = c.dir;
  a.centers = c.scene->centers;
  if ((c.march->flags & RM_MARCH_COLOR_F16) != 0) {
    a.colors = nullptr;
    a.colors_h = reinterpret_cast<const _Float16*>(c.scene->colors);
  } else {
    a.colors = c.scene->colors;
  }
  a.radius = c.scene->radius;
  a.light_dir = c.scene->light_dir;
  a.ambient = c.scene->ambient;
  a.M = M;
  a.Mpad = Mpad;
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
  a.sdev = ctx->sdev;
  a.dbg = c.dbg;
  // Escape skipping needs the mask to be exactly 0 at the certified distance: sigmoid(-msharp D)
  // once msharp log2(e) D > 128 overflows exp2 (use 160), exp(-10 D^2) in kRender long before 50.
  const bool mask_vanishes = c.mode == kRender || a.msharp > 0.0f;
  // Split march (RM_MARCH_SPLIT): forced by the flag or env RM_SPLIT=1, automatic by sphere count
  // and rays per launch (kSplitMinSpheres / kSplitMaxRays, kSplitMinSpheresWide / ...Wide); never with
  // RM_MARCH_NO_SPLIT / env RM_SPLIT=0, in the renderer.rs mode or with the escape pre-pass.
  bool split = false;
  if (c.mode != kRender && (c.march->flags & RM_MARCH_SKIP_ESCAPED) == 0) {
    const char* e = std::getenv("RM_SPLIT");
    const long long n_all = c.cam ? (long long)c.views * c.W * c.H : c.n;
    if ((c.march->flags & RM_MARCH_SPLIT) != 0 || (e && e[0] == '1')) split = true;
    else if ((c.march->flags & RM_MARCH_NO_SPLIT) == 0 && !(e && e[0] == '0'))
      split = (M >= kSplitMinSpheres && n_all <= kSplitMaxRays) || (M >= kSplitMinSpheresWide && n_all <= kSplitMaxRaysWide);
  }
  a.split = split ? 1 : 0;
  // ray mode in every split launch (the scene-uniform shift, per-ray retirement and the ray-level
  // continuation; the split kernels are compiled for it, KArgs::ray_mode)
  a.ray_mode = split ? 1 : 0;
  const int rpb = split ? kSplitRays : kBlock;  // rays per block
  a.cull = ((c.march->flags & RM_MARCH_SKIP_ESCAPED) != 0 && mask_vanishes && !c.t_out && !c.dbg && !split) ? 1 : 0;
  a.cull_min_d = c.mode == kRender ? 50.0f : std::max(50.0f, 160.0f / (a.msharp * 1.44269504f));
  a.lse_slack = (float)(std::log((double)M) / (double)a.k * (1.0 + 1e-6)) + 1e-7f;
  // Escaped-ray early exit: the mask must be exactly 0 at distance gone_d -- exp2 of
  // msharp log2(e) D overflows at 128 (use 130; the reference's sigmoid(-15 D) is 0 from 5.92);
  // exp(-10 D^2) underflows long before 6.
  // Gone rays (the march) in every mode but the diagnostics; the exit itself not when the march t
  // of every ray is requested (t_out) or with RM_MARCH_NO_EARLY_EXIT.
  a.gone_d = 0.0f;
  if (!c.dbg) {
    if (c.mode == kRender) a.gone_d = 6.0f;
    else if (a.msharp > 0.0f) a.gone_d = std::max(6.0f, 130.0f / (a.msharp * 1.44269504f));
  }
  a.early_exit = a.gone_d > 0.0f && (c.march->flags & RM_MARCH_NO_EARLY_EXIT) == 0 && !c.t_out ? 1 : 0;
  if ((c.march->flags & RM_MARCH_ROW_ORDER) != 0) a.tiling = 0;
  a.mfma = (c.march->flags & RM_MARCH_VALU_ONLY) == 0;
  a.shift_max = (c.march->flags & RM_MARCH_FORCE_MAX_SHIFT) != 0;
  if (c.mode == kRender) {  // renderer.rs:27-32, normalised in f32 on the host like the reference
    const float lv[3] = {-0.5f, 0.5f, -1.0f};
    const float len = std::sqrt(lv[0] * lv[0] + lv[1] * lv[1] + lv[2] * lv[2]);
    for (int i = 0; i < 3; ++i) a.light_fixed[i] = lv[i] / len;
  }
  a.rec = rec_floats(Mpad);
  if (use_small(c, M, n)) return run_small(ctx, c, a, n);
  if (c.fused) return fail(ctx, RM_ERR_INVALID_ARG, "fused iteration outside the small kernel");
  // sphere records of this call (rm_prep_kernel): read by every sweep through scalar loads
  if (n > 0) {
    const int np = Mpad / 2, nprep = (np + 255) / 256;
    const size_t need = rec_bytes(np, nprep);
    if (need > ctx->rec_bytes) {
      if (ctx->rec) {
        RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
        RM_HIP(ctx, hipFree(ctx->rec));
        ctx->rec = nullptr;
        ctx->rec_bytes = 0;
      }
      if (hipMalloc(&ctx->rec, need) != hipSuccess) return fail(ctx, RM_ERR_OOM, "record buffer (%zu B)", need);
      ctx->rec_bytes = need;
    }
    // camera mode: the per-view first march step at the eye, shared by every ray of the view
    a.origin = (c.cam && (c.march->flags & (RM_MARCH_PER_RAY_ORIGIN | RM_MARCH_FORCE_MAX_SHIFT)) == 0)
                   ? reinterpret_cast<float*>((char*)ctx->rec + origin_offset(np, nprep))
                   : nullptr;
    hipLaunchKernelGGL(rm_prep_kernel, dim3(nprep), dim3(256), 0, ctx->stream, a, (float4*)ctx->rec);
    RM_HIP(ctx, hipGetLastError());
    if (nprep > 1) {
      float* hdr = reinterpret_cast<float*>((char*)ctx->rec + (size_t)np * (7 * 16 + 8));
      float* esc = reinterpret_cast<float*>((char*)ctx->rec + esc_offset(np, nprep));
      hipLaunchKernelGGL(rm_prep_finish, dim3(1), dim3(256), 0, ctx->stream, a, hdr, esc, nprep);
      RM_HIP(ctx, hipGetLastError());
    }
    if (a.origin != nullptr) {
      if (a.split)
        hipLaunchKernelGGL(rm_origin_kernel<true>, dim3(c.views), dim3(64 * kSplitWaves), 0, ctx->stream, a,
                           (const float4*)ctx->rec, nprep);
      else
        hipLaunchKernelGGL(rm_origin_kernel<false>, dim3(c.views), dim3(64), 0, ctx->stream, a, (const float4*)ctx->rec,
                           nprep);
      RM_HIP(ctx, hipGetLastError());
    }
    a.rec_buf = (const float4*)ctx->rec;
  }
  const size_t lds = lds_bytes();

  if (has_bwd) {
    if ((rc = ensure_ws(ctx, ws_need(std::max<long long>(n, 1), M, rpb))) != RM_OK) return rc;
  }
  float* P = static_cast<float*>(ctx->ws);

  if (n == 0) {  // nothing to render; backward/train still define their outputs
    if (!has_bwd) return RM_OK;
  }
  long long done = 0;
  bool first = true;
  do {
    const long long blocks_left = (n - done + rpb - 1) / rpb;
    const long long nb = std::min<long long>(blocks_left, max_blocks_per_launch());
    const long long nr = std::min<long long>(n - done, nb * rpb);
    a.ray_begin = done;
    a.n_rays = nr;
    a.partials = P;
    a.stats = ctx->stats_dev;
    if (ctx->stats_dev) {
      ctx->stats_blocks += nb;
      ctx->stats_waves += nb * (split ? 1 : kWaves);
    }
    a.esc_flags = nullptr;
    a.block_order = nullptr;
    a.olist_r = nullptr;
    a.ocnt_r = nullptr;
    a.olist_w = nullptr;
    a.ocnt_w = nullptr;
    a.ocnt_z = nullptr;
    a.oturn = nullptr;
    const long long npix = (long long)c.W * c.H;
    if (c.cam && a.tiling == 2 && nb > 1 && done % npix == 0 && nr % npix == 0 && nr == nb * rpb &&
        (c.march->flags & RM_MARCH_NATURAL_ORDER) == 0) {
      if ((rc = ensure_block_order(ctx, c.W / 16, c.H / 16, 256 / rpb)) != RM_OK) return rc;
      a.block_order = ctx->block_order;
      a.order_views = (int)(nr / npix);
      a.order_tiles = (int)(npix / rpb);
    }
    // cost-ordered dispatch from the previous launch over the same views (single-launch calls)
    const bool has_rec = c.mode == kBwd || c.mode == kTrain;
    unsigned long long key = 0;
    if (a.block_order != nullptr && has_rec && nb == blocks_left && done == 0 &&
        (c.march->flags & RM_MARCH_STATIC_ORDER) == 0) {
      key = ((unsigned long long)c.W << 48) ^ ((unsigned long long)c.H << 32) ^ ((unsigned long long)c.views << 24) ^
            ((unsigned long long)Mpad << 1) ^ 1ull ^ ((unsigned long long)split << 2);
      constexpr int kCls = RM_ORDER_CLASSES;
      if (!ctx->olist) {
        RM_HIP(ctx, hipMalloc(&ctx->olist, sizeof(int) * 3 * kCls * kMaxBlocksPerLaunch));
        // the three sets' counts, then the turn word, RM_ORDER_CNT_STRIDE ints apart
        RM_HIP(ctx, hipMalloc(&ctx->ocnt, sizeof(int) * 4 * RM_ORDER_CNT_STRIDE));
        RM_HIP(ctx, hipMemsetAsync(ctx->ocnt, 0, sizeof(int) * 4 * RM_ORDER_CNT_STRIDE, ctx->stream));
        ctx->oturn = ctx->ocnt + 3 * RM_ORDER_CNT_STRIDE;
      }
      // three list sets in rotation: the previous launch's (read), this launch's (appended;
      // cleared by the previous launch) and the next launch's (cleared by this one); which is which
      // the kernel reads from the device turn word, advanced by this call's reduction (order_sets)
      if (ctx->cost_valid && ctx->cost_key == key) {
        a.olist_r = ctx->olist;
        a.ocnt_r = ctx->ocnt;
      }
      a.olist_w = ctx->olist;
      a.ocnt_w = ctx->ocnt;
      a.ocnt_z = ctx->ocnt;
      a.oturn = ctx->oturn;
      if (const char* e = std::getenv("RM_DEBUG_SKIP_ORDER_CLEAR"))  // recovery test (rm_debug_order_counts)
        if (e[0] == '1') a.ocnt_z = nullptr;
    }
    if (has_rec) {
      ctx->cost_valid = key != 0;
      ctx->cost_key = key;
    }
    if (nb > 0 && a.cull) {
      if (!ctx->esc_flags) RM_HIP(ctx, hipMalloc(&ctx->esc_flags, sizeof(int) * kMaxBlocksPerLaunch));
      const dim3 g((unsigned)nb);
      if (c.mode == kFwd) launch_escape<kFwd>(c.cam, g, ctx->stream, a, ctx->esc_flags);
      else if (c.mode == kBwd) launch_escape<kBwd>(c.cam, g, ctx->stream, a, ctx->esc_flags);
      else if (c.mode == kTrain) launch_escape<kTrain>(c.cam, g, ctx->stream, a, ctx->esc_flags);
      else launch_escape<kRender>(c.cam, g, ctx->stream, a, ctx->esc_flags);
      RM_HIP(ctx, hipGetLastError());
      a.esc_flags = ctx->esc_flags;
    }
    if (nb > 0) {
      hipEvent_t ev0, ev1;
      if ((rc = next_events(ctx, ev0, ev1)) != RM_OK) return rc;
      dim3 grid((unsigned)nb);
#ifdef RM_BLOCK_TRACE
      if (!ctx->btrace)
        RM_HIP(ctx, hipMalloc(&ctx->btrace, sizeof(unsigned long long) * kTraceWords * kWaves * (size_t)kMaxBlocksPerLaunch));
      a.btrace = ctx->btrace;
      ctx->btrace_waves = nb * kWaves;
#endif
      // Split continuation (bwd / train launches with the early exit): the blocks still marching
      // at step cont_steps stop there, and a second launch runs just those from their saved
      // state, dispatched one after another at its front -- spread evenly over the CUs, where the
      // first launch placed them by a cost order that only partly predicts which 64-ray groups
      // march every step. Bit-identical to one launch (tests/test_gpu_split.py).
      // continuations at increasing steps (split_cont_caps): launch k resumes the blocks the
      // previous launch deferred (list k % 2) and defers, at the next step of the list, into list
      // (k + 1) % 2, whose counts are cleared before it runs
      int caps[kMaxCont + 1];
      const int ncaps = split_cont_caps(a.steps, caps);
      const bool cont = split && c.mode != kRender && c.mode != kFwd && a.early_exit && ncaps > 0 &&
                        a.steps >= 2 * caps[0];
      int* lists[2] = {nullptr, nullptr};
      int* counts[2] = {nullptr, nullptr};
      const bool rmode = cont && a.ray_mode;
      int* rlists[2] = {nullptr, nullptr};
      int* rcounts[2] = {nullptr, nullptr};
      if (cont) {
        const long long rays = nb * kSplitRays;
        // per ray: 7 state rows (8 in ray mode), per group 2 words; the group lists; ray mode: two
        // ray lists of up to `rays` entries and their counts
        const size_t need = (size_t)(8 * rays + 2 * nb) * sizeof(float) +
                            (size_t)(2 * kContClasses * nb + 2 * kContClasses + 16) * sizeof(int) +
                            (size_t)(2 * rays + 16) * sizeof(int);
        if (ctx->cont_bytes < need) {
          if (ctx->cont_buf) RM_HIP(ctx, hipFree(ctx->cont_buf));
          ctx->cont_buf = nullptr;
          ctx->cont_bytes = 0;
          RM_HIP(ctx, hipMalloc(&ctx->cont_buf, need));
          ctx->cont_bytes = need;
        }
        lists[0] = reinterpret_cast<int*>(ctx->cont_buf + 8 * rays + 2 * nb);
        lists[1] = lists[0] + kContClasses * nb;
        counts[0] = lists[1] + kContClasses * nb;
        counts[1] = counts[0] + kContClasses;
        rcounts[0] = counts[1] + kContClasses;
        rcounts[1] = rcounts[0] + 8;  // a 32-byte line each
        rlists[0] = rcounts[1] + 8;
        rlists[1] = rlists[0] + rays;
        a.cont_state = ctx->cont_buf;
        a.cont_rays = rays;
        a.cont_list_w = lists[0];
        a.cont_count_w = counts[0];
        a.cont_cap = caps[0];
        a.cont_resume = 0;
        a.cont_stride = (int)nb;
        a.cont_order = env_is("RM_CONT_ORDER", '0') ? 0 : 1;
        RM_HIP(ctx, hipMemsetAsync(counts[0], 0, 2 * kContClasses * sizeof(int), ctx->stream));
        if (rmode) {  // the first launch appends the marching rays to ray list 0
          a.ray_list_w = rlists[0];
          a.ray_count_w = rcounts[0];
          RM_HIP(ctx, hipMemsetAsync(rcounts[0], 0, 16 * sizeof(int), ctx->stream));
        }
      }
      if (c.mode == kFwd) launch_ray<kFwd>(c.cam, split, grid, lds, ctx->stream, a, ev0, ev1);
      else if (c.mode == kBwd) launch_ray<kBwd>(c.cam, split, grid, lds, ctx->stream, a, ev0, ev1);
      else if (c.mode == kTrain) launch_ray<kTrain>(c.cam, split, grid, lds, ctx->stream, a, ev0, ev1);
      else launch_ray<kRender>(c.cam, false, grid, lds, ctx->stream, a, ev0, ev1);
      RM_HIP(ctx, hipGetLastError());
      // ray mode: continuation k marches the rays of ray list k % 2 (deferring at the next cap into
      // list (k + 1) % 2, whose count is cleared first: continuation k - 1 read it), then one resume
      // launch runs the deferred groups' post-march forward and backward from their final states
      for (int ph = 0; rmode && ph < ncaps; ++ph) {
        KArgs b = a;
        b.ray_cont = 1;
        b.cont_resume = caps[ph];
        b.cont_cap = caps[ph + 1];
        b.ray_list = rlists[ph & 1];
        b.ray_count = rcounts[ph & 1];
        b.ray_list_w = rlists[(ph + 1) & 1];
        b.ray_count_w = rcounts[(ph + 1) & 1];
        if (b.cont_cap > 0) RM_HIP(ctx, hipMemsetAsync(b.ray_count_w, 0, sizeof(int), ctx->stream));
        b.cont_list_w = nullptr;
        b.cont_count_w = nullptr;
        b.ocnt_z = nullptr;
        b.olist_r = nullptr;
        b.ocnt_r = nullptr;
        b.ocnt_w = nullptr;  // no groups of its own: the resume launch appends them
        b.olist_w = nullptr;
        hipEvent_t e0, e1;
        if ((rc = next_events(ctx, e0, e1)) != RM_OK) return rc;
        if (c.mode == kBwd) launch_cont<kBwd>(c.cam, grid, lds, ctx->stream, b, e0, e1);
        else launch_cont<kTrain>(c.cam, grid, lds, ctx->stream, b, e0, e1);
        RM_HIP(ctx, hipGetLastError());
      }
      if (rmode) {
        KArgs b = a;
        b.cont_resume = a.steps;
        b.cont_cap = 0;
        b.cont_list = lists[0];
        b.cont_count = counts[0];
        b.cont_list_w = nullptr;
        b.cont_count_w = nullptr;
        b.ray_list_w = nullptr;
        b.ray_count_w = nullptr;
        b.ocnt_z = nullptr;
        b.olist_r = nullptr;
        b.ocnt_r = nullptr;
        hipEvent_t e0, e1;
        if ((rc = next_events(ctx, e0, e1)) != RM_OK) return rc;
        if (c.mode == kBwd) launch_cont<kBwd>(c.cam, grid, lds, ctx->stream, b, e0, e1);
        else launch_cont<kTrain>(c.cam, grid, lds, ctx->stream, b, e0, e1);
        RM_HIP(ctx, hipGetLastError());
      }
    }
    if (has_bwd && (rc = reduce_and_finalize(ctx, c, a, nb, first, first && nb == blocks_left)) != RM_OK) return rc;
    done += nr;
    first = false;
  } while (done < n);
  return RM_OK;
}

}  // namespace

extern "C" {

#ifndef RM_SOURCE_SHA
#define RM_SOURCE_SHA "unknown"  // _build.py passes the sha256 of the kernel sources
#endif
const char* rm_version(void) { return "burn_raymarching_amd 0.1.0 (gfx950) src " RM_SOURCE_SHA; }

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

int rm_bind_step_scalars(rm_context* ctx, rm_step_scalars* dev) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->sdev = dev;
  return RM_OK;
}

int rm_set_stream(rm_context* ctx, void* stream) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->stream = static_cast<hipStream_t>(stream);
  return RM_OK;
}

int rm_timing_enable(rm_context* ctx, int32_t enable) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->timing = enable != 0;
  // pre-create a pool so event creation stays out of timed regions
  while (ctx->timing && ctx->events.size() < 256) {
    std::pair<hipEvent_t, hipEvent_t> pr;
    RM_HIP(ctx, hipEventCreate(&pr.first));
    RM_HIP(ctx, hipEventCreate(&pr.second));
    ctx->events.push_back(pr);
  }
  return RM_OK;
}

int rm_timing_collect(rm_context* ctx, double* total_ms, int64_t* launches, int32_t reset) {
  if (!ctx || !total_ms || !launches) return RM_ERR_INVALID_ARG;
  double acc = 0.0;
  for (size_t i = 0; i < ctx->events_used; ++i) {
    RM_HIP(ctx, hipEventSynchronize(ctx->events[i].second));
    float ms = 0.0f;
    RM_HIP(ctx, hipEventElapsedTime(&ms, ctx->events[i].first, ctx->events[i].second));
    acc += ms;
  }
  *total_ms = acc;
  *launches = (int64_t)ctx->events_used;
  if (reset) ctx->events_used = 0;
  return RM_OK;
}

int rm_debug_order_counts(rm_context* ctx, int32_t* counts, int32_t capacity, int32_t* classes, int32_t* next_set) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  constexpr int kCls = RM_ORDER_CLASSES;
  if (classes) *classes = kCls;
  if (counts && capacity < 3 * kCls) return fail(ctx, RM_ERR_INVALID_ARG, "counts needs %d entries", 3 * kCls);
  RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  std::vector<int> host(4 * RM_ORDER_CNT_STRIDE, 0);  // the sets' counts and the device turn word
  if (ctx->ocnt) RM_HIP(ctx, hipMemcpy(host.data(), ctx->ocnt, sizeof(int) * host.size(), hipMemcpyDeviceToHost));
  if (next_set) *next_set = host[3 * RM_ORDER_CNT_STRIDE];
  if (counts)
    for (int st = 0; st < 3; ++st)
      for (int c = 0; c < kCls; ++c) counts[st * kCls + c] = host[st * RM_ORDER_CNT_STRIDE + c * RM_ORDER_CLS_STRIDE];
  return RM_OK;
}

#ifdef RM_BLOCK_TRACE
// Measurement build only (not in include/raymarch.h): the per-wave records of the last per-ray
// launch, 4 x u64 per wave in launch order (see rm_ray_kernel). Synchronises the stream.
int rm_debug_block_trace(rm_context* ctx, unsigned long long* host, int64_t cap_waves, int64_t* n_waves) {
  if (!ctx || !host || !n_waves) return RM_ERR_INVALID_ARG;
  RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  const long long n = std::min<long long>(ctx->btrace_waves, cap_waves);
  *n_waves = n;
  if (n > 0) RM_HIP(ctx, hipMemcpy(host, ctx->btrace, sizeof(unsigned long long) * kTraceWords * n, hipMemcpyDeviceToHost));
  return RM_OK;
}
#endif

int rm_debug_stall(rm_context* ctx, int32_t max_ms) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (max_ms < 1 || max_ms > 600000) return fail(ctx, RM_ERR_INVALID_ARG, "max_ms %d out of [1, 600000]", max_ms);
  if (!ctx->stall_flag)
    RM_HIP(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->stall_flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
  __atomic_store_n(ctx->stall_flag, 0, __ATOMIC_RELEASE);
  int* dflag = nullptr;
  RM_HIP(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), ctx->stall_flag, 0));
  hipLaunchKernelGGL(rm::rm_stall_kernel, dim3(1), dim3(64), 0, ctx->stream, dflag,
                     (unsigned long long)max_ms * 100000ull);  // s_memrealtime: 100 MHz
  RM_HIP(ctx, hipGetLastError());
  return RM_OK;
}

int rm_debug_stall_release(rm_context* ctx) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (ctx->stall_flag) __atomic_store_n(ctx->stall_flag, 1, __ATOMIC_RELEASE);
  return RM_OK;
}

int rm_stats_enable(rm_context* ctx, int32_t enable) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (enable && !ctx->stats_dev) {
    RM_HIP(ctx, hipMalloc(&ctx->stats_dev, kStatsWords * sizeof(unsigned long long)));
    RM_HIP(ctx, hipMemsetAsync(ctx->stats_dev, 0, kStatsWords * sizeof(unsigned long long), ctx->stream));
    ctx->stats_blocks = 0;
    ctx->stats_waves = 0;
  } else if (!enable && ctx->stats_dev) {
    RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
    RM_HIP(ctx, hipFree(ctx->stats_dev));
    ctx->stats_dev = nullptr;
  }
  return RM_OK;
}

int rm_stats_collect(rm_context* ctx, rm_stats* out, int32_t reset) {
  if (!ctx || !out) return RM_ERR_INVALID_ARG;
  if (!ctx->stats_dev) return fail(ctx, RM_ERR_INVALID_ARG, "stats are not enabled");
  unsigned long long v[kStatsWords];
  RM_HIP(ctx, hipMemcpyAsync(v, ctx->stats_dev, sizeof v, hipMemcpyDeviceToHost, ctx->stream));
  RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
  out->blocks = ctx->stats_blocks;
  out->blocks_skipped = (int64_t)v[0];
  out->waves = ctx->stats_waves;
  out->waves_exited = (int64_t)v[1];
  out->steps_saved = (int64_t)v[2];
  out->seeded_rays = (int64_t)v[4];
  out->seeded_rays_a = (int64_t)v[5];
#ifdef RM_LANE_STATS
  std::fprintf(stderr, "RM_LANE_STATS escaped_lane_sweeps %llu\n", v[3]);
#endif
#ifdef RM_RAY_STATS
  std::fprintf(stderr, "RM_RAY_STATS needed_lane_steps %llu waves %lld steps_saved %llu after_cap_run %llu "
               "after_cap_packed %llu\n", v[3], (long long)ctx->stats_waves, v[2], v[6], v[7]);
#endif
  if (reset) {
    RM_HIP(ctx, hipMemsetAsync(ctx->stats_dev, 0, sizeof v, ctx->stream));
    ctx->stats_blocks = 0;
    ctx->stats_waves = 0;
  }
  return RM_OK;
}

void rm_destroy(rm_context* ctx) {
  if (!ctx) return;
  if (ctx->stall_flag) {  // a pending stall ends before its flag goes away
    __atomic_store_n(ctx->stall_flag, 1, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipHostFree(ctx->stall_flag);
  }
  if (ctx->stats_dev || ctx->esc_flags || ctx->rec || ctx->block_order || ctx->olist || ctx->cont_buf) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->stats_dev) (void)hipFree(ctx->stats_dev);
    if (ctx->esc_flags) (void)hipFree(ctx->esc_flags);
    if (ctx->block_order) (void)hipFree(ctx->block_order);
    if (ctx->olist) (void)hipFree(ctx->olist);
    if (ctx->cont_buf) (void)hipFree(ctx->cont_buf);
    if (ctx->ocnt) (void)hipFree(ctx->ocnt);
    if (ctx->rec) (void)hipFree(ctx->rec);
  }
  if (ctx->arrivals || ctx->red_arrivals || ctx->batch || ctx->cams_dev || ctx->opt_pre || ctx->opt_arrival) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->arrivals) (void)hipFree(ctx->arrivals);
    if (ctx->red_arrivals) (void)hipFree(ctx->red_arrivals);
    if (ctx->batch) (void)hipFree(ctx->batch);
    if (ctx->opt_pre) (void)hipFree(ctx->opt_pre);
    if (ctx->opt_arrival) (void)hipFree(ctx->opt_arrival);
    if (ctx->cams_dev) (void)hipFree(ctx->cams_dev);
    if (ctx->cams_pin) (void)hipHostFree(ctx->cams_pin);
    for (hipEvent_t& e : ctx->cam_ev)
      if (e) (void)hipEventDestroy(e);
  }
  for (auto& pr : ctx->events) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
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
  m->flags = 0;
}

int rm_reserve(rm_context* ctx, int64_t max_rays, int32_t max_spheres) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (max_rays < 0 || max_spheres < 1 || max_spheres > RM_MAX_SPHERES)
    return fail(ctx, RM_ERR_INVALID_ARG, "bad reserve sizes");
  // the small buffers the calls otherwise allocate on first use: the arrival counters of the
  // in-kernel reductions (zeroed) and the fused iteration's optimizer hand-off
  if (!ctx->arrivals) {
    RM_HIP(ctx, hipMalloc(&ctx->arrivals, 64));
    RM_HIP(ctx, hipMemsetAsync(ctx->arrivals, 0, 64, ctx->stream));
  }
  if (!ctx->red_arrivals) {
    RM_HIP(ctx, hipMalloc(&ctx->red_arrivals, sizeof(unsigned) * kRedArrivals));
    RM_HIP(ctx, hipMemsetAsync(ctx->red_arrivals, 0, sizeof(unsigned) * kRedArrivals, ctx->stream));
  }
  if (!ctx->opt_arrival) {
    RM_HIP(ctx, hipMalloc(&ctx->opt_arrival, 128));
    RM_HIP(ctx, hipMemsetAsync(ctx->opt_arrival, 0, 128, ctx->stream));
  }
  if (!ctx->opt_pre) RM_HIP(ctx, hipMalloc(&ctx->opt_pre, sizeof(float) * (4 * kOptPreStride + 2)));
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

int rm_render(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays, const float* centers,
              const float* colors, const float* radius, int32_t num_spheres, float* out) {
  rm_scene sc{centers, colors, radius, nullptr, nullptr, num_spheres};
  rm_march m;
  rm_march_default(&m);  // 40 steps, k = 32, eps 1e-4, exp(-10 d) (renderer.rs:17-19, :52)
  Call c;
  c.mode = kRender;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = num_rays;
  c.scene = &sc;
  c.march = &m;
  c.out = out;
  return run(ctx, c);
}

int rm_render_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width, int32_t height,
                     const float* centers, const float* colors, const float* radius, int32_t num_spheres,
                     float* out) {
  rm_scene sc{centers, colors, radius, nullptr, nullptr, num_spheres};
  rm_march m;
  rm_march_default(&m);
  Call c;
  c.mode = kRender;
  c.cam = true;
  c.cams = cams;
  c.views = num_views;
  c.W = width;
  c.H = height;
  c.scene = &sc;
  c.march = &m;
  c.out = out;
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
  ctx->opt_prepared = false;  // the parameters may have changed since a prepared step (see run)
  if (!raw_packed || !act_packed) return fail(ctx, RM_ERR_INVALID_ARG, "NULL packed buffer");
  if (num_spheres < 1 || num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  const int n = 7 * num_spheres + 4;
  hipLaunchKernelGGL(rm::rm_activate_kernel, dim3((n + 255) / 256), dim3(256), 0, ctx->stream, raw_packed,
                     num_spheres, act_packed);
  RM_HIP(ctx, hipGetLastError());
  return RM_OK;
}

int rm_gather_rays(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                   int64_t num_src, const int32_t* indices, int64_t num_rays, float* out_org, float* out_dir,
                   float* out_targets) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->opt_prepared = false;
  if (num_rays < 0 || num_src < 0) return fail(ctx, RM_ERR_INVALID_ARG, "negative size");
  if (num_rays == 0) return RM_OK;
  if (!indices) return fail(ctx, RM_ERR_INVALID_ARG, "indices is NULL");
  if ((out_org && !ray_org) || (out_dir && !ray_dir) || (out_targets && !targets))
    return fail(ctx, RM_ERR_INVALID_ARG, "an output is requested without its source array");
  if (!out_org && !out_dir && !out_targets) return fail(ctx, RM_ERR_INVALID_ARG, "no output requested");
  const long long nel = 3 * (long long)num_rays;
  hipLaunchKernelGGL(rm::rm_gather_kernel, dim3((unsigned)((nel + 255) / 256)), dim3(256), 0, ctx->stream, ray_org,
                     ray_dir, targets, (long long)num_src, indices, (long long)num_rays, out_org, out_dir,
                     out_targets);
  RM_HIP(ctx, hipGetLastError());
  return RM_OK;
}

}  // extern "C"

namespace {
// the sampler's per-call key: (seed, stream, counter) mixed on the host
unsigned long long sample_key(uint64_t seed, uint64_t stream, uint64_t counter) {
  auto mix = [](unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  return mix(mix(mix(seed) ^ stream) ^ counter);
}
}  // namespace

extern "C" {

int rm_sample_batch(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets, int64_t num_src,
                    const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg, uint64_t seed,
                    uint64_t stream, uint64_t counter, float* out_org, float* out_dir, float* out_targets,
                    int32_t* indices_out) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->opt_prepared = false;
  if (num_src < 0 || num_fg < 0 || n_uniform < 0 || n_fg < 0) return fail(ctx, RM_ERR_INVALID_ARG, "negative size");
  const long long n = n_uniform + n_fg;
  if (n == 0) return RM_OK;
  if (num_src == 0 || num_src > INT32_MAX) return fail(ctx, RM_ERR_INVALID_ARG, "num_src %lld out of [1, 2^31)", (long long)num_src);
  if (n_fg > 0 && (num_fg == 0 || !fg_indices)) return fail(ctx, RM_ERR_INVALID_ARG, "n_fg > 0 needs foreground indices");
  if ((out_org && !ray_org) || (out_dir && !ray_dir) || (out_targets && !targets))
    return fail(ctx, RM_ERR_INVALID_ARG, "an output is requested without its source array");
  if (!out_org && !out_dir && !out_targets && !indices_out) return fail(ctx, RM_ERR_INVALID_ARG, "no output requested");
  const unsigned long long key = sample_key(seed, stream, counter);
  hipLaunchKernelGGL(rm::rm_sample_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, ray_org, ray_dir,
                     targets, (long long)num_src, fg_indices, (long long)num_fg, (long long)n_uniform, n, key, out_org,
                     out_dir, out_targets, indices_out);
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

int rm_optimizer_step_f16(rm_context* ctx, float* raw_packed, const float* grad_act_packed, float* adam_m,
                          float* adam_v, int32_t num_spheres, int32_t step, float lr, float weight_decay,
                          int32_t with_penalties, float* loss_penalty, float* act_out, uint16_t* colors_f16_out) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (!raw_packed || !grad_act_packed || !adam_m || !adam_v)
    return fail(ctx, RM_ERR_INVALID_ARG, "NULL optimizer buffer");
  if (num_spheres < 1 || num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  if (step < 1 && !ctx->sdev) return fail(ctx, RM_ERR_INVALID_ARG, "step counts from 1");
  const int M = num_spheres;
  const int n = 7 * M + 4;
  const int nb = (n + 255) / 256;
  const bool prepared = ctx->opt_prepared && ctx->prep_raw == raw_packed && ctx->prep_M == M &&
                        ctx->prep_step == step && ctx->prep_pen == (with_penalties ? 1 : 0) &&
                        ctx->prep_loss_penalty == loss_penalty && !ctx->sdev;
  ctx->opt_prepared = false;
  if (prepared) {  // the gradient-independent part ran in the sampled launch (rm_train_step_sampled_prepared)
    hipLaunchKernelGGL(rm::rm_optimizer_post_small, dim3(1), dim3(256), 0, ctx->stream, raw_packed, grad_act_packed,
                       adam_m, adam_v, M, lr, weight_decay, act_out, reinterpret_cast<_Float16*>(colors_f16_out),
                       static_cast<const float*>(ctx->opt_pre));
    RM_HIP(ctx, hipGetLastError());
    return RM_OK;
  }
  if (M <= rm::kOptSmallMaxM && !env_is("RM_OPT_SMALL", '0')) {  // one block: snapshot, repulsion rows, update
    hipLaunchKernelGGL(rm::rm_optimizer_small, dim3(1), dim3(256), 0, ctx->stream, raw_packed, grad_act_packed, adam_m,
                       adam_v, M, step, lr, weight_decay, with_penalties ? 1 : 0, loss_penalty, act_out,
                       reinterpret_cast<_Float16*>(colors_f16_out), ctx->sdev);
    RM_HIP(ctx, hipGetLastError());
    return RM_OK;
  }
  // workspace: snapshot of the pre-step params | repulsion rows [M][4] | penalty partials
  const size_t need = ((size_t)n + 4 * (size_t)M + (size_t)nb + 64) * sizeof(float);
  int rc = ensure_ws(ctx, std::max(ctx->ws_bytes, need));
  if (rc != RM_OK) return rc;
  float* snap = static_cast<float*>(ctx->ws);
  float* pair = snap + n;
  float* parts = loss_penalty ? pair + 4 * M : nullptr;
  hipLaunchKernelGGL(rm::rm_penalty_pairs, dim3(M), dim3(256), 0, ctx->stream, raw_packed, M,
                     with_penalties ? 1 : 0, snap, pair);
  RM_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(rm::rm_optimizer_kernel, dim3(nb), dim3(256), 0, ctx->stream, snap, raw_packed,
                     grad_act_packed, adam_m, adam_v, pair, M, step, lr, weight_decay, with_penalties ? 1 : 0, parts,
                     act_out, reinterpret_cast<_Float16*>(colors_f16_out), ctx->sdev);
  RM_HIP(ctx, hipGetLastError());
  if (ctx->sdev) {
    hipLaunchKernelGGL(rm::rm_step_advance, dim3(1), dim3(64), 0, ctx->stream, ctx->sdev);
    RM_HIP(ctx, hipGetLastError());
  }
  if (loss_penalty) {
    hipLaunchKernelGGL(rm::rm_sum_small, dim3(1), dim3(64), 0, ctx->stream, parts, nb, loss_penalty);
    RM_HIP(ctx, hipGetLastError());
  }
  return RM_OK;
}

int rm_optimizer_step(rm_context* ctx, float* raw_packed, const float* grad_act_packed, float* adam_m,
                      float* adam_v, int32_t num_spheres, int32_t step, float lr, float weight_decay,
                      int32_t with_penalties, float* loss_penalty, float* act_out) {
  return rm_optimizer_step_f16(ctx, raw_packed, grad_act_packed, adam_m, adam_v, num_spheres, step, lr, weight_decay,
                               with_penalties, loss_penalty, act_out, nullptr);
}

int rm_train_step_camera_adam(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width,
                              int32_t height, const float* targets, float progress, float inv_count,
                              const rm_march* march, float* act_packed, float* grad_packed, float* raw_packed,
                              float* adam_m, float* adam_v, int32_t num_spheres, int32_t step, float lr,
                              float weight_decay, int32_t with_penalties, float* loss_sum, float* loss_penalty,
                              uint16_t* colors_f16_out) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->opt_prepared = false;
  if (!act_packed || !grad_packed || !raw_packed || !adam_m || !adam_v || !march)
    return fail(ctx, RM_ERR_INVALID_ARG, "NULL model buffer");
  if (num_spheres < 1 || num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  const bool f16 = (march->flags & RM_MARCH_COLOR_F16) != 0;
  if (f16 != (colors_f16_out != nullptr))
    return fail(ctx, RM_ERR_INVALID_ARG, "colors_f16_out goes with RM_MARCH_COLOR_F16 (and only with it)");
  if (step < 1 && !ctx->sdev) return fail(ctx, RM_ERR_INVALID_ARG, "step counts from 1");
  const int M = num_spheres;
  rm_scene sc;
  rm_scene_from_packed(act_packed, M, &sc);
  if (f16) sc.colors = reinterpret_cast<const float*>(colors_f16_out);  // the fp16 colours the step renders
  rm_grads gr;
  rm_grads_from_packed(grad_packed, M, &gr);
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
  c.scene = &sc;
  c.march = march;
  c.grads = &gr;
  c.loss_sum = loss_sum;
  c.accumulate = 0;
  const Call::Adam ad{raw_packed, adam_m, adam_v, act_packed, loss_penalty, reinterpret_cast<_Float16*>(colors_f16_out),
                      step, with_penalties ? 1 : 0, lr, weight_decay};
  c.adam = &ad;
  ctx->adam_done = false;
  int rc = run(ctx, c);
  const bool done = ctx->adam_done;
  ctx->adam_done = false;
  if (rc != RM_OK || done) return rc;
  // not fused (more than 64 spheres, the small-scene kernel, sub-launches): the optimizer call
  return rm_optimizer_step_f16(ctx, raw_packed, grad_packed, adam_m, adam_v, M, step, lr, weight_decay,
                               with_penalties, loss_penalty, act_packed, colors_f16_out);
}

}  // extern "C"

namespace {

// rm_sample_batch into the context's batch buffer, then rm_train_step on it: the separate-call
// form of the sampled step (rm_train_iteration's and rm_train_step_sampled's other sizes)
int sample_then_train(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                      int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg,
                      uint64_t seed, uint64_t stream, uint64_t counter, float progress, float inv_count,
                      const rm_scene* sc, const rm_march* march, const rm_grads* gr, float* loss_sum) {
  const long long n = n_uniform + n_fg;
  int rc;
  if (n > 0) {
    const size_t need = sizeof(float) * 9 * (size_t)n;
    if (need > ctx->batch_bytes) {
      if (ctx->batch) {
        RM_HIP(ctx, hipStreamSynchronize(ctx->stream));
        RM_HIP(ctx, hipFree(ctx->batch));
        ctx->batch = nullptr;
        ctx->batch_bytes = 0;
      }
      if (hipMalloc(&ctx->batch, need) != hipSuccess) return fail(ctx, RM_ERR_OOM, "batch buffer (%zu B)", need);
      ctx->batch_bytes = need;
    }
  }
  float* bo = ctx->batch;
  float* bd = bo ? bo + 3 * n : nullptr;
  float* bt = bo ? bo + 6 * n : nullptr;
  if (n > 0 && (rc = rm_sample_batch(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg, seed,
                                     stream, counter, bo, bd, bt, nullptr)) != RM_OK)
    return rc;
  return rm_train_step(ctx, bo, bd, bt, n, progress, inv_count, sc, march, gr, loss_sum, nullptr, 0);
}

// the sampled step's validation (rm_train_iteration and rm_train_step_sampled)
int check_sampling(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                   int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg) {
  if (!ray_org || !ray_dir || !targets) return fail(ctx, RM_ERR_INVALID_ARG, "NULL dataset array");
  if (num_src < 1 || num_src > INT32_MAX || n_uniform < 0 || n_fg < 0 || num_fg < 0)
    return fail(ctx, RM_ERR_INVALID_ARG, "bad sampling sizes");
  if (n_fg > 0 && (num_fg == 0 || !fg_indices)) return fail(ctx, RM_ERR_INVALID_ARG, "n_fg > 0 needs foreground indices");
  return RM_OK;
}

// one launch of the small-scene kernel with its in-kernel final reduction for this call
bool sampled_one_launch(const Call& c, int M, long long n) {
  const int rpb = kBlock / small_lpr(c, n);
  return use_small(c, M, n) && (n + rpb - 1) / rpb <= kSmallFinalMaxBlocks &&
         (n + rpb - 1) / rpb <= max_blocks_per_launch() && !env_is("RM_SMALL_FINAL", '0') &&
         !env_is("RM_FUSED_ITER", '0');
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {
// rm_train_step_sampled[_prepared]; raw_packed != nullptr: prepare the next optimizer step
int sampled_step(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets, int64_t num_src,
                 const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg, uint64_t seed,
                 uint64_t stream, uint64_t counter, float progress, float inv_count, const rm_scene* scene,
                 const rm_march* march, const rm_grads* grads, float* loss_sum, const float* raw_packed, int32_t step,
                 int32_t with_penalties, float* loss_penalty) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->opt_prepared = false;  // a preparation is for the optimizer call right after its own step
  int rc;
  if ((rc = check_sampling(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg)) != RM_OK)
    return rc;
  if (!scene || !march || !grads) return fail(ctx, RM_ERR_INVALID_ARG, "NULL scene / march / grads");
  if (scene->num_spheres < 1 || scene->num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  const long long n = n_uniform + n_fg;
  Call c;
  c.mode = kTrain;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = n;
  c.targets = targets;
  c.progress = progress;
  c.inv_count = inv_count;
  c.scene = scene;
  c.march = march;
  c.grads = grads;
  c.loss_sum = loss_sum;
  c.accumulate = 0;
  // one launch: the small kernel draws its rays and reduces the gradient in its last block
  if (n > 0 && sampled_one_launch(c, scene->num_spheres, n) && ctx->sdev == nullptr) {
    SmallArgs fz;
    std::memset(&fz, 0, sizeof fz);
    fz.src_org = ray_org;
    fz.src_dir = ray_dir;
    fz.src_tgt = targets;
    fz.fg = fg_indices;
    fz.num_src = num_src;
    fz.num_fg = num_fg;
    fz.n_uniform = n_uniform;
    fz.key = sample_key(seed, stream, counter);
    const int M = scene->num_spheres;
    const bool prep = raw_packed != nullptr && M <= kOptSmallMaxM && !env_is("RM_OPT_SMALL", '0') &&
                      !env_is("RM_OPT_PREPARE", '0');
    fz.adam = prep ? 2 : 0;
    if (prep) {  // the extra block: opt_small_pre of rm_optimizer_small on these parameters
      fz.raw = const_cast<float*>(raw_packed);
      fz.m1 = fz.m2 = const_cast<float*>(raw_packed);  // loaded with the parameters, not used
      fz.step = step;
      fz.with_pen = with_penalties ? 1 : 0;
      fz.loss_penalty = loss_penalty;
    }
    c.fused = &fz;
    rc = run(ctx, c);
    if (rc == RM_OK && prep) {
      ctx->opt_prepared = true;
      ctx->prep_raw = raw_packed;
      ctx->prep_loss_penalty = loss_penalty;
      ctx->prep_M = M;
      ctx->prep_step = step;
      ctx->prep_pen = with_penalties ? 1 : 0;
    }
    return rc;
  }
  return sample_then_train(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg, seed, stream,
                           counter, progress, inv_count, scene, march, grads, loss_sum);
}
}  // namespace

extern "C" {

int rm_train_step_sampled(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                          int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform,
                          int64_t n_fg, uint64_t seed, uint64_t stream, uint64_t counter, float progress,
                          float inv_count, const rm_scene* scene, const rm_march* march, const rm_grads* grads,
                          float* loss_sum) {
  return sampled_step(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg, seed, stream,
                      counter, progress, inv_count, scene, march, grads, loss_sum, nullptr, 0, 0, nullptr);
}

int rm_train_step_sampled_prepared(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                                   int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform,
                                   int64_t n_fg, uint64_t seed, uint64_t stream, uint64_t counter, float progress,
                                   float inv_count, const rm_scene* scene, const rm_march* march,
                                   const rm_grads* grads, float* loss_sum, const float* raw_packed, int32_t step,
                                   int32_t with_penalties, float* loss_penalty) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  if (!raw_packed) return fail(ctx, RM_ERR_INVALID_ARG, "NULL raw parameters");
  if (step < 1) return fail(ctx, RM_ERR_INVALID_ARG, "step counts from 1");
  if (ctx->sdev) return fail(ctx, RM_ERR_INVALID_ARG, "prepared steps do not take bound step scalars");
  return sampled_step(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg, seed, stream,
                      counter, progress, inv_count, scene, march, grads, loss_sum, raw_packed, step, with_penalties,
                      loss_penalty);
}

int rm_train_iteration(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                       int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg,
                       uint64_t seed, uint64_t stream, uint64_t counter, float progress, float inv_count,
                       const rm_march* march, float* act_packed, float* grad_packed, float* raw_packed,
                       float* adam_m, float* adam_v, int32_t num_spheres, int32_t step, float lr,
                       float weight_decay, int32_t with_penalties, float* loss_sum, float* loss_penalty) {
  if (!ctx) return RM_ERR_INVALID_ARG;
  ctx->opt_prepared = false;
  int rc;
  if ((rc = check_sampling(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg)) != RM_OK)
    return rc;
  if (!act_packed || !grad_packed || !raw_packed || !adam_m || !adam_v || !march)
    return fail(ctx, RM_ERR_INVALID_ARG, "NULL model buffer");
  if (num_spheres < 1 || num_spheres > RM_MAX_SPHERES) return fail(ctx, RM_ERR_INVALID_ARG, "bad num_spheres");
  if ((march->flags & RM_MARCH_COLOR_F16) != 0)
    return fail(ctx, RM_ERR_INVALID_ARG, "rm_train_iteration trains fp32 colour models");
  if (step < 1 && !ctx->sdev) return fail(ctx, RM_ERR_INVALID_ARG, "step counts from 1");
  const int M = num_spheres;
  const long long n = n_uniform + n_fg;
  rm_scene sc;
  rm_scene_from_packed(act_packed, M, &sc);
  rm_grads gr;
  rm_grads_from_packed(grad_packed, M, &gr);
  Call c;
  c.mode = kTrain;
  c.cam = false;
  c.org = ray_org;
  c.dir = ray_dir;
  c.n = n;
  c.targets = targets;
  c.progress = progress;
  c.inv_count = inv_count;
  c.scene = &sc;
  c.march = march;
  c.grads = &gr;
  c.loss_sum = loss_sum;
  c.accumulate = 0;
  // one launch: the small kernel with its in-kernel final reduction (RM_FUSED_ITER=0: three calls)
  const bool fused = sampled_one_launch(c, M, n) && M <= kOptSmallMaxM && ctx->sdev == nullptr;
  if (fused) {
    SmallArgs fz;
    std::memset(&fz, 0, sizeof fz);
    fz.src_org = ray_org;
    fz.src_dir = ray_dir;
    fz.src_tgt = targets;
    fz.fg = fg_indices;
    fz.num_src = num_src;
    fz.num_fg = num_fg;
    fz.n_uniform = n_uniform;
    fz.key = sample_key(seed, stream, counter);
    fz.raw = raw_packed;
    fz.m1 = adam_m;
    fz.m2 = adam_v;
    fz.step = step;
    fz.with_pen = with_penalties ? 1 : 0;
    fz.lr = lr;
    fz.wd = weight_decay;
    fz.loss_penalty = loss_penalty;
    fz.act_out = act_packed;
    fz.adam = 1;
    c.fused = &fz;
    return run(ctx, c);
  }
  // the same three steps as separate calls: draw + gather, train step, optimizer
  if ((rc = sample_then_train(ctx, ray_org, ray_dir, targets, num_src, fg_indices, num_fg, n_uniform, n_fg, seed,
                              stream, counter, progress, inv_count, &sc, march, &gr, loss_sum)) != RM_OK)
    return rc;
  return rm_optimizer_step(ctx, raw_packed, grad_packed, adam_m, adam_v, M, step, lr, weight_decay, with_penalties,
                           loss_penalty, act_packed);
}

}  // extern "C"
