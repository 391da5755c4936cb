// Lone-wave cost of the march's matrix-core loop (rm_kernels.hip lse_mfma) on gfx950.
//
// The C5 workload (4096 spheres, 128 steps, one view) ends with about one live wave per SIMD, and
// a wave alone runs the march ~3x slower than its issue cost (tools/block_trace.py,
// tools/gpu_pmc_lone.sh: 71 % of its cycles in SQ_WAIT_ANY). This kernel replays the loop
// (fragments of 256 row blocks = 288 KB, 4 MFMAs + 16 x (max, sqrt, exp, fma) per row block)
// standalone, one wave alone on the chip or 4 waves per SIMD everywhere, in variants that remove
// one ingredient at a time:
//   0 as in the kernel: A / w fragments from global memory one row block ahead
//   1 no loads: the same fragments every row block (registers)
//   2 loads + MFMA only (no sqrt / exp consume)
//   3 loads four row blocks ahead (a ring of four register slots, explicit waits)
//   4 fragments from LDS (nrb <= 64; staged once)
//   5 v_mfma_f32_32x32x16_bf16 tiles (2 K halves x 2 ray tiles per 32 spheres) instead of
//     16x16x32: half the MFMA issue per (sphere, ray) value
// and prints cycles per row block per wave (s_memtime) and wall time.
//
// Build: hipcc --offload-arch=gfx950 -O3 march_loop.hip -o march_loop ; run: ./march_loop [nrb] [steps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float qclamp(float q, float qmin) {
  return __int_as_float(max(__float_as_int(q), __float_as_int(qmin)));
}

template <int VAR>
__global__ __launch_bounds__(256) void march_loop(const uint4* __restrict__ At, const float* __restrict__ Wt, int nrb,
                                                  int steps, float* out, long long* cyc) {
  __shared__ uint4 sA[VAR == 4 ? 64 * 64 : 1];
  __shared__ float sW[VAR == 4 ? 64 * 32 : 1];
  const int lane = threadIdx.x & 63, g = lane >> 4;
  if constexpr (VAR == 4) {
    for (int e = threadIdx.x; e < nrb * 64; e += blockDim.x) sA[e] = At[e];
    for (int e = threadIdx.x; e < nrb * 32; e += blockDim.x) sW[e] = Wt[e];
    __syncthreads();
  }
  bf16x8 B[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    uint4 v = make_uint4(0x3F803F80u ^ (lane * 7 + cb), 0x3F803F80u, 0x3F803F80u + lane, 0x3F80u);
    B[cb] = __builtin_bit_cast(bf16x8, v);
  }
  const float QMIN = 1e-6f;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
  auto load_a = [&](int rb) {
    if constexpr (VAR == 4) return __builtin_bit_cast(bf16x8, sA[rb * 64 + lane]);
    return __builtin_bit_cast(bf16x8, At[rb * 64 + lane]);
  };
  auto load_w = [&](int rb) {
    if constexpr (VAR == 4) return *reinterpret_cast<const float4*>(sW + rb * 32 + 4 * g);
    return *reinterpret_cast<const float4*>(Wt + rb * 32 + 4 * g);
  };
  auto tile = [&](const bf16x8& A, f32x4 (&D)[4]) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) D[cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[cb], zero, 0, 0, 0);
  };
  auto consume = [&](const f32x4 (&D)[4], const float4& w) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      float q[4] = {D[cb].x, D[cb].y, D[cb].z, D[cb].w};
      const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        if constexpr (VAR == 2) {
          acc[cb] += q[v] * wv[v];
        } else {
          const float rho = __builtin_amdgcn_sqrtf(qclamp(q[v], QMIN));
          acc[cb] = fmaf(wv[v], __builtin_amdgcn_exp2f(-rho), acc[cb]);
        }
      }
    }
  };
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  long long t0 = __builtin_readcyclecounter();
  for (int st = 0; st < steps; ++st) {
    f32x4 D[4];
    if constexpr (VAR == 5) {
      // 32x32x16 tiles: per 32-sphere block two K halves x two 32-ray column tiles; a lane holds
      // 16 values per column tile (the same sqrt / exp / fma per value as the 16x16x32 loop)
      const f32x16 z16 = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f,
                          0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
      float acc2[2] = {0.0f, 0.0f};
      bf16x8 A0 = load_a(0), A1 = load_a(1);
      float4 wv4[4];
      for (int rb = 0; rb < nrb; rb += 2) {  // one 32-sphere block = two 16-sphere row blocks of data
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          f32x16 Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A0, B[2 * c], z16, 0, 0, 0);
          Dv = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A1, B[2 * c + 1], Dv, 0, 0, 0);
          if (c == 0) {
            const int rn = min(rb + 2, nrb - 2);
            A0 = load_a(rn);
            A1 = load_a(rn + 1);
#pragma unroll
            for (int u = 0; u < 4; ++u) wv4[u] = load_w(rb + (u >> 1));
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float4 w4 = wv4[r >> 2];
            const float wr = (r & 3) == 0 ? w4.x : ((r & 3) == 1 ? w4.y : ((r & 3) == 2 ? w4.z : w4.w));
            const float rho = __builtin_amdgcn_sqrtf(qclamp(Dv[r], QMIN));
            acc2[c] = fmaf(wr, __builtin_amdgcn_exp2f(-rho), acc2[c]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      acc[0] += acc2[0];
      acc[1] += acc2[1];
    } else if constexpr (VAR == 1) {
      const bf16x8 A = load_a(st & 1);
      const float4 w = load_w(st & 1);
      for (int rb = 0; rb < nrb; ++rb) {
        tile(A, D);
        __builtin_amdgcn_sched_barrier(0);
        consume(D, w);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (VAR == 3) {
      bf16x8 A0 = load_a(0), A1 = load_a(1), A2 = load_a(2), A3 = load_a(3);
      float4 w0 = load_w(0), w1 = load_w(1), w2 = load_w(2), w3 = load_w(3);
      for (int rb = 0; rb < nrb; rb += 4) {
        const int n0 = min(rb + 4, nrb - 1), n1 = min(rb + 5, nrb - 1), n2 = min(rb + 6, nrb - 1),
                  n3 = min(rb + 7, nrb - 1);
        tile(A0, D);
        consume(D, w0);
        A0 = load_a(n0);
        w0 = load_w(n0);
        __builtin_amdgcn_sched_barrier(0);
        tile(A1, D);
        consume(D, w1);
        A1 = load_a(n1);
        w1 = load_w(n1);
        __builtin_amdgcn_sched_barrier(0);
        tile(A2, D);
        consume(D, w2);
        A2 = load_a(n2);
        w2 = load_w(n2);
        __builtin_amdgcn_sched_barrier(0);
        tile(A3, D);
        consume(D, w3);
        A3 = load_a(n3);
        w3 = load_w(n3);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      bf16x8 A = load_a(0);
      float4 w = load_w(0);
      for (int rb = 0; rb < nrb; rb += 2) {
        tile(A, D);
        const bf16x8 A1 = load_a(rb + 1);
        const float4 w1 = load_w(rb + 1);
        __builtin_amdgcn_sched_barrier(0);
        consume(D, w);
        __builtin_amdgcn_sched_barrier(0);
        tile(A1, D);
        const int rn = min(rb + 2, nrb - 1);
        A = load_a(rn);
        w = load_w(rn);
        __builtin_amdgcn_sched_barrier(0);
        consume(D, w1);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  long long t1 = __builtin_readcyclecounter();
  const float r = acc[0] + acc[1] + acc[2] + acc[3];
  if (r == 1234.5f) out[0] = r;  // keep the work
  if (lane == 0 && blockIdx.x == 0 && threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int VAR>
void run(const uint4* At, const float* Wt, int nrb, int steps, float* out, long long* cyc, int blocks, int threads) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(march_loop<VAR>, dim3(blocks), dim3(threads), 0, 0, At, Wt, nrb, 1, out, cyc);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(march_loop<VAR>, dim3(blocks), dim3(threads), 0, 0, At, Wt, nrb, steps, out, cyc);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  long long c = 0;
  CHECK(hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost));
  printf("variant %d  blocks %5d x %3d threads  nrb %3d  steps %3d: %9.3f ms  %8.1f cycles/row block (wave 0, "
         "s_memtime)  %8.1f ns/row block (wall)\n",
         VAR, blocks, threads, nrb, steps, ms, (double)c / ((double)nrb * steps), ms * 1e6 / ((double)nrb * steps));
}

int main(int argc, char** argv) {
  const int nrb = argc > 1 ? atoi(argv[1]) : 256;
  const int steps = argc > 2 ? atoi(argv[2]) : 16;
  std::vector<uint32_t> a((size_t)nrb * 64 * 4);
  std::vector<float> w((size_t)nrb * 32);
  for (size_t i = 0; i < a.size(); ++i) a[i] = 0x3C003C00u + (uint32_t)(i * 2654435761u % 512u);
  for (size_t i = 0; i < w.size(); ++i) w[i] = 1.0f + (float)(i % 7) * 0.01f;
  uint4* At;
  float* Wt;
  float* out;
  long long* cyc;
  CHECK(hipMalloc(&At, a.size() * 4));
  CHECK(hipMalloc(&Wt, w.size() * 4));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMalloc(&cyc, 64));
  CHECK(hipMemcpy(At, a.data(), a.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(Wt, w.data(), w.size() * 4, hipMemcpyHostToDevice));
  for (int cfg = 0; cfg < 3; ++cfg) {
    // one wave on the chip / one wave per SIMD on 16 CUs (the C5 tail) / 4 waves per SIMD everywhere
    const int blocks = cfg == 0 ? 1 : (cfg == 1 ? 16 : 1024), threads = cfg == 0 ? 64 : 256;
    run<0>(At, Wt, nrb, steps, out, cyc, blocks, threads);
    run<1>(At, Wt, nrb, steps, out, cyc, blocks, threads);
    run<2>(At, Wt, nrb, steps, out, cyc, blocks, threads);
    run<3>(At, Wt, nrb, steps, out, cyc, blocks, threads);
    if (nrb <= 64) run<4>(At, Wt, nrb, steps, out, cyc, blocks, threads);
    run<5>(At, Wt, nrb, steps, out, cyc, blocks, threads);
  }
  return 0;
}
