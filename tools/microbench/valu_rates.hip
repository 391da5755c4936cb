// VALU / transcendental issue-rate microbenchmark for gfx950 (MI355X).
//
// Purpose: price the instructions of the sphere-SDF inner loop (v_fma_f32,
// v_pk_fma_f32, v_sqrt_f32, v_exp_f32, v_log_f32, v_rcp_f32, v_max_f32 and a
// mixed fma+exp stream) so the render kernels' roofline uses measured, not
// assumed, per-eval costs. Each thread runs 8 independent chains of the
// instruction under test (inline asm, so the compiler cannot fold or fuse),
// the grid fills every SIMD 8 waves deep, and the result is reported as
// wave-instructions per cycle per CU at the measured wall time and as
// lane-ops per second chip-wide.
//
// Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

enum Op { OP_FMA, OP_PKFMA, OP_SQRT, OP_EXP, OP_LOG, OP_RCP, OP_MAX, OP_MIX_FMA4_EXP1, OP_MIX_FMA2_EXP1_SQRT1,
          OP_ADD, OP_MAX3, OP_PKADD, OP_RSQ, OP_MAXLIT, OP_COUNT };
static const char* kNames[OP_COUNT] = {
  "v_fma_f32", "v_pk_fma_f32", "v_sqrt_f32", "v_exp_f32", "v_log_f32", "v_rcp_f32", "v_max_f32",
  "mix 4 fma + 1 exp", "mix 2 fma + 1 exp + 1 sqrt", "v_add_f32", "v_max3_f32", "v_pk_add_f32", "v_rsq_f32",
  "v_max_f32 literal"};
// instructions per chain-step for each op (used to convert to per-instruction rates)
static const int kInstPerStep[OP_COUNT] = {1, 1, 1, 1, 1, 1, 1, 5, 4, 1, 1, 1, 1, 1};

template <int OP>
__global__ __launch_bounds__(256) void bench(float* out, int iters, float seed) {
  float a0 = seed + threadIdx.x * 1e-7f, a1 = a0 + 1e-3f, a2 = a0 + 2e-3f, a3 = a0 + 3e-3f;
  float a4 = a0 + 4e-3f, a5 = a0 + 5e-3f, a6 = a0 + 6e-3f, a7 = a0 + 7e-3f;
  float b = 0.999f, c = 1e-4f;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
  f2 pb = {b, b}, pc = {c, c};
  for (int i = 0; i < iters; ++i) {
#define R8(STMT) STMT(a0) STMT(a1) STMT(a2) STMT(a3) STMT(a4) STMT(a5) STMT(a6) STMT(a7)
    if constexpr (OP == OP_FMA) {
#define S(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
      R8(S)
#undef S
    } else if constexpr (OP == OP_PKFMA) {
#define S(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(pb), "v"(pc));
      S(p0) S(p1) S(p2) S(p3) S(p0) S(p1) S(p2) S(p3)
#undef S
    } else if constexpr (OP == OP_SQRT) {
#define S(x) asm volatile("v_sqrt_f32 %0, %0" : "+v"(x));
      R8(S)
#undef S
    } else if constexpr (OP == OP_EXP) {
#define S(x) asm volatile("v_exp_f32 %0, -%0" : "+v"(x));
      R8(S)
#undef S
    } else if constexpr (OP == OP_LOG) {
#define S(x) asm volatile("v_log_f32 %0, %0" : "+v"(x));
      R8(S)
#undef S
    } else if constexpr (OP == OP_RCP) {
#define S(x) asm volatile("v_rcp_f32 %0, %0" : "+v"(x));
      R8(S)
#undef S
    } else if constexpr (OP == OP_MAX) {
#define S(x) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(c));
      R8(S)
#undef S
    } else if constexpr (OP == OP_ADD) {
#define S(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(c));
      R8(S)
#undef S
    } else if constexpr (OP == OP_MAX3) {
#define S(x) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(x) : "v"(c), "v"(b));
      R8(S)
#undef S
    } else if constexpr (OP == OP_PKADD) {
#define S(x) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(pc));
      S(p0) S(p1) S(p2) S(p3) S(p0) S(p1) S(p2) S(p3)
#undef S
    } else if constexpr (OP == OP_RSQ) {
#define S(x) asm volatile("v_rsq_f32 %0, %0" : "+v"(x));
      R8(S)
#undef S
    } else if constexpr (OP == OP_MAXLIT) {
#define S(x) asm volatile("v_max_f32 %0, 0x358637bd, %0" : "+v"(x));
      R8(S)
#undef S
    } else if constexpr (OP == OP_MIX_FMA4_EXP1) {
#define S(x) asm volatile("v_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\tv_fma_f32 %0, %0, %1, %2\n\tv_exp_f32 %0, -%0" : "+v"(x) : "v"(b), "v"(c));
      R8(S)
#undef S
    } else if constexpr (OP == OP_MIX_FMA2_EXP1_SQRT1) {
#define S(x) asm volatile("v_fma_f32 %0, %0, %1, %2\n\tv_sqrt_f32 %0, %0\n\tv_fma_f32 %0, %0, %1, %2\n\tv_exp_f32 %0, -%0" : "+v"(x) : "v"(b), "v"(c));
      R8(S)
#undef S
    }
#undef R8
  }
  float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x + p2.y + p3.x + p3.y;
  if (r == 12345.678f) out[0] = r;  // keep live
}

template <int OP>
static double run(float* d_out, int blocks, int iters, hipEvent_t e0, hipEvent_t e1) {
  bench<OP><<<blocks, 256>>>(d_out, 16, 1.0f);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  bench<OP><<<blocks, 256>>>(d_out, iters, 1.0f);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  return ms;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const double clk_ghz = prop.clockRate / 1e6;
  printf("device %s, %d CUs, clockRate %.3f GHz\n", prop.gcnArchName, cus, clk_ghz);
  float* d_out;
  CHECK(hipMalloc(&d_out, 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks = cus * 8;  // 8 x 256 threads per CU = 32 waves/CU = 8 waves/SIMD
  const int iters = 16384;
  double ms[OP_COUNT];
  for (int op = 0; op < OP_COUNT; ++op) ms[op] = 1e30;
  // 5 interleaved rounds; keep the fastest (DVFS and warm-up noise only ever slow a run down)
  for (int round = 0; round < 5; ++round) {
    double t;
#define RUN(OPV) t = run<OPV>(d_out, blocks, iters, e0, e1); if (t < ms[OPV]) ms[OPV] = t;
    RUN(OP_FMA) RUN(OP_PKFMA) RUN(OP_SQRT) RUN(OP_EXP) RUN(OP_LOG) RUN(OP_RCP) RUN(OP_MAX)
    RUN(OP_MIX_FMA4_EXP1) RUN(OP_MIX_FMA2_EXP1_SQRT1) RUN(OP_ADD) RUN(OP_MAX3) RUN(OP_PKADD) RUN(OP_RSQ) RUN(OP_MAXLIT)
#undef RUN
  }
  printf("%-28s %10s %14s %18s %16s\n", "op", "ms", "lane-op/s", "wave-inst/clk/CU*", "cyc/wave-inst/SIMD*");
  for (int op = 0; op < OP_COUNT; ++op) {
    const double waves = (double)blocks * 4.0;
    const double wave_insts = waves * iters * 8.0 * kInstPerStep[op];
    const double lane_ops = wave_insts * 64.0 * ((op == OP_PKFMA || op == OP_PKADD) ? 2.0 : 1.0);
    const double sec = ms[op] * 1e-3;
    const double per_clk_cu = wave_insts / (sec * clk_ghz * 1e9) / cus;
    printf("%-28s %10.3f %14.4e %18.3f %16.3f\n", kNames[op], ms[op], lane_ops / sec, per_clk_cu,
           4.0 / per_clk_cu);
  }
  printf("* at the nominal clockRate; DVFS may hold the clock lower under load\n");
  return 0;
}
