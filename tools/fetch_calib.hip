// FETCH_SIZE / WRITE_SIZE calibration on known byte counts (MI355X_MICROARCH.md §HBM: the gfx950
// correction is known for 16 B/lane streams only; other widths must be calibrated in the kernel's
// own access pattern). The train kernel reads dword-wide (AoS float3 targets, one dword per lane
// per component; sphere tables) and stores dword-wide partial records, so this program streams a
// known number of bytes with each of those widths, plus the 16 B/lane case the guide documents:
//   read_dword   1 GiB, one float per lane per iteration (coalesced 256 B per wave instruction)
//   read_f3      1 GiB, AoS float3 per lane (three dword loads at stride 12 B, as the targets)
//   read_x4      1 GiB, one float4 per lane (the guide's calibrated case: FETCH = bytes / 2)
//   write_dword  256 MiB, one float per lane per iteration (as the partial records)
//   write_x4     256 MiB, one float4 per lane
//   write_rec    256 MiB of 8224-B records in the train kernel's pattern: a block writes its
//                record's 8 columns per sphere (coalesced dwords), then adds to columns 0-3
//                (4 of every 8 dwords, read-modify-write) -- counted once as unique bytes
// Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`; tools/fetch_calib.py
// turns the per-dispatch counters into bytes-per-counted-byte factors.
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

// the sums are stored only if they hit an impossible value: the loads cannot be removed, and the
// kernels write (almost) nothing
__global__ void read_dword(const float* __restrict__ a, long n, float* __restrict__ sink) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) s += a[i];
  if (s == -1.2345e30f) sink[threadIdx.x] = s;
}

__global__ void read_f3(const float* __restrict__ a, long n3, float* __restrict__ sink) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n3; i += (long)gridDim.x * blockDim.x)
    s += a[3 * i] + a[3 * i + 1] * 0.5f + a[3 * i + 2] * 0.25f;
  if (s == -1.2345e30f) sink[threadIdx.x] = s;
}

__global__ void read_x4(const float4* __restrict__ a, long n4, float* __restrict__ sink) {
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == -1.2345e30f) sink[threadIdx.x] = s;
}

__global__ void write_dword(float* __restrict__ a, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) a[i] = (float)i;
}

__global__ void write_x4(float4* __restrict__ a, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float f = (float)i;
    a[i] = make_float4(f, f + 1.f, f + 2.f, f + 3.f);
  }
}

constexpr int kRec = 2056;  // floats per record at 256 spheres (8 per sphere + 8 scalars)
__global__ void write_rec(float* __restrict__ a, long nrec) {
  for (long b = blockIdx.x; b < nrec; b += gridDim.x) {
    float* rec = a + b * kRec;
    for (int e = threadIdx.x; e < kRec; e += blockDim.x) rec[e] = (float)(b + e);
    __syncthreads();
    for (int e = threadIdx.x; e < (kRec - 8) / 2; e += blockDim.x) rec[(e >> 2) * 8 + (e & 3)] += 1.0f;
    __syncthreads();
  }
}

int main() {
  const long rbytes = 1L << 30, wbytes = 1L << 28;
  float *r, *w, *sink;
  CHECK(hipMalloc(&r, rbytes));
  CHECK(hipMalloc(&w, wbytes));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(r, 0, rbytes));
  const int grid = 4096, block = 256;
  const long nr = rbytes / 4, nw = wbytes / 4;
  hipLaunchKernelGGL(read_dword, dim3(grid), dim3(block), 0, 0, r, nr, sink);
  hipLaunchKernelGGL(read_f3, dim3(grid), dim3(block), 0, 0, r, nr / 3, sink);
  hipLaunchKernelGGL(read_x4, dim3(grid), dim3(block), 0, 0, (const float4*)r, nr / 4, sink);
  hipLaunchKernelGGL(write_dword, dim3(grid), dim3(block), 0, 0, w, nw);
  hipLaunchKernelGGL(write_x4, dim3(grid), dim3(block), 0, 0, (float4*)w, nw / 4);
  const long nrec = nw / kRec;
  hipLaunchKernelGGL(write_rec, dim3(grid), dim3(block), 0, 0, w, nrec);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  // the exact byte counts each dispatch moves (read_f3 covers 3 * floor(n / 3) floats)
  std::printf("{\"read_dword\": %ld, \"read_f3\": %ld, \"read_x4\": %ld, \"write_dword\": %ld, \"write_x4\": %ld, "
              "\"write_rec\": %ld}\n", rbytes, (nr / 3) * 3 * 4, rbytes, wbytes, wbytes, nrec * kRec * 4);
  CHECK(hipFree(r));
  CHECK(hipFree(w));
  CHECK(hipFree(sink));
  return 0;
}
