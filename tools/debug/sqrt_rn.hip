// Debug: which device sqrt / div spellings are correctly rounded on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
__global__ void k(const float* x, const float* y, float* o, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = x[i], b = y[i];
  o[8*i+0] = __fsqrt_rn(a);
  o[8*i+1] = sqrtf(a);
  o[8*i+2] = __builtin_sqrtf(a);
  o[8*i+3] = (float)sqrt((double)a);
  o[8*i+4] = __fdiv_rn(a, b);
  o[8*i+5] = a / b;
  o[8*i+6] = (float)((double)a / (double)b);
  o[8*i+7] = (float)__builtin_sqrt((double)a);
}
int main() {
  const int n = 1 << 20;
  std::vector<float> X(n), Y(n), O(8*n);
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) { s = s * 1664525u + 1013904223u; X[i] = 1.0f + (s >> 8) * (0.6f / (1 << 24)); s = s * 1664525u + 1013904223u; Y[i] = 0.5f + (s >> 8) * (2.0f / (1 << 24)); }
  float *dx, *dy, *dO; hipMalloc(&dx, 4*n); hipMalloc(&dy, 4*n); hipMalloc(&dO, 32*n);
  hipMemcpy(dx, X.data(), 4*n, hipMemcpyHostToDevice); hipMemcpy(dy, Y.data(), 4*n, hipMemcpyHostToDevice);
  k<<<n/256, 256>>>(dx, dy, dO, n);
  hipMemcpy(O.data(), dO, 32*n, hipMemcpyDeviceToHost);
  const char* names[8] = {"__fsqrt_rn", "sqrtf", "__builtin_sqrtf", "(float)sqrt(double)", "__fdiv_rn", "a/b", "(float)(double div)", "(float)__builtin_sqrt(double)"};
  for (int v = 0; v < 8; ++v) {
    int bad = 0;
    for (int i = 0; i < n; ++i) {
      float ref = (v < 4 || v == 7) ? std::sqrt(X[i]) : X[i] / Y[i];
      if (O[8*i+v] != ref) ++bad;
    }
    printf("%-22s mismatches %d / %d\n", names[v], bad, n);
  }
}
