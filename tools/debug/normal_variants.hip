// Debug experiment: accuracy of fp32 6-tap finite-difference normals (scene.rs:81-128) on gfx950
// under different formulations. Reads points/spheres from argv files, writes normals per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
__device__ float softmin_sum(const float* q, const float* kr, int M, float nkappa, float& m) {
  return 0;
}
template <int V>
__global__ void k(const float* P, int n, const float* C, const float* R, int M, float k, float eps, float* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float p[3] = {P[3*i], P[3*i+1], P[3*i+2]};
  const float kappa = k * 1.4426950408889634f;
  float D[6];
  for (int t = 0; t < 6; ++t) {
    float tap[3] = {p[0], p[1], p[2]};
    int a = t / 2; float sg = (t & 1) ? -eps : eps;
    tap[a] = tap[a] + sg;
    float m = -INFINITY, s = 0;
    // two-pass exact max
    float vs[64];
    for (int j = 0; j < M; ++j) {
      float cx = C[3*j], cy = C[3*j+1], cz = C[3*j+2];
      float q;
      if (V == 0 || V == 1 || V == 3) {  // direct from p with analytic tap offset
        float ex = p[0]-cx, ey = p[1]-cy, ez = p[2]-cz;
        float Q = fmaf(ez, ez, fmaf(ey, ey, fmaf(ex, ex, eps*eps)));
        float e = a == 0 ? ex : (a == 1 ? ey : ez);
        q = fmaf(e, 2*sg, Q);
      } else {  // expansion at the tap point (reference form)
        float pp = tap[0]*tap[0] + tap[1]*tap[1] + tap[2]*tap[2];
        float cc = cx*cx + cy*cy + cz*cz;
        float pc = tap[0]*cx + tap[1]*cy + tap[2]*cz;
        q = (pp + cc) - pc * 2.0f;
      }
      q = fmaxf(q, 1e-6f);
      float rho = (V == 1 || V == 3) ? __fsqrt_rn(q) : __builtin_amdgcn_sqrtf(q);
      float v = (V == 3) ? (R[j] - rho) * (-k) * -1.0f : fmaf(rho, -kappa, kappa * R[j]);
      vs[j] = v; m = fmaxf(m, v);
    }
    for (int j = 0; j < M; ++j) s += (V == 3) ? expf(vs[j] - m) : __builtin_amdgcn_exp2f(vs[j] - m);
    D[t] = (V == 3) ? -(logf(s) + m) / k : -(__builtin_amdgcn_logf(s) + m) / kappa;
  }
  float nx = D[0]-D[1], ny = D[2]-D[3], nz = D[4]-D[5];
  float len = sqrtf(nx*nx + ny*ny + nz*nz + 1e-6f);
  out[3*i] = nx/len; out[3*i+1] = ny/len; out[3*i+2] = nz/len;
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb"); int n, M; float kk;
  fread(&n, 4, 1, f); fread(&M, 4, 1, f); fread(&kk, 4, 1, f);
  std::vector<float> P(3*n), C(3*M), R(M);
  fread(P.data(), 4, 3*n, f); fread(C.data(), 4, 3*M, f); fread(R.data(), 4, M, f); fclose(f);
  float *dP, *dC, *dR, *dO; hipMalloc(&dP, 12*n); hipMalloc(&dC, 12*M); hipMalloc(&dR, 4*M); hipMalloc(&dO, 12*n);
  hipMemcpy(dP, P.data(), 12*n, hipMemcpyHostToDevice); hipMemcpy(dC, C.data(), 12*M, hipMemcpyHostToDevice);
  hipMemcpy(dR, R.data(), 4*M, hipMemcpyHostToDevice);
  FILE* o = fopen(argv[2], "wb"); std::vector<float> O(3*n);
  for (int v = 0; v < 4; ++v) {
    if (v == 0) k<0><<<(n+255)/256, 256>>>(dP, n, dC, dR, M, kk, 1e-4f, dO);
    if (v == 1) k<1><<<(n+255)/256, 256>>>(dP, n, dC, dR, M, kk, 1e-4f, dO);
    if (v == 2) k<2><<<(n+255)/256, 256>>>(dP, n, dC, dR, M, kk, 1e-4f, dO);
    if (v == 3) k<3><<<(n+255)/256, 256>>>(dP, n, dC, dR, M, kk, 1e-4f, dO);
    hipMemcpy(O.data(), dO, 12*n, hipMemcpyDeviceToHost);
    fwrite(O.data(), 4, 3*n, o);
  }
  fclose(o); return 0;
}
