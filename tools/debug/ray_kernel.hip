// Debug: in-kernel camera_ray vs host-computed rays (correctly rounded ops).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include "../../burn_raymarching_amd/csrc/rm_device.h"
__global__ void k(rm::CamBasis c, int W, int H, float* d, float* dbg) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * H) return;
  float o[3], dd[3];
  rm::camera_ray(c, i % W, i / W, W, H, o, dd);
  d[3*i] = dd[0]; d[3*i+1] = dd[1]; d[3*i+2] = dd[2];
  float u = __fadd_rn(__fmul_rn(__fdiv_rn((float)(i % W), (float)W), 2.0f), -1.0f);
  dbg[2*i] = u; dbg[2*i+1] = __fsqrt_rn((float)i * 0.37f + 1.0f);
  if (i == 12) {
    const float v = -__fadd_rn(__fmul_rn(__fdiv_rn((float)(i / W), (float)H), 2.0f), -1.0f);
    const float rs = __fmul_rn(u, c.half_w), us = __fmul_rn(v, c.half_h);
    float dx = __fadd_rn(__fadd_rn(__fmul_rn(c.right[0], rs), __fmul_rn(c.up[0], us)), c.fwd[0]);
    float dy = __fadd_rn(__fadd_rn(__fmul_rn(c.right[1], rs), __fmul_rn(c.up[1], us)), c.fwd[1]);
    float dz = __fadd_rn(__fadd_rn(__fmul_rn(c.right[2], rs), __fmul_rn(c.up[2], us)), c.fwd[2]);
    const float ss = __fadd_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)), __fmul_rn(dz, dz));
    printf("dev: u %.9g v %.9g rs %.9g us %.9g dx %.9g dy %.9g dz %.9g ss %.9g len %.9g\n", u, v, rs, us, dx, dy, dz, ss, (float)__builtin_sqrt((double)ss));
  }
}
int main() {
  const int W = 40, H = 24;
  float eye[3] = {2.5f, 0.5f, 0.0f};
  rm::CamBasis b;
  float fr[3] = {-eye[0], -eye[1], -eye[2]};
  float len = std::sqrt(fr[0]*fr[0] + fr[1]*fr[1] + fr[2]*fr[2]);
  for (int i = 0; i < 3; ++i) b.fwd[i] = fr[i] / len;
  float up_w[3] = {0, 1, 0}, rr[3] = {b.fwd[1]*up_w[2] - b.fwd[2]*up_w[1], b.fwd[2]*up_w[0] - b.fwd[0]*up_w[2], b.fwd[0]*up_w[1] - b.fwd[1]*up_w[0]};
  len = std::sqrt(rr[0]*rr[0] + rr[1]*rr[1] + rr[2]*rr[2]);
  for (int i = 0; i < 3; ++i) b.right[i] = rr[i] / len;
  b.up[0] = b.right[1]*b.fwd[2] - b.right[2]*b.fwd[1]; b.up[1] = b.right[2]*b.fwd[0] - b.right[0]*b.fwd[2]; b.up[2] = b.right[0]*b.fwd[1] - b.right[1]*b.fwd[0];
  b.half_h = std::tan(50.0f * (3.14159265358979323846f / 180.0f) / 2.0f); b.half_w = ((float)W / (float)H) * b.half_h;
  for (int i = 0; i < 3; ++i) b.eye[i] = eye[i];
  float *dd, *dbg; hipMalloc(&dd, 12*W*H); hipMalloc(&dbg, 8*W*H);
  k<<<(W*H+255)/256, 256>>>(b, W, H, dd, dbg);
  std::vector<float> D(3*W*H), G(2*W*H);
  hipMemcpy(D.data(), dd, 12*W*H, hipMemcpyDeviceToHost); hipMemcpy(G.data(), dbg, 8*W*H, hipMemcpyDeviceToHost);
  int bad = 0, badu = 0, bads = 0;
  for (int i = 0; i < W*H; ++i) {
    int x = i % W, y = i / W;
    volatile float u = ((float)x / (float)W) * 2.0f - 1.0f;
    volatile float v = -(((float)y / (float)H) * 2.0f - 1.0f);
    volatile float rs = u * b.half_w, us = v * b.half_h;
    volatile float p0 = b.right[0] * rs; volatile float p1 = b.up[0] * us; volatile float dx = p0 + p1; dx = dx + b.fwd[0];
    p0 = b.right[1] * rs; p1 = b.up[1] * us; volatile float dy = p0 + p1; dy = dy + b.fwd[1];
    p0 = b.right[2] * rs; p1 = b.up[2] * us; volatile float dz = p0 + p1; dz = dz + b.fwd[2];
    volatile float s0 = dx*dx; volatile float s1 = dy*dy; volatile float s2 = dz*dz; volatile float ss = s0 + s1; ss = ss + s2;
    float l = std::sqrt((float)ss);
    if (i == 12) printf("host: u %.9g v %.9g rs %.9g us %.9g dx %.9g dy %.9g dz %.9g ss %.9g len %.9g\n", (float)u, (float)v, (float)rs, (float)us, (float)dx, (float)dy, (float)dz, (float)ss, l);
    float h[3] = {dx / l, dy / l, dz / l};
    if (G[2*i] != u) ++badu;
    if (G[2*i+1] != std::sqrt((float)i * 0.37f + 1.0f)) ++bads;
    for (int c = 0; c < 3; ++c) if (h[c] != D[3*i+c]) { if (bad < 5) printf("px %d c %d host %.9g dev %.9g\n", i, c, h[c], D[3*i+c]); ++bad; }
  }
  printf("mismatch dir comps %d, u %d, sqrt %d of %d\n", bad, badu, bads, W*H);
}
