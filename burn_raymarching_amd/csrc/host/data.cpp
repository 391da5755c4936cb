// librm_host.so, part 2: host-side data logic. Camera rays (camera.rs:30-90), the seeded
// RNG, SceneDataset (dataset.rs:4-82), prune_and_split (training.rs:87-238) and the initial
// model of train.rs:100-126. All f32 arithmetic is written in the reference's operation
// order and built with -ffp-contract=off, so results match the Rust program's f32 values.
#include <cmath>
#include <cstring>

#include "rmh_common.hpp"

using namespace rmh;

namespace {

void normalize3(const float v[3], float o[3]) {  // camera.rs:7-14
  const float len = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (len == 0.0f) {
    o[0] = o[1] = o[2] = 0.0f;
  } else {
    o[0] = v[0] / len;
    o[1] = v[1] / len;
    o[2] = v[2] / len;
  }
}

void cross3(const float a[3], const float b[3], float o[3]) {  // camera.rs:20-26
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

}  // namespace

struct rmh_dataset {
  int64_t num_pixels = 0;
  std::vector<int32_t> fg, bg;
};

extern "C" {

void rmh_camera_rays(int32_t width, int32_t height, const float eye[3], const float target[3], float fov_deg,
                     float* org, float* dir) {
  const float world_up[3] = {0.0f, 1.0f, 0.0f};
  const float fwd_raw[3] = {target[0] - eye[0], target[1] - eye[1], target[2] - eye[2]};
  float fwd[3], right_raw[3], right[3], up[3];
  normalize3(fwd_raw, fwd);
  cross3(fwd, world_up, right_raw);
  normalize3(right_raw, right);
  cross3(right, fwd, up);
  const float aspect = (float)width / (float)height;
  const float theta = fov_deg * ((float)M_PI / 180.0f) / 2.0f;  // f32::to_radians() / 2
  const float half_h = std::tan(theta);
  const float half_w = aspect * half_h;
  for (int32_t y = 0; y < height; ++y) {
    for (int32_t x = 0; x < width; ++x) {
      const float u = ((float)x / (float)width) * 2.0f - 1.0f;
      const float v = -(((float)y / (float)height) * 2.0f - 1.0f);
      const float rs = u * half_w, us = v * half_h;
      const float dx = right[0] * rs + up[0] * us + fwd[0];
      const float dy = right[1] * rs + up[1] * us + fwd[1];
      const float dz = right[2] * rs + up[2] * us + fwd[2];
      const float len = std::sqrt(dx * dx + dy * dy + dz * dz);
      const size_t i = ((size_t)y * width + x) * 3;
      dir[i] = dx / len;
      dir[i + 1] = dy / len;
      dir[i + 2] = dz / len;
      org[i] = eye[0];
      org[i + 1] = eye[1];
      org[i + 2] = eye[2];
    }
  }
}

void rmh_rng_seed(rmh_rng* rng, uint64_t seed, uint64_t stream) {
  rng->state = 0;
  rng->inc = (stream << 1u) | 1u;
  rmh_rng_u32(rng);
  rng->state += seed;
  rmh_rng_u32(rng);
}

uint32_t rmh_rng_u32(rmh_rng* rng) {
  const uint64_t old = rng->state;
  rng->state = old * 6364136223846793005ULL + rng->inc;
  const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
  const uint32_t rot = (uint32_t)(old >> 59u);
  return (xorshifted >> rot) | (xorshifted << ((-rot) & 31));
}

uint32_t rmh_rng_below(rmh_rng* rng, uint32_t n) {
  uint64_t m = (uint64_t)rmh_rng_u32(rng) * n;
  uint32_t l = (uint32_t)m;
  if (l < n) {
    const uint32_t t = (uint32_t)(-n) % n;
    while (l < t) {
      m = (uint64_t)rmh_rng_u32(rng) * n;
      l = (uint32_t)m;
    }
  }
  return (uint32_t)(m >> 32);
}

float rmh_rng_uniform(rmh_rng* rng, float lo, float hi) {
  const float u = (float)(rmh_rng_u32(rng) >> 8) * (1.0f / 16777216.0f);
  const float r = lo + (hi - lo) * u;
  return r < hi ? r : lo;  // keep the half-open range under rounding
}

int rmh_dataset_create(const float* targets, int64_t num_pixels, rmh_dataset** out) {
  if (!out || num_pixels < 0 || (num_pixels > 0 && !targets)) return fail(RMH_ERR_INVALID_ARG, "bad dataset args");
  if (num_pixels > INT32_MAX) return fail(RMH_ERR_INVALID_ARG, "more than 2^31 pixels (indices are i32)");
  auto* ds = new rmh_dataset;
  ds->num_pixels = num_pixels;
  for (int64_t i = 0; i < num_pixels; ++i) {
    const float s = targets[3 * i] + targets[3 * i + 1] + targets[3 * i + 2];  // dataset.rs:28
    (s > 0.05f ? ds->fg : ds->bg).push_back((int32_t)i);
  }
  *out = ds;
  return RMH_OK;
}

void rmh_dataset_destroy(rmh_dataset* ds) { delete ds; }

void rmh_dataset_counts(const rmh_dataset* ds, int64_t* num_fg, int64_t* num_bg) {
  if (num_fg) *num_fg = ds ? (int64_t)ds->fg.size() : 0;
  if (num_bg) *num_bg = ds ? (int64_t)ds->bg.size() : 0;
}

void rmh_dataset_sample_count(const rmh_dataset* ds, int32_t batch, float uniform_ratio, int64_t* n_uniform,
                              int64_t* n_fg) {
  // dataset.rs:54-61
  int64_t nu = (int64_t)((float)batch * uniform_ratio);
  if (nu < 0) nu = 0;
  if (nu > batch) nu = batch;
  int64_t nf = batch - nu;
  const int64_t fg = ds ? (int64_t)ds->fg.size() : 0;
  if (fg > 0 && fg < nf) {
    nf = fg;
    nu = batch - nf;
  }
  // dataset.rs:67: with no foreground pixel the boost draws are skipped and the batch is short
  if (fg == 0) nf = 0;
  if (n_uniform) *n_uniform = nu;
  if (n_fg) *n_fg = nf;
}

void rmh_dataset_fg(const rmh_dataset* ds, const int32_t** fg, int64_t* num_fg) {
  if (fg) *fg = ds && !ds->fg.empty() ? ds->fg.data() : nullptr;
  if (num_fg) *num_fg = ds ? (int64_t)ds->fg.size() : 0;
}

int rmh_dataset_sample(const rmh_dataset* ds, int32_t batch, float uniform_ratio, rmh_rng* rng, int32_t* indices,
                       int32_t* count) {
  if (!ds || !rng || !count || batch < 0 || (batch > 0 && !indices))
    return fail(RMH_ERR_INVALID_ARG, "bad sample args");
  if (ds->num_pixels == 0 && batch > 0) return fail(RMH_ERR_INVALID_ARG, "empty dataset");
  int64_t n_uniform = 0, n_fg = 0;
  rmh_dataset_sample_count(ds, batch, uniform_ratio, &n_uniform, &n_fg);
  const int64_t fg = (int64_t)ds->fg.size();
  int64_t k = 0;
  for (int64_t i = 0; i < n_uniform; ++i) indices[k++] = (int32_t)rmh_rng_below(rng, (uint32_t)ds->num_pixels);
  for (int64_t i = 0; i < n_fg; ++i) indices[k++] = ds->fg[rmh_rng_below(rng, (uint32_t)fg)];
  *count = (int32_t)k;
  return RMH_OK;
}

void rmh_initial_model(float* raw) {
  const int M = 7;
  std::memset(raw, 0, sizeof(float) * (7 * M + 4));
  const float dirs[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
  for (int i = 0; i < 6; ++i)
    for (int a = 0; a < 3; ++a) raw[3 * i + a] = dirs[i][a] * 0.1f;  // train.rs:111-124
  // colours raw 0, radius raw 0 (train.rs:104-105); centre 6 at the origin
  raw[7 * M + 0] = 0.0f;  // light_dir (0, 1, 0), train.rs:106
  raw[7 * M + 1] = 1.0f;
  raw[7 * M + 2] = 0.0f;
  raw[7 * M + 3] = -1.4f;  // ambient raw, train.rs:107
}

int rmh_prune_and_split(const float* raw, int32_t M, const float* init_centers, int32_t stage, int32_t stages,
                        rmh_rng* rng, float* out, int32_t* out_M) {
  return rmh_prune_and_split_ex(raw, M, init_centers, stage, stages, 1.0f, 0.05f, 0, rng, out, out_M);
}

int rmh_prune_and_split_ex(const float* raw, int32_t M, const float* init_centers, int32_t stage, int32_t stages,
                           float split_scale, float split_move, int32_t max_spheres, rmh_rng* rng, float* out,
                           int32_t* out_M) {
  if (!raw || !init_centers || !rng || !out || !out_M || M < 1 || stage < 0 || stages < 1 || !(split_scale >= 0.0f) ||
      !(split_move >= 0.0f) || max_spheres < 0)
    return fail(RMH_ERR_INVALID_ARG, "bad prune_and_split arguments");
  const float* cen = raw;
  const float* col = raw + 3 * M;
  const float* rad = raw + 6 * M;
  std::vector<float> nc, ncol, nr;
  for (int32_t i = 0; i < M; ++i) {
    const float r = softplus_f32(rad[i]);  // eval radius: softplus without +0.01 (training.rs:131)
    const float raw_radius = rad[i];
    const float cx = cen[3 * i], cy = cen[3 * i + 1], cz = cen[3 * i + 2];
    const float dx0 = cx - init_centers[3 * i], dy0 = cy - init_centers[3 * i + 1],
                dz0 = cz - init_centers[3 * i + 2];
    const float move_dist_sq = dx0 * dx0 + dy0 * dy0 + dz0 * dz0;
    const float rr = col[3 * i], rg = col[3 * i + 1], rb = col[3 * i + 2];
    const float er = sigmoid_f32(rr), eg = sigmoid_f32(rg), eb = sigmoid_f32(rb);
    if (r > 1.0f - (float)stage * 0.04f || r < 0.005f) continue;  // training.rs:167
    if (cx * cx + cy * cy + cz * cz > 1.44f) continue;             // training.rs:172-175
    if (er + eg + eb < 0.05f) continue;                            // training.rs:178
    auto keep = [&](float x, float y, float z, float rawr) {
      nc.insert(nc.end(), {x, y, z});
      ncol.insert(ncol.end(), {rr, rg, rb});
      nr.push_back(rawr);
    };
    if (stage < stages - 1) {
      // training.rs:185-188 (split_scale 1, split_move 0.05: the reference's f32 values exactly)
      const float split_threshold = split_scale * (0.25f * std::pow(0.65f, (float)stage));
      // the cap (growth runs): the two children plus every later sphere kept must still fit
      const bool fits = max_spheres == 0 || (int64_t)nr.size() + 2 + (M - 1 - i) <= (int64_t)max_spheres;
      if (r > split_threshold && move_dist_sq > split_move * split_move && fits) {
        // training.rs:192-222: random unit direction, children at +-r/2 with radius 0.8 r
        const float z = rmh_rng_uniform(rng, -1.0f, 1.0f);
        const float theta = rmh_rng_uniform(rng, 0.0f, 6.2831855f);
        const float r_xy = std::sqrt(1.0f - z * z);
        const float dx = r_xy * std::cos(theta), dy = r_xy * std::sin(theta), dz = z;
        const float offset = r * 0.5f;
        const float target_r = std::fmax(r * 0.8f, 0.01f);
        const float new_raw_r = std::log(std::fmax(std::exp(target_r) - 1.0f, 1e-6f));
        keep(cx + dx * offset, cy + dy * offset, cz + dz * offset, new_raw_r);
        keep(cx - dx * offset, cy - dy * offset, cz - dz * offset, new_raw_r);
        continue;
      }
    }
    keep(cx, cy, cz, raw_radius);
  }
  const int32_t N = (int32_t)nr.size();
  if (N == 0) return fail(RMH_ERR_INVALID_ARG, "prune_and_split removed every sphere");
  std::memcpy(out, nc.data(), sizeof(float) * 3 * N);
  std::memcpy(out + 3 * N, ncol.data(), sizeof(float) * 3 * N);
  std::memcpy(out + 6 * N, nr.data(), sizeof(float) * N);
  std::memcpy(out + 7 * N, raw + 7 * M, sizeof(float) * 4);  // light_dir, ambient carried over
  *out_M = N;
  return RMH_OK;
}

}  // extern "C"
