// librm_host.so, part 3: the GPU-driving programs of the reference, over the C ABI of
// libraymarch_hip.so: the multi-stage training driver (train.rs:23-330), the preview
// (train.rs:335-366) and the target generator (generate.rs:20-112).
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>

#include "raymarch.h"
#include "rmh_common.hpp"

using namespace rmh;

namespace {

#define HIPCHK(call)                                                                            \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) return fail(RMH_ERR_GPU, "%s: %s", #call, hipGetErrorString(e_));     \
  } while (0)

#define RMCHK(ctx, call)                                                                        \
  do {                                                                                          \
    int r_ = (call);                                                                            \
    if (r_ != RM_OK) return fail(RMH_ERR_GPU, "%s: %s", #call, rm_last_error(ctx));             \
  } while (0)

// Device buffer owned by the host driver.
// Page-locked host memory (the loss readback: an async copy the stream wait then covers)
struct PinnedBuf {
  void* p = nullptr;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t alloc(size_t n) { return hipHostMalloc(&p, n, hipHostMallocDefault); }
  float* f() const { return (float*)p; }
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t alloc(size_t n) {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = n;
    return hipMalloc(&p, n ? n : 4);
  }
  float* f() const { return (float*)p; }
  int32_t* i() const { return (int32_t*)p; }
};

// A rank that leaves rmh_train with an error releases its side of the collectives
// (rmh_collective.abort: the RCCL one aborts its communicator). The other ranks learn of it through
// their own watchdog (rmh_collective.wait at every synchronisation point of the driver) or from
// the launcher, which ends the remaining ranks when one fails.
struct AbortOnError {
  const rmh_collective* comm = nullptr;
  bool done = false;
  ~AbortOnError() {
    if (!done && comm && comm->world > 1 && comm->abort) comm->abort(comm->state);
  }
};

// One rm_context + stream for a driver call.
struct Gpu {
  hipStream_t stream = nullptr;
  rm_context* ctx = nullptr;
  ~Gpu() {
    if (ctx) rm_destroy(ctx);
    if (stream) (void)hipStreamDestroy(stream);
  }
  int open(int device) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    if (rm_create(device, stream, &ctx) != RM_OK) return fail(RMH_ERR_GPU, "rm_create(device %d) failed", device);
    return RMH_OK;
  }
};

// Training steps a rank enqueues ahead of the GPU when it runs with collectives (rmh_train).
constexpr int32_t kStepsInFlight = 32;

// Waits for the driver's stream: through the collective's watchdog when collectives may be in
// flight (a dead peer then ends in an error instead of a hang), else hipStreamSynchronize.
int sync_stream(const Gpu& g, const rmh_collective* comm) {
  if (comm && comm->wait) {
    const int rc = comm->wait(comm->state, g.stream);
    if (rc != RMH_OK) {
      const std::string why = rmh_last_error();
      return fail(rc, "waiting for the stream: %s", why.c_str());
    }
    return RMH_OK;
  }
  HIPCHK(hipStreamSynchronize(g.stream));
  return RMH_OK;
}

// IEEE binary16, round to nearest even (the conversion torch's .half() and the optimizer's
// colors_f16_out use), for the initial fp16 colours of a stage.
uint16_t f32_to_f16(float x) {
  uint32_t u;
  std::memcpy(&u, &x, 4);
  const uint32_t sign = (u >> 16) & 0x8000u;
  const uint32_t ax = u & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u));  // inf / nan
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds past 65504: inf
  if (ax < 0x38800000u) {  // subnormal half (or zero): scale by 2^24 and round
    float a;
    std::memcpy(&a, &ax, 4);
    return (uint16_t)(sign | (uint32_t)std::nearbyint(a * 16777216.0f));
  }
  const uint32_t mant = ax & 0x7fffffu;
  uint32_t h = ((ax >> 23) - 112u) << 10 | (mant >> 13);
  const uint32_t rest = mant & 0x1fffu;
  if (rest > 0x1000u || (rest == 0x1000u && (h & 1u))) ++h;  // carries into the exponent correctly
  return (uint16_t)(sign | h);
}

bool file_exists(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "rb");
  if (!f) return false;
  std::fclose(f);
  return true;
}

// cameras.json names files relative to the reference's working directory ("data/target_0.png");
// try that, then relative to the json's directory, then the bare file name next to the json.
std::string resolve_image(const std::string& json_path, const std::string& file) {
  if (file_exists(file)) return file;
  const std::string dir = dirname_of(json_path);
  const std::string a = join_path(dir, file);
  if (file_exists(a)) return a;
  const size_t s = file.rfind('/');
  return join_path(dir, s == std::string::npos ? file : file.substr(s + 1));
}

void camera_struct(rm_camera& c, const float eye[3], const float target[3], float fov) {
  for (int k = 0; k < 3; ++k) {
    c.eye[k] = eye[k];
    c.target[k] = target[k];
  }
  c.fov_deg = fov;
}

// save_tiled_preview (train.rs:335-366): render_diff at k = 32 of the activated packed model,
// whole image in one camera-mode launch (the reference chunks 4096 rays only to save VRAM).
int preview_packed(Gpu& g, const float* act_dev, const uint16_t* colors_f16, int32_t M, int32_t W, int32_t H,
                   int32_t steps, const std::string& path) {
  rm_scene sc;
  rm_scene_from_packed(act_dev, M, &sc);
  rm_march m;
  rm_march_default(&m);
  m.steps = steps;
  if (colors_f16) {  // an fp16-colour model previews with the colours it trains with
    sc.colors = (const float*)colors_f16;
    m.flags |= RM_MARCH_COLOR_F16;
  }
  m.smooth_k = 32.0f;
  rm_camera cam;
  const float eye[3] = {0.0f, 0.0f, -2.5f}, tgt[3] = {0.0f, 0.0f, 0.0f};  // train.rs:37-44
  camera_struct(cam, eye, tgt, 50.0f);
  DevBuf out;
  HIPCHK(out.alloc(sizeof(float) * 3 * (size_t)W * H));
  RMCHK(g.ctx, rm_render_diff_camera(g.ctx, &cam, 1, W, H, &sc, &m, out.f(), nullptr));
  std::vector<float> host(3 * (size_t)W * H);
  HIPCHK(hipMemcpyAsync(host.data(), out.p, out.bytes, hipMemcpyDeviceToHost, g.stream));
  HIPCHK(hipStreamSynchronize(g.stream));
  return rmh_image_save(path.c_str(), host.data(), W, H);
}

// train.rs:210-262: centers raw, colours sigmoid, radii softplus (no +0.01), light raw,
// ambient sigmoid.
int export_scene(const std::vector<float>& raw, int32_t M, const std::string& path) {
  std::vector<float> col(3 * (size_t)M), rad(M);
  for (int32_t i = 0; i < 3 * M; ++i) col[i] = sigmoid_f32(raw[3 * M + i]);
  for (int32_t i = 0; i < M; ++i) rad[i] = softplus_f32(raw[6 * M + i]);
  const float amb = sigmoid_f32(raw[7 * M + 3]);
  return rmh_scene_save(path.c_str(), M, raw.data(), col.data(), rad.data(), raw.data() + 7 * M, &amb);
}

}  // namespace

extern "C" {

void rmh_train_config_default(rmh_train_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof *c);
  c->cameras_json = "data/cameras.json";
  c->out_dir = ".";
  c->width = 256;
  c->height = 256;
  c->stages = 5;
  c->steps_per_stage = 700;
  c->batch = 16384;
  c->march_steps = 40;
  c->max_smooth = 32.0f;
  c->base_lr = 0.05f;
  c->weight_decay = 1e-5f;
  c->log_every = 100;
  c->previews = 1;
  c->seed = 0;
  c->device = 0;
  c->split_scale = 1.0f;   // training.rs:185
  c->split_move = 0.05f;   // training.rs:188
}

int rmh_train(const rmh_train_config* cfg, rmh_train_result* result, float* raw_out, int32_t raw_capacity) {
  if (!cfg || !cfg->cameras_json) return fail(RMH_ERR_INVALID_ARG, "NULL config");
  if (cfg->width < 1 || cfg->height < 1 || cfg->stages < 1 || cfg->steps_per_stage < 1 || cfg->batch < 1 ||
      cfg->march_steps < 1 || std::isnan(cfg->split_scale) || std::isnan(cfg->split_move) || cfg->max_spheres < 0)
    return fail(RMH_ERR_INVALID_ARG, "bad training configuration");
  const bool f16 = cfg->color_f16 != 0;
  // the growth knobs: 0 (a zeroed struct) = the reference's value, < 0 = no such condition
  // (rmh_prune_and_split_ex takes 0 for that) -- ADVICE r04: a zeroed config is the reference rule
  const float split_scale = cfg->split_scale == 0.0f ? 1.0f : std::max(cfg->split_scale, 0.0f);
  const float split_move = cfg->split_move == 0.0f ? 0.05f : std::max(cfg->split_move, 0.0f);
  const int32_t W = cfg->width, H = cfg->height;
  const rmh_collective* comm = cfg->comm;
  const int32_t world = comm ? comm->world : 1, rank = comm ? comm->rank : 0;
  if (world < 1 || rank < 0 || rank >= world || (world > 1 && (!comm->all_reduce_sum || !comm->broadcast)))
    return fail(RMH_ERR_INVALID_ARG, "bad collective (rank %d of %d)", rank, world);
  if (cfg->batch < world) return fail(RMH_ERR_INVALID_ARG, "batch %d < %d ranks", cfg->batch, world);
  const bool lead = rank == 0;  // logs, previews and scene.json
  AbortOnError abort_guard;
  abort_guard.comm = comm;
  const bool verbose = cfg->log_every > 0 && lead;

  // ---- 1. cameras and targets (train.rs:62-96) ----
  rmh_camera_entry* cams = nullptr;
  int32_t ncam = 0;
  int rc = rmh_cameras_load(cfg->cameras_json, &cams, &ncam);
  if (rc) return rc;
  std::unique_ptr<rmh_camera_entry, void (*)(void*)> cams_guard(cams, std::free);
  if (ncam < 1) return fail(RMH_ERR_FORMAT, "%s holds no camera", cfg->cameras_json);
  const int64_t per_view = (int64_t)W * H;
  const int64_t P = per_view * ncam;
  std::vector<float> h_org(3 * P), h_dir(3 * P), h_tgt(3 * P);
  for (int32_t v = 0; v < ncam; ++v) {
    rmh_camera_rays(W, H, cams[v].origin, cams[v].target, cams[v].fov, h_org.data() + 3 * per_view * v,
                    h_dir.data() + 3 * per_view * v);
    const std::string img = resolve_image(cfg->cameras_json, cams[v].file);
    int32_t iw = 0, ih = 0;
    float* lin = nullptr;
    if ((rc = rmh_image_load(img.c_str(), &iw, &ih, &lin)) != RMH_OK) return rc;
    std::unique_ptr<float, void (*)(void*)> lin_guard(lin, std::free);
    if (iw != W || ih != H) return fail(RMH_ERR_FORMAT, "%s is %dx%d, expected %dx%d", img.c_str(), iw, ih, W, H);
    std::memcpy(h_tgt.data() + 3 * per_view * v, lin, sizeof(float) * 3 * per_view);
  }
  rmh_dataset* ds_raw = nullptr;
  if ((rc = rmh_dataset_create(h_tgt.data(), P, &ds_raw)) != RMH_OK) return rc;
  std::unique_ptr<rmh_dataset, void (*)(rmh_dataset*)> ds(ds_raw, rmh_dataset_destroy);
  int64_t nfg = 0, nbg = 0;
  rmh_dataset_counts(ds.get(), &nfg, &nbg);
  if (verbose) {
    std::printf("Total training pixels: %lld\n", (long long)P);
    std::printf("Foreground pixels: %lld, Background pixels: %lld\n", (long long)nfg, (long long)nbg);
  }

  Gpu g;
  if ((rc = g.open(cfg->device)) != RMH_OK) return rc;
  DevBuf d_org, d_dir, d_tgt, d_fg;
  HIPCHK(d_org.alloc(sizeof(float) * 3 * P));
  HIPCHK(d_dir.alloc(sizeof(float) * 3 * P));
  HIPCHK(d_tgt.alloc(sizeof(float) * 3 * P));
  HIPCHK(hipMemcpyAsync(d_org.p, h_org.data(), d_org.bytes, hipMemcpyHostToDevice, g.stream));
  HIPCHK(hipMemcpyAsync(d_dir.p, h_dir.data(), d_dir.bytes, hipMemcpyHostToDevice, g.stream));
  HIPCHK(hipMemcpyAsync(d_tgt.p, h_tgt.data(), d_tgt.bytes, hipMemcpyHostToDevice, g.stream));
  // this rank's share of the batch (B/P rays per rank, the remainder spread)
  auto share = [&](int32_t q) { return cfg->batch / world + (q < cfg->batch % world ? 1 : 0); };
  const int32_t B = share(rank);
  // the foreground list of the dataset, for the device sampler (rm_train_step_sampled /
  // rm_train_iteration draw the batch from it)
  const int32_t* h_fg = nullptr;
  int64_t n_fg_list = 0;
  rmh_dataset_fg(ds.get(), &h_fg, &n_fg_list);
  HIPCHK(d_fg.alloc(sizeof(int32_t) * (size_t)std::max<int64_t>(n_fg_list, 1)));
  if (n_fg_list > 0) HIPCHK(hipMemcpyAsync(d_fg.p, h_fg, sizeof(int32_t) * n_fg_list, hipMemcpyHostToDevice, g.stream));
  // batches: rank-distinct streams of the device sampler, one counter value per step
  const uint64_t sample_stream = 1 + 1000 * (uint64_t)rank;
  rmh_rng rng_split;
  rmh_rng_seed(&rng_split, cfg->seed, 2);

  // ---- 2. initial model (train.rs:100-126) ----
  int32_t M = 7;
  std::vector<float> raw(7 * M + 4);
  rmh_initial_model(raw.data());
  const std::string out_dir = cfg->out_dir ? cfg->out_dir : "";
  const float total_steps = (float)(cfg->stages * cfg->steps_per_stage);
  float last_loss = 0.0f;
  int32_t steps_done = 0;
  double seconds = 0.0;

  rm_march march;
  rm_march_default(&march);
  march.steps = cfg->march_steps;
  if (f16) march.flags |= RM_MARCH_COLOR_F16;
  PinnedBuf h_loss;  // the loss sum and penalty read back on reporting steps
  HIPCHK(h_loss.alloc(2 * sizeof(float)));
  if (verbose) std::printf("Start Multi-Stage Optimization...\n");

  for (int32_t stage = 0; stage < cfg->stages; ++stage) {
    if (verbose) std::printf("=== Stage %d/%d (N = %d) ===\n", stage + 1, cfg->stages, M);
    const size_t np = 7 * (size_t)M + 4;
    DevBuf d_raw, d_act, d_grad, d_m, d_v, d_col_h;
    HIPCHK(d_raw.alloc(sizeof(float) * np));
    HIPCHK(d_act.alloc(sizeof(float) * np));
    // [packed gradient (np) | loss sum | penalty]: the first np + 1 floats are the one all-reduce
    HIPCHK(d_grad.alloc(sizeof(float) * (np + 2)));
    float* d_loss = d_grad.f() + np;
    HIPCHK(d_m.alloc(sizeof(float) * np));
    HIPCHK(d_v.alloc(sizeof(float) * np));
    HIPCHK(hipMemcpyAsync(d_raw.p, raw.data(), sizeof(float) * np, hipMemcpyHostToDevice, g.stream));
    HIPCHK(hipMemsetAsync(d_m.p, 0, d_m.bytes, g.stream));  // Adam re-created per stage (train.rs:160)
    HIPCHK(hipMemsetAsync(d_v.p, 0, d_v.bytes, g.stream));
    RMCHK(g.ctx, rm_scene_activate(g.ctx, d_raw.f(), M, d_act.f()));
    uint16_t* col_h = nullptr;  // fp16-colour models: the activated colours the renders read
    if (f16) {
      std::vector<float> col(3 * (size_t)M);
      std::vector<uint16_t> half(3 * (size_t)M);
      HIPCHK(hipMemcpyAsync(col.data(), d_act.f() + 3 * M, sizeof(float) * col.size(), hipMemcpyDeviceToHost,
                            g.stream));
      HIPCHK(hipStreamSynchronize(g.stream));
      for (size_t i = 0; i < col.size(); ++i) half[i] = f32_to_f16(col[i]);
      HIPCHK(d_col_h.alloc(sizeof(uint16_t) * half.size()));
      HIPCHK(hipMemcpyAsync(d_col_h.p, half.data(), d_col_h.bytes, hipMemcpyHostToDevice, g.stream));
      col_h = (uint16_t*)d_col_h.p;
    }
    RMCHK(g.ctx, rm_reserve(g.ctx, B, M));
    const std::vector<float> init_centers(raw.begin(), raw.begin() + 3 * M);
    const double base_lr = (double)cfg->base_lr * std::pow(0.6, stage);  // train.rs:166
    rm_scene sc;
    rm_scene_from_packed(d_act.f(), M, &sc);
    if (f16) sc.colors = (const float*)col_h;
    rm_grads gr;
    rm_grads_from_packed(d_grad.f(), M, &gr);

    if ((rc = sync_stream(g, comm)) != RMH_OK) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    for (int32_t step = 1; step <= cfg->steps_per_stage; ++step) {
      const float global_step = (float)(stage * cfg->steps_per_stage + step);
      const float progress = global_step / total_steps;
      march.smooth_k = 5.0f + (cfg->max_smooth - 5.0f) * progress;  // train.rs:174
      const float uniform_ratio = 0.8f - 0.4f * progress;             // train.rs:176
      // sample_batch (dataset.rs:47-82) on the device: the count rule, then draw + gather
      int64_t n_uni = 0, n_boost = 0;
      rmh_dataset_sample_count(ds.get(), B, uniform_ratio, &n_uni, &n_boost);
      // the global ray count of this step: every rank's share under the same count rule
      int64_t n_global = 0;
      for (int32_t q = 0; q < world; ++q) {
        int64_t qu = 0, qf = 0;
        rmh_dataset_sample_count(ds.get(), share(q), uniform_ratio, &qu, &qf);
        n_global += qu + qf;
      }
      // model.forward + compute_loss + backward (train.rs:182-190), mean over the n*3 elements
      const float inv_count = 1.0f / (3.0f * (float)n_global);
      const double lr = step > cfg->steps_per_stage / 2 ? base_lr * 0.2 : base_lr;  // train.rs:193-197
      const bool last = stage == cfg->stages - 1 && step == cfg->steps_per_stage;
      const bool read_loss = (verbose && step % cfg->log_every == 0) || last;
      if (!comm && !f16) {
        // one process, no collective: draw + render + backward + optimizer in one call (one
        // launch for the small models of the schedule; the penalty share only on reporting steps)
        RMCHK(g.ctx, rm_train_iteration(g.ctx, d_org.f(), d_dir.f(), d_tgt.f(), P, d_fg.i(), n_fg_list, n_uni, n_boost,
                                        cfg->seed, sample_stream, (uint64_t)global_step, progress, inv_count, &march,
                                        d_act.f(), d_grad.f(), d_raw.f(), d_m.f(), d_v.f(), M, step, (float)lr,
                                        cfg->weight_decay, 1, d_loss, read_loss ? d_loss + 1 : nullptr));
      } else {
        // draw + render + backward (one launch for the small models, whose extra block also runs
        // the optimizer's gradient-independent part), then the all-reduce, then the update
        RMCHK(g.ctx, rm_train_step_sampled_prepared(g.ctx, d_org.f(), d_dir.f(), d_tgt.f(), P, d_fg.i(), n_fg_list,
                                                    n_uni, n_boost, cfg->seed, sample_stream, (uint64_t)global_step,
                                                    progress, inv_count, &sc, &march, &gr, d_loss, d_raw.f(), step, 1,
                                                    read_loss ? d_loss + 1 : nullptr));
        if (comm && (rc = comm->all_reduce_sum(comm->state, d_grad.f(), (int64_t)np + 1, g.stream)) != RMH_OK)
          return fail(rc, "all-reduce of the gradient (stage %d, step %d): %s", stage, step, rmh_last_error());
        // the penalty share of the loss costs a summation launch: only on the steps that report it
        if (f16)
          RMCHK(g.ctx, rm_optimizer_step_f16(g.ctx, d_raw.f(), d_grad.f(), d_m.f(), d_v.f(), M, step, (float)lr,
                                             cfg->weight_decay, 1, read_loss ? d_loss + 1 : nullptr, d_act.f(), col_h));
        else
          RMCHK(g.ctx, rm_optimizer_step(g.ctx, d_raw.f(), d_grad.f(), d_m.f(), d_v.f(), M, step, (float)lr,
                                         cfg->weight_decay, 1, read_loss ? d_loss + 1 : nullptr, d_act.f()));
      }
      ++steps_done;
      // With collectives every rank drains its stream under the watchdog every kStepsInFlight
      // steps, not only where rank 0 reads the loss: a rank whose peer stopped then meets the
      // watchdog within kStepsInFlight steps instead of blocking inside a launch or ncclAllReduce
      // once the HIP queue fills, and the watchdog's timeout measures at most that many steps of
      // queued work, not a whole stage's backlog.
      if (comm && world > 1 && !read_loss && step % kStepsInFlight == 0 && (rc = sync_stream(g, comm)) != RMH_OK)
        return rc;
      if (read_loss) {
        // into page-locked memory on the stream, then one wait under the watchdog
        HIPCHK(hipMemcpyAsync(h_loss.p, d_loss, 2 * sizeof(float), hipMemcpyDeviceToHost, g.stream));
        if ((rc = sync_stream(g, comm)) != RMH_OK) return rc;
        const float* s = h_loss.f();
        last_loss = s[0] * inv_count + s[1];  // training.rs:34 + penalties
        if (verbose && step % cfg->log_every == 0) {
          std::printf("  Step %d | Loss: %.5f | k: %.1f", step, last_loss, march.smooth_k);
          if (const char* e = std::getenv("RMH_LOG_BITS"); e && e[0] == '1') {  // diagnosis: the loss bits
            uint32_t b[2];
            std::memcpy(b, s, sizeof b);
            std::printf(" | bits %08x %08x", b[0], b[1]);
          }
          std::printf("\n");
        }
      }
    }
    const auto t_enq = std::chrono::steady_clock::now();  // the host has issued the stage's steps
    if ((rc = sync_stream(g, comm)) != RMH_OK) return rc;
    const auto t_end = std::chrono::steady_clock::now();
    seconds += std::chrono::duration<double>(t_end - t0).count();
    if (const char* e = std::getenv("RMH_STAGE_TIMES"); e && e[0] == '1')  // measurement: host issue vs drain
      std::fprintf(stderr, "stage %d: issued in %.3f ms, drained %.3f ms later\n", stage + 1,
                   1e3 * std::chrono::duration<double>(t_enq - t0).count(),
                   1e3 * std::chrono::duration<double>(t_end - t_enq).count());
    HIPCHK(hipMemcpy(raw.data(), d_raw.p, sizeof(float) * np, hipMemcpyDeviceToHost));
    if (cfg->on_generation) cfg->on_generation(cfg->user, stage, M, raw.data());

    if (stage == cfg->stages - 1) {  // train.rs:206-290
      if (lead && !out_dir.empty()) {
        if ((rc = export_scene(raw, M, join_path(out_dir, "scene.json"))) != RMH_OK) return rc;
        if (verbose) std::printf("  => Saved to scene.json (N = %d)\n", M);
        if (cfg->previews &&
            (rc = preview_packed(g, d_act.f(), col_h, M, W, H, cfg->march_steps,
                                 join_path(out_dir, "steps/final_1.png"))))
          return rc;
      }
      break;
    }
    if (lead && cfg->previews && !out_dir.empty()) {
      char name[64];
      std::snprintf(name, sizeof name, "steps/stage_%d.png", stage);
      if ((rc = preview_packed(g, d_act.f(), col_h, M, W, H, cfg->march_steps, join_path(out_dir, name)))) return rc;
    }
    // ---- C. prune & split (train.rs:300-328) ----
    // rank 0 decides the next generation and broadcasts it: its size, then its raw params
    std::vector<float> next(14 * (size_t)M + 4);
    int32_t nextM = 0;
    int split_rc = RMH_OK;
    if (lead)
      split_rc = rmh_prune_and_split_ex(raw.data(), M, init_centers.data(), stage, cfg->stages, split_scale,
                                        split_move, cfg->max_spheres, &rng_split, next.data(), &nextM);
    if (split_rc != RMH_OK && !comm) return split_rc;
    if (comm) {  // (with one rank too: the RCCL path is the same)
      DevBuf d_next;
      HIPCHK(d_next.alloc(sizeof(float) * next.size()));
      // the size doubles as the status word: -1 tells every rank that rank 0 failed
      float fm = split_rc == RMH_OK ? (float)nextM : -1.0f;  // M' <= 2M <= 2^17: exact in fp32
      HIPCHK(hipMemcpyAsync(d_next.p, &fm, sizeof fm, hipMemcpyHostToDevice, g.stream));
      if ((rc = comm->broadcast(comm->state, d_next.f(), 1, 0, g.stream)) != RMH_OK)
        return fail(rc, "broadcast of the next size: %s", rmh_last_error());
      if ((rc = sync_stream(g, comm)) != RMH_OK) return rc;
      HIPCHK(hipMemcpy(&fm, d_next.p, sizeof fm, hipMemcpyDeviceToHost));
      nextM = (int32_t)fm;
      if (split_rc != RMH_OK) return split_rc;  // rank 0, after telling the others
      if (nextM < 0) return fail(RMH_ERR_GPU, "rank 0 failed in prune_and_split (stage %d)", stage);
      if (nextM < 1 || 7 * (size_t)nextM + 4 > next.size()) return fail(RMH_ERR_GPU, "broadcast size %d", nextM);
      const size_t nn = 7 * (size_t)nextM + 4;
      if (lead) HIPCHK(hipMemcpyAsync(d_next.p, next.data(), sizeof(float) * nn, hipMemcpyHostToDevice, g.stream));
      if ((rc = comm->broadcast(comm->state, d_next.f(), (int64_t)nn, 0, g.stream)) != RMH_OK)
        return fail(rc, "broadcast of the next generation: %s", rmh_last_error());
      if ((rc = sync_stream(g, comm)) != RMH_OK) return rc;
      HIPCHK(hipMemcpy(next.data(), d_next.p, sizeof(float) * nn, hipMemcpyDeviceToHost));
    }
    if (nextM > RM_MAX_SPHERES) return fail(RMH_ERR_INVALID_ARG, "model grew past RM_MAX_SPHERES");
    next.resize(7 * (size_t)nextM + 4);
    raw.swap(next);
    M = nextM;
    if (verbose) std::printf("  => Pruning & Splitting complete. Next N = %d\n", M);
  }

  if (raw_out) {
    if (raw_capacity < 7 * M + 4) return fail(RMH_ERR_INVALID_ARG, "raw_out holds %d floats, need %d", raw_capacity,
                                              7 * M + 4);
    std::memcpy(raw_out, raw.data(), sizeof(float) * (7 * (size_t)M + 4));
  }
  abort_guard.done = true;
  if (result) {
    result->num_spheres = M;
    result->steps = steps_done;
    result->final_loss = last_loss;
    result->seconds = seconds;
    result->step_ms = steps_done ? 1e3 * seconds / steps_done : 0.0;
  }
  return RMH_OK;
}

int rmh_preview(const char* scene_json, const char* png_path, int32_t W, int32_t H, const float eye[3],
                const float target[3], float fov_deg, float radius_offset, int32_t device) {
  if (!scene_json || !png_path || !eye || !target || W < 1 || H < 1) return fail(RMH_ERR_INVALID_ARG, "bad arguments");
  int32_t M = 0;
  float *c = nullptr, *col = nullptr, *r = nullptr, ld[3], amb = 0.0f;
  int rc = rmh_scene_load(scene_json, &M, &c, &col, &r, ld, &amb);
  if (rc) return rc;
  std::unique_ptr<float, void (*)(void*)> g1(c, std::free), g2(col, std::free), g3(r, std::free);
  if (M < 1) return fail(RMH_ERR_FORMAT, "%s has no sphere", scene_json);
  std::vector<float> act(7 * (size_t)M + 4);
  std::memcpy(act.data(), c, sizeof(float) * 3 * M);
  std::memcpy(act.data() + 3 * M, col, sizeof(float) * 3 * M);
  for (int32_t i = 0; i < M; ++i) act[6 * M + i] = r[i] + radius_offset;
  std::memcpy(act.data() + 7 * M, ld, sizeof ld);
  act[7 * M + 3] = amb;
  Gpu g;
  if ((rc = g.open(device)) != RMH_OK) return rc;
  DevBuf d_act, out;
  HIPCHK(d_act.alloc(sizeof(float) * act.size()));
  HIPCHK(hipMemcpyAsync(d_act.p, act.data(), d_act.bytes, hipMemcpyHostToDevice, g.stream));
  rm_scene sc;
  rm_scene_from_packed(d_act.f(), M, &sc);
  rm_march m;
  rm_march_default(&m);  // S = 40, k = 32 (train.rs:355)
  rm_camera cam;
  camera_struct(cam, eye, target, fov_deg);
  HIPCHK(out.alloc(sizeof(float) * 3 * (size_t)W * H));
  RMCHK(g.ctx, rm_render_diff_camera(g.ctx, &cam, 1, W, H, &sc, &m, out.f(), nullptr));
  std::vector<float> host(3 * (size_t)W * H);
  HIPCHK(hipMemcpyAsync(host.data(), out.p, out.bytes, hipMemcpyDeviceToHost, g.stream));
  HIPCHK(hipStreamSynchronize(g.stream));
  return rmh_image_save(png_path, host.data(), W, H);
}

int rmh_generate(const char* out_dir, const char* prefix, int32_t W, int32_t H, int32_t device) {
  if (!out_dir || W < 1 || H < 1) return fail(RMH_ERR_INVALID_ARG, "bad arguments");
  const std::string pre = prefix ? prefix : "";
  // generate.rs:29-40: the three-sphere "dango"
  const float centers[9] = {-0.3f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.3f, 0.0f, 0.0f};
  const float colors[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  const float radii[3] = {0.2f, 0.15f, 0.2f};
  // generate.rs:44-86: 8 views around at y = 0.5, one from the top, one from below
  std::vector<rmh_camera_entry> cams;
  const int num_h = 8;
  const float radius = 2.5f, fov = 50.0f;
  auto add = [&](float x, float y, float z) {
    rmh_camera_entry e;
    std::memset(&e, 0, sizeof e);
    std::snprintf(e.file, sizeof e.file, "%starget_%zu.png", pre.c_str(), cams.size());
    e.origin[0] = x;
    e.origin[1] = y;
    e.origin[2] = z;
    e.fov = fov;
    cams.push_back(e);
  };
  for (int i = 0; i < num_h; ++i) {
    const float angle = (float)i * (2.0f * (float)M_PI / (float)num_h);
    add(radius * std::cos(angle), 0.5f, radius * std::sin(angle));
  }
  add(0.0f, 2.5f, -0.001f);
  add(0.0f, -1.5f, -2.0f);
  const int V = (int)cams.size();
  Gpu g;
  int rc;
  if ((rc = g.open(device)) != RMH_OK) return rc;
  DevBuf d_c, d_col, d_r, out;
  HIPCHK(d_c.alloc(sizeof centers));
  HIPCHK(d_col.alloc(sizeof colors));
  HIPCHK(d_r.alloc(sizeof radii));
  HIPCHK(hipMemcpyAsync(d_c.p, centers, sizeof centers, hipMemcpyHostToDevice, g.stream));
  HIPCHK(hipMemcpyAsync(d_col.p, colors, sizeof colors, hipMemcpyHostToDevice, g.stream));
  HIPCHK(hipMemcpyAsync(d_r.p, radii, sizeof radii, hipMemcpyHostToDevice, g.stream));
  std::vector<rm_camera> rc_cams(V);
  for (int v = 0; v < V; ++v) camera_struct(rc_cams[v], cams[v].origin, cams[v].target, cams[v].fov);
  const size_t per_view = 3 * (size_t)W * H;
  HIPCHK(out.alloc(sizeof(float) * per_view * V));
  RMCHK(g.ctx, rm_render_camera(g.ctx, rc_cams.data(), V, W, H, d_c.f(), d_col.f(), d_r.f(), 3, out.f()));
  std::vector<float> host(per_view * V);
  HIPCHK(hipMemcpyAsync(host.data(), out.p, out.bytes, hipMemcpyDeviceToHost, g.stream));
  HIPCHK(hipStreamSynchronize(g.stream));
  const std::string dir = out_dir;
  for (int v = 0; v < V; ++v) {
    char name[64];
    std::snprintf(name, sizeof name, "target_%d.png", v);
    if ((rc = rmh_image_save(join_path(dir, name).c_str(), host.data() + per_view * v, W, H)) != RMH_OK) return rc;
  }
  return rmh_cameras_save(join_path(dir, "cameras.json").c_str(), cams.data(), V);
}

}  // extern "C"
