/*
 * raymarch.h -- C ABI of libraymarch_hip.so, the MI355X (gfx950) differentiable
 * SDF-sphere raymarcher.
 *
 * This boundary replaces the reference's hot path, the per-ray differentiable
 * render of kokutoupan/burn_raymarching:
 *
 *   render_diff<B: Backend>(ray_org [N,3], ray_dir [N,3], centers [M,3], colors [M,3],
 *                           radius [M,1], light_dir [3], ambient [1], smooth_k: f32)
 *       -> Tensor<B,2> [N,3]                              (src/renderer_diff.rs:6-15)
 *
 * called from SceneModel::forward (src/model/scene.rs:35-57) by the training step
 * (src/bin/train.rs:182) and the preview (src/bin/train.rs:355), together with its
 * gradient, which the reference gets from burn-autodiff via loss.backward()
 * (src/bin/train.rs:189-190). The reference has no FFI for this path; a Rust host
 * would bind these entry points with `extern "C"`.
 *
 * Conventions
 *  - Every tensor argument is a caller-owned DEVICE pointer to fp32, row-major, AoS
 *    [n][3] exactly like the reference's tensors. Camera descriptors are host structs.
 *  - Scene parameters are the ACTIVATED values render_diff receives
 *    (scene.rs:41-45): colors = sigmoid(raw), radius = softplus(raw)+0.01,
 *    ambient = sigmoid(raw), light_dir raw (normalised inside, renderer_diff.rs:49-50).
 *    rm_scene_activate() produces them from the raw Param tensors.
 *  - Every call is asynchronous on the context's stream; the caller synchronises.
 *  - Return value: RM_OK (0) or an RM_ERR_* code; rm_last_error() has the text.
 *    Invalid arguments never launch work. A context is not thread-safe; use one
 *    context per host thread / stream.
 *  - Results are deterministic: every cross-ray sum is reduced in a fixed order.
 */
#ifndef RAYMARCH_H_
#define RAYMARCH_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RM_OK 0
#define RM_ERR_INVALID_ARG 1
#define RM_ERR_HIP 2
#define RM_ERR_OOM 3
#define RM_ERR_UNSUPPORTED 4

/* Limits of this build. */
#define RM_MAX_VIEWS_PER_CALL 128    /* camera descriptors per rm_*_camera call */
#define RM_MAX_SPHERES 65536

typedef struct rm_context rm_context;

/* Activated scene parameters (device pointers), scene.rs:9-16 after scene.rs:41-45. */
typedef struct rm_scene {
  const float* centers;   /* [M,3]                                      */
  const float* colors;    /* [M,3] sigmoid(raw colors)                   */
  const float* radius;    /* [M]   softplus(raw radius) + 0.01           */
  const float* light_dir; /* [3]   raw light direction                   */
  const float* ambient;   /* [1]   sigmoid(raw ambient)                  */
  int32_t num_spheres;    /* M >= 1                                      */
} rm_scene;

/* March / shading constants. rm_march_default() fills the reference's values. */
typedef struct rm_march {
  int32_t steps;          /* fixed march steps, renderer_diff.rs:22 (40)             */
  float smooth_k;         /* soft-min sharpness k, sdf.rs:30 (train 5->32, preview 32) */
  float normal_eps;       /* finite-difference normal step, scene.rs:91 (1e-4)       */
  float color_sharpness;  /* softmax(-c * dist) colour blend, renderer_diff.rs:74 (10) */
  float mask_sharpness;   /* sigmoid(-c * D) silhouette, renderer_diff.rs:88 (15)     */
  int32_t flags;          /* RM_MARCH_* bits (default 0)                              */
} rm_march;

/* Skip the per-sphere work of ray blocks that provably escape the scene: every ray of the
 * block ends its march past the scene's bounding sphere at a distance where the silhouette
 * mask is exactly 0 in f32, so out = 0 and all its gradient terms are 0 -- the values the full
 * computation produces. The proof is a conservative f64 march of a bounding-sphere lower bound
 * in a pre-pass kernel (escapes() in rm_kernels.hip); camera mode then renders 16x16 pixel
 * tiles per block. Pays for compact scenes seen in camera mode (previews, target generation);
 * off by default because the pre-pass and the uneven block costs lose when few blocks escape.
 * Ignored when t_march or debug outputs are requested. */
#define RM_MARCH_SKIP_ESCAPED 1
/* Camera mode: launch rays in row order instead of 16x16 pixel tiles per 256-ray block (8x8
 * per wave; the default when width and height are multiples of 16). Changes only the
 * summation order of the gradients. */
#define RM_MARCH_ROW_ORDER 2
/* Disable the escaped-ray early exit: by default a wave stops marching once all its rays
 * recede from the scene's bounding sphere at a distance where the silhouette mask is exactly
 * 0 in fp32 (their outputs and gradient terms are then exactly 0, as the full computation
 * gives). Set for A/B timing; t_march and debug outputs disable it automatically (rays that
 * provably escape still step by the escape bound, see t_march below). */
#define RM_MARCH_NO_EARLY_EXIT 4
/* Camera mode with 16x16 tiles and whole views per launch: dispatch the ray blocks in launch
 * order instead of centre-out (tiles nearest the image centre first, views interleaved, so the
 * blocks that march every step start first and the cheap border blocks fill the tail). The
 * dispatch order changes no result bit: gradient partials are indexed by tile. A/B timing. */
#define RM_MARCH_NATURAL_ORDER 8
/* Run the march's sphere sums on the vector units only. By default the squared distances of
 * the unshifted / fixed-shift march steps come from bf16 matrix-core products of exact
 * three-part splits of the fp32 operands (equal to the fp32 expansion form to rounding) and
 * the vector units do only sqrt, exp2 and the accumulate. A/B timing. */
#define RM_MARCH_VALU_ONLY 16
/* Camera mode: every ray of a view starts at the eye, so by default the first march step's
 * soft-min D(eye) is evaluated once per view (in the per-call record kernel, by the march's own
 * code path for that step) and shared by all rays of the view -- bit-identical results, one
 * march step fewer per ray. This flag makes every ray evaluate it itself. A/B timing. */
#define RM_MARCH_PER_RAY_ORIGIN 32
/* Train / backward calls over the same views (one launch): by default the ray blocks are
 * dispatched grouped by the cost they had in the previous such call (march steps their waves
 * ran, plus the post-march work of live waves), dearest first; this flag keeps the static
 * centre-out order. Results are identical either way. A/B timing. */
#define RM_MARCH_STATIC_ORDER 64
/* Testing: every march step takes the running-maximum log-sum-exp shift (the vector path that
 * follows the reference's exact max, sdf.rs:36-37) instead of the provably safe unshifted /
 * fixed-shift forms; implies RM_MARCH_PER_RAY_ORIGIN. Results agree to fp32 rounding. */
#define RM_MARCH_FORCE_MAX_SHIFT 128
/* fp16 colour / fp32 SDF (BASELINE configs[4]): rm_scene.colors points to IEEE binary16
 * [M,3] activated colours instead of fp32. The per-call record kernel widens them exactly;
 * the colour blend, the SDF, the march and every gradient stay fp32 (grads->colors is fp32,
 * the master gradient). See rm_optimizer_step_f16 for the optimizer side. */
#define RM_MARCH_COLOR_F16 256
/* Split march: a ray block takes 32 rays (half an 8x8 pixel quadrant in camera mode) held by all
 * four waves of the block; every march step each wave sums a quarter of the spheres on the
 * matrix cores and the quarters are added in a fixed order, so the waves march in lockstep;
 * the post-march sweeps are split the same way, and the backward shares the sphere groups out
 * over the four waves. A ray that marches every step then spreads over four SIMDs: for launches that fill
 * the GPU a few times (BASELINE configs[4]), where a few rays march all steps while the rest
 * leave early. Taken automatically from 256 spheres for launches of at most 262,144 rays and
 * from 512 spheres for at most 1,048,576 rays; this flag forces it, RM_MARCH_NO_SPLIT forbids
 * it. Results agree to fp32 rounding (the sphere sums are added in another order). */
#define RM_MARCH_SPLIT 512
#define RM_MARCH_NO_SPLIT 1024

/* Pinhole LookAt camera, camera.rs:30-37. Rays are generated in-kernel exactly as
 * create_camera_rays (camera.rs:41-87): rows y then x, u = x/W*2-1, v = -(y/H*2-1). */
typedef struct rm_camera {
  float eye[3];
  float target[3];
  float fov_deg;
} rm_camera;

/* Gradient outputs (device pointers) w.r.t. the ACTIVATED parameters, except
 * light_dir which is w.r.t. the raw light direction (the normalisation is inside
 * render_diff). Any pointer may be NULL to skip that output. */
typedef struct rm_grads {
  float* centers;    /* [M,3] */
  float* colors;     /* [M,3] */
  float* radius;     /* [M]   */
  float* light_dir;  /* [3]   */
  float* ambient;    /* [1]   */
} rm_grads;

/* ---- context --------------------------------------------------------------- */
/* "burn_raymarching_amd <version> (gfx950) src <hash>": <hash> = the first 16 hex digits of the
 * sha256 of the kernel sources the library was built from (burn_raymarching_amd/_build.py). */
const char* rm_version(void);
/* stream: a hipStream_t (NULL = the null stream). */
int rm_create(int32_t device, void* stream, rm_context** out_ctx);
int rm_set_stream(rm_context* ctx, void* stream);
void rm_destroy(rm_context* ctx);
const char* rm_last_error(const rm_context* ctx);
void rm_march_default(rm_march* m);
/* Pre-size the workspace for backward/train calls of up to max_rays rays and
 * max_spheres spheres, and allocate the context's small per-call buffers (reduction arrival
 * counters, the fused iteration's optimizer hand-off), so later calls never allocate (needed
 * for hipGraph capture; keeps first-call allocations out of a timed loop). */
int rm_reserve(rm_context* ctx, int64_t max_rays, int32_t max_spheres);

/* ---- forward: renderer_diff.rs:6-91 --------------------------------------- */
/* out [N,3] receives render_diff(ray_org, ray_dir, scene..., smooth_k).
 * t_march (nullable) [N] receives the detached march distance t after `steps`
 * steps (renderer_diff.rs:20-26), which rm_render_diff_backward can reuse. For a ray that
 * provably escapes the scene -- receding from its bounding sphere so far that the silhouette
 * mask, out and every gradient term are exactly 0 in fp32 -- the march continues with steps
 * of that escape bound (|p - c| - R - ln(M)/k, never longer than the soft-min step), so its
 * t_march is at most the reference's t and already past the distance where the mask is 0;
 * every other ray's t_march is the reference march to fp32 rounding. Either t gives the same
 * out and gradients. */
int rm_render_diff(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
                   const rm_scene* scene, const rm_march* march, float* out, float* t_march);
/* Camera mode: rays of `num_views` cameras at width x height generated in-kernel;
 * out is [num_views*height*width, 3] in view, row, column order. */
int rm_render_diff_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width,
                          int32_t height, const rm_scene* scene, const rm_march* march, float* out,
                          float* t_march);

/* ---- backward: the burn-autodiff gradient of render_diff ------------------ */
/* grad_out [N,3] = dL/d(out). t_march (nullable) = the forward's saved march t;
 * when given the march is not replayed. accumulate != 0 adds into the grads. */
int rm_render_diff_backward(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
                            const rm_scene* scene, const rm_march* march, const float* grad_out,
                            const float* t_march, const rm_grads* grads, int32_t accumulate);
int rm_render_diff_backward_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width,
                                   int32_t height, const rm_scene* scene, const rm_march* march,
                                   const float* grad_out, const float* t_march, const rm_grads* grads,
                                   int32_t accumulate);

/* ---- fused train step: forward + compute_loss seed + backward ------------- */
/* The reconstruction term of compute_loss (training.rs:17-34): for each ray,
 * W = 10 where sum(target) > 0.01 else 1 + 4*progress, loss += sum_c |out-target|*W,
 * g = W*sign(out-target)*inv_count (inv_count = 1/(3*N_global) gives the mean).
 * loss_sum (device, 1 float) receives sum |out-target|*W (multiply by inv_count
 * for the mean), added to its current value when accumulate != 0. out (nullable)
 * receives the forward image. targets are linear RGB [N,3]. */
int rm_train_step(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                  int64_t num_rays, float progress, float inv_count, const rm_scene* scene,
                  const rm_march* march, const rm_grads* grads, float* loss_sum, float* out,
                  int32_t accumulate);
int rm_train_step_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width,
                         int32_t height, const float* targets, float progress, float inv_count,
                         const rm_scene* scene, const rm_march* march, const rm_grads* grads,
                         float* loss_sum, float* out, int32_t accumulate);

/* ---- non-differentiable target renderer: renderer.rs:4-80 (used by generate.rs) ---- */
/* 40 march steps at k = 32, detached normal, fixed light (-0.5, 0.5, -1)/|.|, lighting =
 * diffuse + 0.1, colour = sum(col exp(-10 d)) / (sum(exp(-10 d)) + 1e-5), mask = exp(-10 D^2).
 * centers/colors/radius are device pointers ([M,3], [M,3], [M]); out [N,3]. */
int rm_render(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
              const float* centers, const float* colors, const float* radius, int32_t num_spheres, float* out);
int rm_render_camera(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width, int32_t height,
                     const float* centers, const float* colors, const float* radius, int32_t num_spheres,
                     float* out);

/* ---- batch gather: SceneDataset::sample_batch, dataset.rs:75-79 ---------------- */
/* out_*[i] = src[indices[i]] for the ray origin, direction and target arrays ([num_src,3]
 * each; any output may be NULL to skip it). indices is a device int32 [num_rays]; an index
 * outside [0, num_src) gives a zero row. */
int rm_gather_rays(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                   int64_t num_src, const int32_t* indices, int64_t num_rays, float* out_org, float* out_dir,
                   float* out_targets);

/* ---- batch sampler on the device: SceneDataset::sample_batch, dataset.rs:47-82 ------------- */
/* Draws n_uniform pixel indices uniformly from [0, num_src), then n_fg more uniformly from the
 * foreground list fg_indices[0, num_fg) (device int32; dataset.rs:54-73 -- the counts come from
 * the caller, see rmh_dataset_sample_count), and gathers those rows of ray_org / ray_dir /
 * targets ([num_src,3] device arrays) into out_* ([n_uniform+n_fg,3]; any NULL to skip it);
 * indices_out (nullable, int32) receives the drawn indices. The generator is counter-based (row
 * i of call (seed, stream, counter) is a splitmix64 draw of those four numbers), so a batch is
 * reproducible and independent of the launch; the reference's draws (rand::rng()) are unseeded,
 * so batches match it in distribution. One kernel: no host sampling, no host-to-device copy. */
int rm_sample_batch(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets, int64_t num_src,
                    const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg, uint64_t seed,
                    uint64_t stream, uint64_t counter, float* out_org, float* out_dir, float* out_targets,
                    int32_t* indices_out);

/* ---- hipGraph capture of a training step ----------------------------------- */
/* A step's calls (train step, optimizer) can be captured once in a hipGraph
 * (hipStreamBeginCapture on the context's stream ... hipStreamEndCapture, hipGraphInstantiate)
 * and replayed with hipGraphLaunch. What changes from one step to the next lives on the device:
 *  - the per-step scalars: while an rm_step_scalars record is bound to the context
 *    (rm_bind_step_scalars), rm_train_step[_camera] take progress = min(index / total, 1) in fp32
 *    (train.rs:171-172) instead of their `progress` argument, and rm_optimizer_step[_f16] take
 *    Adam's step from `step` instead of their argument and then advance the record on the device
 *    (step += 1, index += 1) -- the optimizer ends a training step;
 *  - the cost-ordered dispatch rotates its list sets on the device by itself.
 * rm_reserve before the capture keeps every call allocation-free; kernel timing (rm_timing_enable)
 * and rm_train_iteration's one-launch form are not for capture (with a bound record,
 * rm_train_iteration runs its three calls). dev = NULL unbinds; the record is the caller's device
 * memory and must outlive the binding. */
typedef struct rm_step_scalars {
  int32_t step;     /* Adam's step of the next optimizer call (counts from 1) */
  int32_t index;    /* the global step of the next train call ... */
  int32_t total;    /* ... out of total: progress = index / total */
  int32_t reserved;
} rm_step_scalars;
int rm_bind_step_scalars(rm_context* ctx, rm_step_scalars* dev);

/* ---- diagnostics ------------------------------------------------------------ */
/* Per-ray forward intermediates dbg [N][24] = {t, t_final, n.x, n.y, n.z, lighting,
 * mix.r, mix.g, mix.b, D_final, mask, n.l, min delta, Zw, Zb, 0, D(+x), D(-x), D(+y),
 * D(-y), D(+z), D(-z), 0, 0} (renderer_diff.rs
 * stages) for parity debugging against the oracle. Not on the hot path. */
int rm_debug_intermediates(rm_context* ctx, const float* ray_org, const float* ray_dir, int64_t num_rays,
                           const rm_scene* scene, const rm_march* march, float* dbg);

/* Cost-ordered dispatch state (tests): copies the 3 x classes per-class block counts of the
 * three list sets (see RM_MARCH_STATIC_ORDER) into counts[0 .. 3*classes) after synchronising
 * the stream; *classes = the build's class count, *next_set = the set the next keyed launch
 * appends to (it reads set (next_set + 2) % 3, whose total equals the launch's block count
 * when the cost order is used and differs when the launch falls back to the static order).
 * Environment RM_DEBUG_SKIP_ORDER_CLEAR=1 makes a launch leave the next set's counts
 * uncleared (the state a failed launch in the rotation leaves), for the recovery test. */
int rm_debug_order_counts(rm_context* ctx, int32_t* counts, int32_t capacity, int32_t* classes, int32_t* next_set);

/* Stream stall (tests of a caller's watchdog, e.g. rmh_collective.wait): enqueues on the context's
 * stream one wave that spins until rm_debug_stall_release(ctx) or until max_ms (1 .. 600000) have
 * passed, whichever comes first -- it always ends by itself. rm_destroy releases a pending one. */
int rm_debug_stall(rm_context* ctx, int32_t max_ms);
int rm_debug_stall_release(rm_context* ctx);

/* ---- kernel timing (benchmark instrumentation) ------------------------------ */
/* rm_timing_enable(ctx, 1): every later render / backward / train call records a
 * hipEvent pair around each launch of its main per-ray kernel on the context's
 * stream. rm_timing_collect synchronises those events and returns the summed kernel
 * time in milliseconds and the number of launches (reset != 0 clears the record). */
int rm_timing_enable(rm_context* ctx, int32_t enable);
int rm_timing_collect(rm_context* ctx, double* total_ms, int64_t* launches, int32_t reset);

/* ---- work statistics -------------------------------------------------------- */
/* rm_stats_enable(ctx, 1): count, for every later per-ray launch, the ray blocks (256 rays)
 * launched, those skipped whole by RM_MARCH_SKIP_ESCAPED, and the waves (64 rays) that left
 * the march early because all their rays escaped, with the march steps they saved, and the rays
 * the backward modes' two gradient sweeps ran for (the rays with non-zero seeds: a ray whose
 * seeds are 0 contributes exact zeros and is not swept; the general kernel counts them, the
 * small kernel (M <= 32) reports 0).
 * rm_stats_collect synchronises the stream; reset != 0 clears the counters. */
typedef struct rm_stats {
  int64_t blocks;          /* ray blocks launched */
  int64_t blocks_skipped;  /* blocks skipped by RM_MARCH_SKIP_ESCAPED */
  int64_t waves;           /* waves launched (4 per block) */
  int64_t waves_exited;    /* waves that stopped marching early (all rays escaped) */
  int64_t steps_saved;     /* march steps those waves did not run */
  int64_t seeded_rays;     /* rays the first backward sweep (at p) ran for */
  int64_t seeded_rays_a;   /* rays the second backward sweep (at p_approx) ran for */
} rm_stats;
int rm_stats_enable(rm_context* ctx, int32_t enable);
int rm_stats_collect(rm_context* ctx, rm_stats* out, int32_t reset);

/* ---- model helpers: SceneModel activations, compute_loss penalties, Adam ---- */
/* Packed parameter layout used by the helpers (raw Param tensors or their grads):
 *   [centers 3M | colors 3M | radius M | light_dir 3 | ambient 1]  (7M+4 floats)
 * rm_scene_activate writes the activated values in the same packed layout
 * (scene.rs:41-45) so an rm_scene can point into it (see rm_scene_from_packed). */
int rm_scene_activate(rm_context* ctx, const float* raw_packed, int32_t num_spheres, float* act_packed);
void rm_scene_from_packed(const float* act_packed, int32_t num_spheres, rm_scene* out_scene);
void rm_grads_from_packed(float* grad_packed, int32_t num_spheres, rm_grads* out_grads);

/* Optimizer step on the raw packed params (train.rs:161-198): the activated-space
 * gradient (packed, e.g. all-reduced across ranks) is chained through scene.rs:41-45,
 * the compute_loss parameter penalties (training.rs:38-82) are added when
 * with_penalties != 0, then Burn's Adam (beta1 0.9, beta2 0.999, eps 1e-5) with
 * coupled L2 weight decay `weight_decay` updates raw_packed in place. adam_m and
 * adam_v are (7M+4)-float device buffers (zero them when re-initialising the
 * optimizer, train.rs:160-163); step counts from 1. loss_penalty (nullable, device
 * float) receives the penalty value at the pre-step parameters. act_out (nullable)
 * receives the activated packed parameters of the UPDATED model (what
 * rm_scene_activate would return), so the next render needs no separate launch. */
int rm_optimizer_step(rm_context* ctx, float* raw_packed, const float* grad_act_packed, float* adam_m,
                      float* adam_v, int32_t num_spheres, int32_t step, float lr, float weight_decay,
                      int32_t with_penalties, float* loss_penalty, float* act_out);

/* rm_optimizer_step for fp16-colour models (RM_MARCH_COLOR_F16, BASELINE configs[4]): the
 * same update (fp32 master parameters, moments and gradient), and colors_f16_out (nullable,
 * device, [M,3] IEEE binary16) receives the updated activated colours rounded to nearest --
 * the colour tensor of the next fp16-colour render. */
int rm_optimizer_step_f16(rm_context* ctx, float* raw_packed, const float* grad_act_packed, float* adam_m,
                          float* adam_v, int32_t num_spheres, int32_t step, float lr, float weight_decay,
                          int32_t with_penalties, float* loss_penalty, float* act_out, uint16_t* colors_f16_out);

/* One single-process training step on whole views (train.rs:182-198: model.forward, compute_loss,
 * loss.backward(), optim.step), replacing rm_train_step_camera -> rm_optimizer_step[_f16] with the
 * same arguments and the same results bit for bit:
 *   1. the render of act_packed (activated packed parameters; with RM_MARCH_COLOR_F16 in
 *      march->flags the colours come from colors_f16_out), the loss seed and the backward into
 *      grad_packed ((7M+4) floats, overwritten) and loss_sum (1 float, overwritten), as
 *      rm_train_step_camera with progress and inv_count;
 *   2. the optimizer step on raw_packed / adam_m / adam_v (step, lr, weight_decay,
 *      with_penalties, loss_penalty nullable) writing the updated activated parameters to
 *      act_packed (and, fp16-colour models, their rounded colours to colors_f16_out), as
 *      rm_optimizer_step_f16 with act_out = act_packed.
 * Models of up to 64 spheres run the optimizer inside the call's gradient reduction, in the block
 * that completes the gradient (env RM_FUSED_ADAM=0 turns this off): one launch fewer per step.
 * Otherwise -- more spheres, the small-scene kernel, more than one ray sub-launch -- the two calls
 * run as such. Bound step scalars (rm_bind_step_scalars) apply as to the two calls. Not for
 * data-parallel training: the gradient is consumed before it could be all-reduced. */
int rm_train_step_camera_adam(rm_context* ctx, const rm_camera* cams, int32_t num_views, int32_t width,
                              int32_t height, const float* targets, float progress, float inv_count,
                              const rm_march* march, float* act_packed, float* grad_packed, float* raw_packed,
                              float* adam_m, float* adam_v, int32_t num_spheres, int32_t step, float lr,
                              float weight_decay, int32_t with_penalties, float* loss_sum, float* loss_penalty,
                              uint16_t* colors_f16_out);

/* One step of the reference training loop (train.rs:169-198) for one process, replacing the
 * sequence rm_sample_batch -> rm_train_step -> rm_optimizer_step with the same arguments and
 * the same results bit for bit:
 *   1. the batch: rows drawn from the dataset arrays ray_org / ray_dir / targets ([num_src,3])
 *      as rm_sample_batch draws them (n_uniform + n_fg rows; seed, stream, counter);
 *   2. the render of the scene act_packed (activated packed parameters), the loss seed and the
 *      backward into grad_packed ((7M+4) floats, overwritten) and loss_sum (1 float, overwritten),
 *      as rm_train_step with progress, inv_count and march;
 *   3. the optimizer step on raw_packed / adam_m / adam_v (step, lr, weight_decay,
 *      with_penalties, loss_penalty nullable) writing the updated activated parameters back into
 *      act_packed, as rm_optimizer_step with act_out = act_packed.
 * Models of up to 32 spheres and batches of up to 16,384 rays run as ONE launch (the small-scene
 * kernel draws and gathers its rays, an extra block of the launch runs the optimizer's
 * gradient-independent part beside the ray blocks and the last block applies the update; env
 * RM_FUSED_ITER=0 turns this off); other sizes run the three calls. fp32 colour models only.
 * Not for data-parallel training: the gradient is consumed before it could be all-reduced. */
/* The data-parallel rank's step before its all-reduce (train.rs:179-190 on the rank's share of
 * the batch), replacing the sequence rm_sample_batch -> rm_train_step with the same arguments and
 * the same results bit for bit: the rows drawn from the dataset arrays as rm_sample_batch draws
 * them (n_uniform + n_fg rows; seed, stream, counter), then the render of `scene`, the loss seed
 * and the backward into `grads` and loss_sum (overwritten), as rm_train_step with progress,
 * inv_count and march (accumulate 0, no per-ray output). The gradient is left for the caller's
 * all-reduce and rm_optimizer_step[_f16]. Models of up to 32 spheres and batches of up to 16,384
 * rays run as ONE launch (the small-scene kernel draws and gathers its rays and its last block
 * completes the gradient; env RM_FUSED_ITER=0 turns this off); other sizes run the two calls. */
int rm_train_step_sampled(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                          int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform,
                          int64_t n_fg, uint64_t seed, uint64_t stream, uint64_t counter, float progress,
                          float inv_count, const rm_scene* scene, const rm_march* march, const rm_grads* grads,
                          float* loss_sum);

/* rm_train_step_sampled, and in the same launch the gradient-independent part of the optimizer
 * step that follows the all-reduce (penalties incl. the repulsion rows, the chain-rule factors,
 * Adam's bias corrections; loss_penalty (nullable) written here) on raw_packed / step /
 * with_penalties: the next rm_optimizer_step on this context with the same raw_packed,
 * num_spheres, step, with_penalties and loss_penalty then runs the update only -- the same bits
 * as without the preparation. The contents of raw_packed (and of the buffers the gradient comes
 * from) must not change between the two calls except through the caller's all-reduce of the
 * gradient: the library cannot see a host copy into raw_packed or a parameter broadcast, and the
 * update would use the factors prepared on the old values. Any other call of this library on the
 * context in between (every render, train, sampling, gather and activation entry point) drops the
 * preparation, as do different arguments: the optimizer step then computes everything itself. Models of
 * up to 32 spheres and batches of up to 16,384 rays (the one-launch case); otherwise it is
 * rm_train_step_sampled. Not with bound step scalars (rm_bind_step_scalars). */
int rm_train_step_sampled_prepared(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                                   int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform,
                                   int64_t n_fg, uint64_t seed, uint64_t stream, uint64_t counter, float progress,
                                   float inv_count, const rm_scene* scene, const rm_march* march,
                                   const rm_grads* grads, float* loss_sum, const float* raw_packed, int32_t step,
                                   int32_t with_penalties, float* loss_penalty);

int rm_train_iteration(rm_context* ctx, const float* ray_org, const float* ray_dir, const float* targets,
                       int64_t num_src, const int32_t* fg_indices, int64_t num_fg, int64_t n_uniform, int64_t n_fg,
                       uint64_t seed, uint64_t stream, uint64_t counter, float progress, float inv_count,
                       const rm_march* march, float* act_packed, float* grad_packed, float* raw_packed,
                       float* adam_m, float* adam_v, int32_t num_spheres, int32_t step, float lr,
                       float weight_decay, int32_t with_penalties, float* loss_sum, float* loss_penalty);

#ifdef __cplusplus
}
#endif

#endif /* RAYMARCH_H_ */
