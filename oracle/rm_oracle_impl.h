/*
 * rm_oracle_impl.h -- CPU restatement of kokutoupan/burn_raymarching's differentiable
 * render path (TEST INFRASTRUCTURE ONLY: the parity checker and the CPU baseline;
 * nothing in the product links or calls it).
 *
 * This header is included twice by rm_oracle.c, once with REAL=float (the
 * reference's fp32 arithmetic in the reference's op order) and once with
 * REAL=double (the fp64 restatement every tolerance is stated against).
 *
 * Every function cites the reference file:line it restates. The reference is
 * Rust on Burn 0.20.1 (Cargo.lock:516-519); its tensor ops are restated here
 * scalar-by-scalar with the same expansion-form distances, the same detached-max
 * log-sum-exp, the same 6-tap finite-difference normal and the same detach points.
 * The backward is the closed form of burn-autodiff over that graph (SURVEY.md
 * §8(a) a13); tests/test_oracle_autodiff.py pins it against torch fp64 autograd of
 * a literal op-by-op restatement (oracle/autodiff_ref.py).
 *
 * Parity pins: the forward is pinned by the reference's own fixtures
 * (steps/final_1.png <- scene.json via render_diff, data/target_*.png <- render);
 * the backward has no reference fixture and is pinned by autograd.
 */

#ifndef REAL
#error "define REAL before including rm_oracle_impl.h"
#endif

/* ---- math shims ------------------------------------------------------------- */
#define RF(x) ((REAL)(x))

/* camera.rs:7-14 math::normalize -- fp32 in the reference */
static void FN(normalize3)(const REAL v[3], REAL out[3]) {
  REAL len = SQRT(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (len == RF(0)) {
    out[0] = out[1] = out[2] = RF(0);
  } else {
    out[0] = v[0] / len;
    out[1] = v[1] / len;
    out[2] = v[2] / len;
  }
}

/* camera.rs:20-26 math::cross */
static void FN(cross3)(const REAL a[3], const REAL b[3], REAL out[3]) {
  out[0] = a[1] * b[2] - a[2] * b[1];
  out[1] = a[2] * b[0] - a[0] * b[2];
  out[2] = a[0] * b[1] - a[1] * b[0];
}

/* camera.rs:30-90 create_camera_rays: LookAt pinhole rays, row y then x,
 * u = x/W*2-1, v = -(y/H*2-1) (no half-pixel offset). */
void FN(orc_camera_rays)(int width, int height, const float eye_f[3], const float target_f[3],
                         float fov_deg, REAL* ray_org, REAL* ray_dir) {
  REAL eye[3] = {RF(eye_f[0]), RF(eye_f[1]), RF(eye_f[2])};
  REAL tgt[3] = {RF(target_f[0]), RF(target_f[1]), RF(target_f[2])};
  const REAL world_up[3] = {RF(0), RF(1), RF(0)};            /* camera.rs:41 */
  REAL fwd_raw[3] = {tgt[0] - eye[0], tgt[1] - eye[1], tgt[2] - eye[2]};
  REAL fwd[3], right_raw[3], right[3], up[3];
  FN(normalize3)(fwd_raw, fwd);                                /* camera.rs:42 */
  FN(cross3)(fwd, world_up, right_raw);
  FN(normalize3)(right_raw, right);                            /* camera.rs:43 */
  FN(cross3)(right, fwd, up);                                  /* camera.rs:44 */
  REAL aspect = (REAL)width / (REAL)height;                    /* camera.rs:48 */
  /* camera.rs:50: fov_deg.to_radians() / 2.0 ; Rust f32::to_radians = x * (PI/180) */
  REAL theta = RF(fov_deg) * (PI_R / RF(180)) / RF(2);
  REAL half_h = TAN(theta);                                    /* camera.rs:51 */
  REAL half_w = aspect * half_h;                               /* camera.rs:52 */
  for (int y = 0; y < height; ++y) {
    for (int x = 0; x < width; ++x) {
      REAL u = ((REAL)x / (REAL)width) * RF(2) - RF(1);        /* camera.rs:62 */
      REAL v = -(((REAL)y / (REAL)height) * RF(2) - RF(1));    /* camera.rs:63 */
      REAL rs = u * half_w, us = v * half_h;                   /* camera.rs:67-68 */
      REAL dx = right[0] * rs + up[0] * us + fwd[0];           /* camera.rs:70-72 */
      REAL dy = right[1] * rs + up[1] * us + fwd[1];
      REAL dz = right[2] * rs + up[2] * us + fwd[2];
      REAL len = SQRT(dx * dx + dy * dy + dz * dz);            /* camera.rs:75 */
      size_t i = ((size_t)y * width + x) * 3;
      ray_dir[i + 0] = dx / len;
      ray_dir[i + 1] = dy / len;
      ray_dir[i + 2] = dz / len;
      ray_org[i + 0] = eye[0];                                 /* camera.rs:83-85 */
      ray_org[i + 1] = eye[1];
      ray_org[i + 2] = eye[2];
    }
  }
}

/* ---- scene SDF ---------------------------------------------------------------- */

/* scene.rs:66-76: expansion-form distance of point p to sphere j:
 * sqrt(max(|p|^2 + |c|^2 - 2 p.c, 1e-6)) - r. Returns rho (before -r) and q. */
static inline REAL FN(rho_sq)(const REAL p[3], REAL psq, const REAL* c) {
  REAL csq = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];         /* scene.rs:68 */
  REAL pdc = p[0] * c[0] + p[1] * c[1] + p[2] * c[2];         /* scene.rs:69 (matmul) */
  return (psq + csq) - pdc * RF(2);                            /* scene.rs:71 */
}

/* sdf.rs:30-44 soft_min_tensor over the distances of p to all spheres
 * (scene.rs:60-79 scene_sdf_value). Also returns the detached max (of -k*dist)
 * and the clamped sum so the backward can form softmax(-k*dist). */
static REAL FN(scene_sdf)(const REAL p[3], const REAL* centers, const REAL* radius, int M, REAL k,
                          REAL* out_max, REAL* out_sum) {
  REAL psq = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];         /* scene.rs:67 */
  REAL mx = -INFINITY;
  for (int j = 0; j < M; ++j) {
    REAL q = FN(rho_sq)(p, psq, centers + 3 * j);
    REAL d = SQRT(FMAX(q, RF(1e-6))) - radius[j];              /* scene.rs:72-76 */
    REAL v = d * (-k);                                         /* sdf.rs:36 */
    if (v > mx) mx = v;                                        /* sdf.rs:37 (detached) */
  }
  REAL s = RF(0);
  for (int j = 0; j < M; ++j) {
    REAL q = FN(rho_sq)(p, psq, centers + 3 * j);
    REAL d = SQRT(FMAX(q, RF(1e-6))) - radius[j];
    s += EXP(d * (-k) - mx);                                   /* sdf.rs:39-40 */
  }
  REAL sc = FMAX(s, RF(1e-8));                                 /* sdf.rs:43 clamp_min */
  if (out_max) *out_max = mx;
  if (out_sum) *out_sum = sc;
  return (LOG(sc) + mx) / (-k);                                /* sdf.rs:43 */
}

/* ---- forward ------------------------------------------------------------------ */

typedef struct {
  REAL t;          /* march t after S detached steps (renderer_diff.rs:20-26) */
  REAL pa[3];      /* p_approx (renderer_diff.rs:30) */
  REAL amax, asum; /* soft-min normalizer at p_approx (for alpha = softmax(-k*dist_a)) */
  REAL tf;         /* t_final = t + dist_last (renderer_diff.rs:36) */
  REAL p[3];       /* p_final (renderer_diff.rs:39) */
  REAL n[3];       /* detached normal (renderer_diff.rs:41-46) */
  REAL dd[6];      /* the six tap distances (scene.rs:111) */
  REAL ldn[3], ldlen;
  REAL sdot, diff, L;
  REAL wmax, wsum;  /* colour softmax normalizer over -10*delta (renderer_diff.rs:74) */
  REAL mix[3];
  REAL bmax, bsum;  /* mask soft-min normalizer over -k*delta (renderer_diff.rs:86) */
  REAL Df, mu;
  REAL out[3];
} FN(RayFwd);

/* renderer_diff.rs:6-91 render_diff, one ray. */
static void FN(forward_ray)(const REAL o[3], const REAL d[3], const REAL* centers, const REAL* colors,
                            const REAL* radius, const REAL ld[3], REAL amb, int M, int steps, REAL k,
                            const REAL* t_in, FN(RayFwd) * f) {
  REAL t = RF(0);                                              /* renderer_diff.rs:20 */
  if (t_in) {
    t = *t_in;
  } else {
    for (int s = 0; s < steps; ++s) {                          /* renderer_diff.rs:22-26 */
      REAL p[3] = {o[0] + d[0] * t, o[1] + d[1] * t, o[2] + d[2] * t};
      t = t + FN(scene_sdf)(p, centers, radius, M, k, NULL, NULL);
    }
  }
  f->t = t;
  for (int i = 0; i < 3; ++i) f->pa[i] = o[i] + d[i] * t;      /* renderer_diff.rs:30 */
  REAL dlast = FN(scene_sdf)(f->pa, centers, radius, M, k, &f->amax, &f->asum); /* :33 */
  f->tf = t + dlast;                                           /* renderer_diff.rs:36 */
  for (int i = 0; i < 3; ++i) f->p[i] = o[i] + d[i] * f->tf;   /* renderer_diff.rs:39 */

  /* scene.rs:81-128 calc_normal_scene: taps +x,-x,+y,-y,+z,-z at eps = 1e-4 */
  const REAL eps = RF(1e-4f);
  REAL dd[6];
  for (int a = 0; a < 3; ++a) {
    for (int sgn = 0; sgn < 2; ++sgn) {
      REAL tap[3] = {f->p[0], f->p[1], f->p[2]};
      tap[a] = tap[a] + (sgn == 0 ? eps : -eps);               /* scene.rs:104 */
      dd[2 * a + sgn] = FN(scene_sdf)(tap, centers, radius, M, k, NULL, NULL);
    }
  }
  for (int q = 0; q < 6; ++q) f->dd[q] = dd[q];
  REAL nx = dd[0] - dd[1], ny = dd[2] - dd[3], nz = dd[4] - dd[5]; /* scene.rs:119-121 */
  REAL len = SQRT(nx * nx + ny * ny + nz * nz + RF(1e-6));    /* scene.rs:125 */
  f->n[0] = nx / len;
  f->n[1] = ny / len;
  f->n[2] = nz / len;

  /* renderer_diff.rs:48-62: lighting */
  REAL ldsq = ld[0] * ld[0] + ld[1] * ld[1] + ld[2] * ld[2];
  f->ldlen = SQRT(ldsq);
  for (int i = 0; i < 3; ++i) f->ldn[i] = ld[i] / f->ldlen;
  f->sdot = f->n[0] * f->ldn[0] + f->n[1] * f->ldn[1] + f->n[2] * f->ldn[2];
  f->diff = f->sdot > RF(0) ? f->sdot : RF(0);                 /* clamp_min(0.0) */
  f->L = amb + f->diff * (RF(1) - amb);

  /* renderer_diff.rs:65-84: softmax(-10*delta) colour blend; :86-90 mask */
  REAL psq = f->p[0] * f->p[0] + f->p[1] * f->p[1] + f->p[2] * f->p[2];
  REAL wmax = -INFINITY, bmax = -INFINITY;
  for (int j = 0; j < M; ++j) {
    REAL q = FN(rho_sq)(f->p, psq, centers + 3 * j);
    REAL dl = SQRT(FMAX(q, RF(1e-6))) - radius[j];
    REAL vw = dl * RF(-10), vb = dl * (-k);
    if (vw > wmax) wmax = vw;
    if (vb > bmax) bmax = vb;
  }
  REAL wsum = RF(0), bsum = RF(0), mix[3] = {RF(0), RF(0), RF(0)};
  for (int j = 0; j < M; ++j) {
    REAL q = FN(rho_sq)(f->p, psq, centers + 3 * j);
    REAL dl = SQRT(FMAX(q, RF(1e-6))) - radius[j];
    REAL ew = EXP(dl * RF(-10) - wmax);
    wsum += ew;
    bsum += EXP(dl * (-k) - bmax);
    for (int c = 0; c < 3; ++c) mix[c] += ew * colors[3 * j + c];
  }
  f->wmax = wmax;
  f->wsum = wsum;
  for (int c = 0; c < 3; ++c) f->mix[c] = mix[c] / wsum;      /* softmax then weighted sum */
  f->bmax = bmax;
  f->bsum = FMAX(bsum, RF(1e-8));
  f->Df = (LOG(f->bsum) + bmax) / (-k);                        /* scene_sdf_value(p_final) */
  f->mu = RF(1) / (RF(1) + EXP(-(f->Df * RF(-15))));           /* sigmoid(-15 D) */
  for (int c = 0; c < 3; ++c) f->out[c] = f->mix[c] * f->L * f->mu; /* :84, :90 */
}

/* ---- backward ------------------------------------------------------------------ */

typedef struct {
  REAL* gc;    /* [M,3] */
  REAL* gr;    /* [M]   */
  REAL* gcol;  /* [M,3] */
  REAL gell[3];/* sum over rays of dL/d(ld_norm), turned into dL/d(ld) at the end */
  REAL gamb;
} FN(GradAcc);

/* The burn-autodiff backward of render_diff for one ray:
 * seeds g_m = g L mu, g_L = (g.m) mu, g_mu = (g.m) L; colour softmax and mask
 * soft-min at p_final; reconnect through t_final = t + sdf(p_approx). The normal
 * (detached, renderer_diff.rs:41-46), t and p_approx (detached, :25, :30) carry no
 * gradient. */
static void FN(backward_ray)(const REAL d[3], const REAL* centers, const REAL* colors,
                             const REAL* radius, REAL amb, int M, REAL k, const FN(RayFwd) * f,
                             const REAL g[3], FN(GradAcc) * acc) {
  REAL gm[3], gdotm = g[0] * f->mix[0] + g[1] * f->mix[1] + g[2] * f->mix[2];
  for (int c = 0; c < 3; ++c) gm[c] = g[c] * f->L * f->mu;
  REAL gL = gdotm * f->mu;
  REAL gmu = gdotm * f->L;
  acc->gamb += gL * (RF(1) - f->diff);                         /* d L / d ambient */
  REAL gs = f->sdot >= RF(0) ? gL * (RF(1) - amb) : RF(0);     /* clamp_min passes at x >= 0 */
  for (int c = 0; c < 3; ++c) acc->gell[c] += gs * f->n[c];
  REAL cmu = gmu * f->mu * (RF(1) - f->mu) * RF(-15);
  REAL mg = f->mix[0] * gm[0] + f->mix[1] * gm[1] + f->mix[2] * gm[2];

  /* sweep at p_final: colour softmax + mask soft-min share delta_j */
  REAL psq = f->p[0] * f->p[0] + f->p[1] * f->p[1] + f->p[2] * f->p[2];
  REAL gp[3] = {RF(0), RF(0), RF(0)};
  for (int j = 0; j < M; ++j) {
    const REAL* c = centers + 3 * j;
    REAL q = FN(rho_sq)(f->p, psq, c);
    REAL rho = SQRT(FMAX(q, RF(1e-6)));
    REAL dl = rho - radius[j];
    REAL w = EXP(dl * RF(-10) - f->wmax) / f->wsum;
    REAL beta = EXP(dl * (-k) - f->bmax) / f->bsum;
    const REAL* col = colors + 3 * j;
    REAL cg = col[0] * gm[0] + col[1] * gm[1] + col[2] * gm[2];
    REAL gdl = RF(-10) * w * (cg - mg) + cmu * beta;
    for (int cc = 0; cc < 3; ++cc) acc->gcol[3 * j + cc] += w * gm[cc];
    acc->gr[j] -= gdl;
    if (q >= RF(1e-6)) {                                       /* clamp_min(1e-6) gate */
      for (int a = 0; a < 3; ++a) {
        REAL u = (f->p[a] - c[a]) / rho;
        gp[a] += gdl * u;
        acc->gc[3 * j + a] -= gdl * u;
      }
    }
  }
  /* reconnect: p = o + d * (t + D(p_a)) -> dL/dD(p_a) = g_p . d */
  REAL gt = gp[0] * d[0] + gp[1] * d[1] + gp[2] * d[2];
  REAL pasq = f->pa[0] * f->pa[0] + f->pa[1] * f->pa[1] + f->pa[2] * f->pa[2];
  for (int j = 0; j < M; ++j) {
    const REAL* c = centers + 3 * j;
    REAL q = FN(rho_sq)(f->pa, pasq, c);
    REAL rho = SQRT(FMAX(q, RF(1e-6)));
    REAL dl = rho - radius[j];
    REAL alpha = EXP(dl * (-k) - f->amax) / f->asum;
    REAL h = gt * alpha;
    acc->gr[j] -= h;
    if (q >= RF(1e-6)) {
      for (int a = 0; a < 3; ++a) acc->gc[3 * j + a] -= h * (f->pa[a] - c[a]) / rho;
    }
  }
}

/* training.rs:17-34 compute_loss reconstruction term: mean(|out - tgt| * W), W = 10 where
 * sum(tgt) > 0.01 else 1 + 4*progress. Returns sum(|diff|*W) for the ray and writes
 * g = W*sign(diff)*inv_count (inv_count = 1/(3N) for the mean). */
static REAL FN(loss_seed)(const REAL out[3], const REAL tgt[3], REAL progress, REAL inv_count, REAL g[3]) {
  REAL tsum = tgt[0] + tgt[1] + tgt[2];
  REAL W = tsum > RF(0.01f) ? RF(10) : RF(1) + progress * RF(4);
  REAL l = RF(0);
  for (int c = 0; c < 3; ++c) {
    REAL df = out[c] - tgt[c];
    l += FABS(df) * W;
    REAL sg = df > RF(0) ? RF(1) : (df < RF(0) ? RF(-1) : RF(0));
    g[c] = W * sg * inv_count;
  }
  return l;
}

/* ---- batched entry points (OpenMP over rays) --------------------------------- */

static void FN(finish_light)(const REAL ld[3], const REAL gell[3], REAL gld[3]) {
  REAL ldsq = ld[0] * ld[0] + ld[1] * ld[1] + ld[2] * ld[2];
  REAL len = SQRT(ldsq);
  REAL ldn[3] = {ld[0] / len, ld[1] / len, ld[2] / len};
  REAL proj = ldn[0] * gell[0] + ldn[1] * gell[1] + ldn[2] * gell[2];
  for (int c = 0; c < 3; ++c) gld[c] = (gell[c] - ldn[c] * proj) / len;
}

/* Forward over N rays (render_diff). t_march (nullable) receives the detached march t. */
void FN(orc_render_diff)(long n, const REAL* org, const REAL* dir, const REAL* centers, const REAL* colors,
                         const REAL* radius, const REAL* ld, const REAL* amb, int M, int steps, REAL k,
                         REAL* out, REAL* t_march) {
#pragma omp parallel for schedule(dynamic, 64)
  for (long i = 0; i < n; ++i) {
    FN(RayFwd) f;
    FN(forward_ray)(org + 3 * i, dir + 3 * i, centers, colors, radius, ld, amb[0], M, steps, k, NULL, &f);
    for (int c = 0; c < 3; ++c) out[3 * i + c] = f.out[c];
    if (t_march) t_march[i] = f.t;
  }
}

/* Diagnostics twin of rm_debug_intermediates: dbg [N][24] = {t, t_final, n, lighting, mix,
 * D_final, mask, n.l, min delta, Zw (shifted at min delta), Zb (shifted), 0}. */
void FN(orc_render_diff_debug)(long n, const REAL* org, const REAL* dir, const REAL* centers, const REAL* colors,
                               const REAL* radius, const REAL* ld, const REAL* amb, int M, int steps, REAL k,
                               REAL* dbg) {
#pragma omp parallel for schedule(dynamic, 64)
  for (long i = 0; i < n; ++i) {
    FN(RayFwd) f;
    FN(forward_ray)(org + 3 * i, dir + 3 * i, centers, colors, radius, ld, amb[0], M, steps, k, NULL, &f);
    REAL* q = dbg + 24 * i;
    q[0] = f.t; q[1] = f.tf; q[2] = f.n[0]; q[3] = f.n[1]; q[4] = f.n[2]; q[5] = f.L;
    q[6] = f.mix[0]; q[7] = f.mix[1]; q[8] = f.mix[2]; q[9] = f.Df; q[10] = f.mu; q[11] = f.sdot;
    q[12] = f.wmax / RF(-10); q[13] = f.wsum; q[14] = f.bsum; q[15] = RF(0);
    for (int t = 0; t < 6; ++t) q[16 + t] = f.dd[t];
    q[22] = q[23] = RF(0);
  }
}

/* Shared body of backward / train step. mode 0: g given (grad_out); mode 1: loss seed
 * from targets. Gradients are OVERWRITTEN. loss_sum (mode 1) receives sum |diff|*W. */
static void FN(bwd_common)(long n, const REAL* org, const REAL* dir, const REAL* centers, const REAL* colors,
                           const REAL* radius, const REAL* ld, const REAL* amb, int M, int steps, REAL k,
                           const REAL* t_march, int mode, const REAL* grad_out, const REAL* targets,
                           REAL progress, REAL inv_count, REAL* out, REAL* loss_sum, REAL* gc, REAL* gr,
                           REAL* gcol, REAL* gld, REAL* gamb) {
  memset(gc, 0, sizeof(REAL) * 3 * M);
  memset(gr, 0, sizeof(REAL) * M);
  memset(gcol, 0, sizeof(REAL) * 3 * M);
  REAL gell[3] = {RF(0), RF(0), RF(0)}, gamb_tot = RF(0), loss_tot = RF(0);
#pragma omp parallel
  {
    FN(GradAcc) acc;
    acc.gc = (REAL*)calloc((size_t)3 * M, sizeof(REAL));
    acc.gr = (REAL*)calloc((size_t)M, sizeof(REAL));
    acc.gcol = (REAL*)calloc((size_t)3 * M, sizeof(REAL));
    acc.gell[0] = acc.gell[1] = acc.gell[2] = RF(0);
    acc.gamb = RF(0);
    REAL lacc = RF(0);
#pragma omp for schedule(static)
    for (long i = 0; i < n; ++i) {
      FN(RayFwd) f;
      FN(forward_ray)(org + 3 * i, dir + 3 * i, centers, colors, radius, ld, amb[0], M, steps, k,
                      t_march ? t_march + i : NULL, &f);
      REAL g[3];
      if (mode == 0) {
        for (int c = 0; c < 3; ++c) g[c] = grad_out[3 * i + c];
      } else {
        lacc += FN(loss_seed)(f.out, targets + 3 * i, progress, inv_count, g);
      }
      if (out)
        for (int c = 0; c < 3; ++c) out[3 * i + c] = f.out[c];
      FN(backward_ray)(dir + 3 * i, centers, colors, radius, amb[0], M, k, &f, g, &acc);
    }
#pragma omp critical
    {
      for (int j = 0; j < 3 * M; ++j) gc[j] += acc.gc[j];
      for (int j = 0; j < M; ++j) gr[j] += acc.gr[j];
      for (int j = 0; j < 3 * M; ++j) gcol[j] += acc.gcol[j];
      for (int c = 0; c < 3; ++c) gell[c] += acc.gell[c];
      gamb_tot += acc.gamb;
      loss_tot += lacc;
    }
    free(acc.gc);
    free(acc.gr);
    free(acc.gcol);
  }
  FN(finish_light)(ld, gell, gld);
  gamb[0] = gamb_tot;
  if (loss_sum) loss_sum[0] = loss_tot;
}

/* Backward of render_diff given g = dL/dout [N,3]. */
void FN(orc_render_diff_backward)(long n, const REAL* org, const REAL* dir, const REAL* centers,
                                  const REAL* colors, const REAL* radius, const REAL* ld, const REAL* amb,
                                  int M, int steps, REAL k, const REAL* t_march, const REAL* grad_out,
                                  REAL* gc, REAL* gr, REAL* gcol, REAL* gld, REAL* gamb) {
  FN(bwd_common)(n, org, dir, centers, colors, radius, ld, amb, M, steps, k, t_march, 0, grad_out, NULL,
                 RF(0), RF(0), NULL, NULL, gc, gr, gcol, gld, gamb);
}

/* Fused train step: forward + training.rs:17-34 seed + backward. */
void FN(orc_train_step)(long n, const REAL* org, const REAL* dir, const REAL* targets, REAL progress,
                        REAL inv_count, const REAL* centers, const REAL* colors, const REAL* radius,
                        const REAL* ld, const REAL* amb, int M, int steps, REAL k, REAL* out, REAL* loss_sum,
                        REAL* gc, REAL* gr, REAL* gcol, REAL* gld, REAL* gamb) {
  FN(bwd_common)(n, org, dir, centers, colors, radius, ld, amb, M, steps, k, NULL, 1, NULL, targets,
                 progress, inv_count, out, loss_sum, gc, gr, gcol, gld, gamb);
}

/* renderer.rs:4-80 render (non-differentiable target renderer used by generate.rs):
 * 40 steps at k=32, fixed light (-0.5,0.5,-1)/|.|, lighting = diffuse + 0.1,
 * normalized exp(-10 d) colour weights (+1e-5), mask exp(-10 D^2). */
void FN(orc_render)(long n, const REAL* org, const REAL* dir, const REAL* centers, const REAL* colors,
                    const REAL* radius, int M, REAL* out) {
  const REAL k = RF(32);
#pragma omp parallel for schedule(dynamic, 64)
  for (long i = 0; i < n; ++i) {
    const REAL* o = org + 3 * i;
    const REAL* d = dir + 3 * i;
    REAL t = RF(0);
    for (int s = 0; s < 40; ++s) {                             /* renderer.rs:17-21 */
      REAL p[3] = {o[0] + d[0] * t, o[1] + d[1] * t, o[2] + d[2] * t};
      t = t + FN(scene_sdf)(p, centers, radius, M, k, NULL, NULL);
    }
    REAL p[3] = {o[0] + d[0] * t, o[1] + d[1] * t, o[2] + d[2] * t};
    const REAL eps = RF(1e-4f);
    REAL dd[6];
    for (int a = 0; a < 3; ++a)
      for (int sg = 0; sg < 2; ++sg) {
        REAL tap[3] = {p[0], p[1], p[2]};
        tap[a] = tap[a] + (sg == 0 ? eps : -eps);
        dd[2 * a + sg] = FN(scene_sdf)(tap, centers, radius, M, k, NULL, NULL);
      }
    REAL nx = dd[0] - dd[1], ny = dd[2] - dd[3], nz = dd[4] - dd[5];
    REAL len = SQRT(nx * nx + ny * ny + nz * nz + RF(1e-6));
    REAL n3[3] = {nx / len, ny / len, nz / len};
    /* renderer.rs:27-32: light normalized on the host in f32 */
    float lv[3] = {-0.5f, 0.5f, -1.0f};
    float llen = sqrtf(powf(lv[0], 2.0f) + powf(lv[1], 2.0f) + powf(lv[2], 2.0f));
    REAL ln[3] = {RF(lv[0] / llen), RF(lv[1] / llen), RF(lv[2] / llen)};
    REAL diffuse = n3[0] * ln[0] + n3[1] * ln[1] + n3[2] * ln[2];
    if (diffuse < RF(0)) diffuse = RF(0);                      /* renderer.rs:38 */
    REAL lighting = diffuse + RF(0.1f);                        /* renderer.rs:40 */
    REAL psq = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
    REAL csum[3] = {RF(0), RF(0), RF(0)}, wsum = RF(0);
    for (int j = 0; j < M; ++j) {
      REAL q = FN(rho_sq)(p, psq, centers + 3 * j);
      REAL dl = SQRT(FMAX(q, RF(1e-6))) - radius[j];
      REAL w = EXP(dl * RF(-10));                              /* renderer.rs:52 */
      wsum += w;
      for (int c = 0; c < 3; ++c) csum[c] += colors[3 * j + c] * w;
    }
    wsum = wsum + RF(1e-5f);                                   /* renderer.rs:68 */
    REAL Ds = FN(scene_sdf)(p, centers, radius, M, k, NULL, NULL);
    REAL mask = EXP(Ds * Ds * RF(-10));                        /* renderer.rs:77 */
    for (int c = 0; c < 3; ++c) out[3 * i + c] = (csum[c] / wsum) * lighting * mask;
  }
}

#undef RF
