/*
 * rm_oracle.c -- TEST INFRASTRUCTURE: the CPU restatement of the reference's
 * differentiable render path, compiled twice (fp32 in the reference's op order,
 * fp64 as the tolerance anchor). Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product
 * (libraymarch_hip.so) never links or calls it.
 *
 * Reference: /root/reference/src/{camera.rs, model/scene.rs, model/sdf.rs,
 * renderer_diff.rs, renderer.rs, training.rs} (kokutoupan/burn_raymarching).
 * Parity pins: forward by the reference fixtures steps/final_1.png and
 * data/target_*.png (tests/golden/); backward by torch fp64 autograd of a
 * literal op-by-op restatement (oracle/autodiff_ref.py); Adam unpinned.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>

/* fp32 instantiation: reference arithmetic (Rust f32 == IEEE binary32, libm) */
#define REAL float
#define FN(name) name##_f32
#define SQRT sqrtf
#define EXP expf
#define LOG logf
#define TAN tanf
#define FMAX fmaxf
#define FABS fabsf
#define PI_R 3.14159265358979323846f
#include "rm_oracle_impl.h"
#undef REAL
#undef FN
#undef SQRT
#undef EXP
#undef LOG
#undef TAN
#undef FMAX
#undef FABS
#undef PI_R

/* fp64 instantiation: the anchor every fp32 tolerance is stated against */
#define REAL double
#define FN(name) name##_f64
#define SQRT sqrt
#define EXP exp
#define LOG log
#define TAN tan
#define FMAX fmax
#define FABS fabs
#define PI_R 3.14159265358979323846
#include "rm_oracle_impl.h"

int orc_version(void) { return 1; }

/* OpenMP threads of the parallel loops (bench.py's cpu_baseline times 1 and n threads). */
#include <omp.h>
void orc_set_threads(int n) { omp_set_num_threads(n > 0 ? n : 1); }
int orc_max_threads(void) { return omp_get_max_threads(); }
