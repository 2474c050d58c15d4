/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- the checker, never the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code.  The product library (ilqg-mujoco_amd/) never links it.
 *
 * Plain-C (C99) restatement of the MuJoCo 2.0 forward-dynamics pipeline that
 * the reference's hot path calls through libmujoco200:
 *   mj_forward / mj_forwardSkip  -- call sites /root/reference/src/mjderivative.cpp:64,68,92,103,124,134,178,198
 *   mj_step                       -- call sites /root/reference/inc/ilqr.h:86,128
 * Restricted to the features used by res/{inverted_pendulum,hopper,humanoid}.xml
 * (SURVEY.md Appendix B): slide/hinge/ball/free joints, CRB mass matrix with
 * MuJoCo's tree LDL', RNE bias, joint springs/dampers, motors, joint limits,
 * plane/sphere/capsule contacts with pyramidal cones, the primal Newton
 * constraint solver, semi-implicit Euler with implicit joint damping, and RK4.
 *
 * MuJoCo 2.0 is closed source and absent here, so agreement with the real
 * engine is PARITY UNPINNED.  What IS pinned: the reference's
 * own FD driver (src/mjderivative.cpp, util.cpp) compiled unmodified against
 * this file (oracle/Makefile -> oracle/_ref/) must reproduce the oracle's FD
 * restatement bit for bit, and the GPU kernels must reproduce this file.
 *
 * Arithmetic contract (shared with the HIP kernels so results can be bit
 * exact): IEEE fp64, no FMA contraction (-ffp-contract=off), sums taken in
 * ascending index order exactly as written here, sin/cos from the fdlibm
 * kernels below (ora_sin/ora_cos), sqrt and division correctly rounded.
 */
#define _POSIX_C_SOURCE 200112L
#include "mujoco/mujoco.h"
#include "ilqg_model_blob.h"
#include "ilqg_model_fields.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* line-search constants of the restated Newton solver */
#define ORA_LS_ITER 50
#ifdef ORA_LS_STUDY /* tools/ls_study (a study build; liboracle.so never defines it) */
void ora_ls_study_begin(int ne, const double* Jv, const double* jar, const double* D, double g1, double g2,
                        double d1, double d2, double gtol);
void ora_ls_study_iter(int it, int bisect, double lo, double hi, double alpha, double d1, double d2);
void ora_ls_study_end(void);
#endif
#ifdef ORA_NT_STUDY
void ora_nt_study_iter(int ne, const double* jar, const double* Jv, double alpha, const int* state);
#endif
#define ORA_LS_TOL 0.01

/* ------------------------------------------------------------------------- */
/* utilities                                                                  */

void mju_error(const char* msg) {
  fprintf(stderr, "ORACLE ERROR: %s\n", msg);
  exit(1);
}
void mju_error_s(const char* msg, const char* text) {
  fprintf(stderr, "ORACLE ERROR: ");
  fprintf(stderr, msg, text);
  fprintf(stderr, "\n");
  exit(1);
}
void* mju_malloc(size_t size) {
  void* p = NULL;
  if (posix_memalign(&p, 64, size ? size : 8)) mju_error("mju_malloc failed");
  return p;
}
void mju_free(void* ptr) { free(ptr); }
void mju_copy(mjtNum* res, const mjtNum* data, int n) {
  if (n > 0) memcpy(res, data, (size_t)n * sizeof(mjtNum));
}
void mju_zero(mjtNum* res, int n) {
  if (n > 0) memset(res, 0, (size_t)n * sizeof(mjtNum));
}
int mj_activate(const char* filename) { (void)filename; return 1; }
void mj_deactivate(void) {}

/* ---- deterministic sin/cos: fdlibm/musl kernels, Cody-Waite pi/2 reduction */
static const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                    S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                    S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
static const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                    C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                    C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
static const double INVPIO2 = 6.36619772367581382433e-01, PIO2_1 = 1.57079632673412561417e+00,
                    PIO2_1T = 6.07710050650619224932e-11, PIO4 = 7.85398163397448278999e-01;

static double k_sin(double x, double y, int iy) {
  double z = x * x, w = z * z;
  double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  double v = z * x;
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
static double k_cos(double x, double y) {
  double z = x * x, w = z * z;
  double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}
static int rem_pio2(double x, double* y0, double* y1) {
  double fn = floor(x * INVPIO2 + 0.5);
  double r = x - fn * PIO2_1;
  double w = fn * PIO2_1T;
  *y0 = r - w;
  *y1 = (r - *y0) - w;
  return (int)fn;
}
mjtNum ora_sin(mjtNum x) {
  double y0, y1;
  int n;
  ORA_FLOP_TRANS();
  if (fabs(x) < PIO4) return x == 0 ? x : k_sin((double)x, 0.0, 0);
  n = rem_pio2((double)x, &y0, &y1);
  switch (n & 3) {
    case 0: return k_sin(y0, y1, 1);
    case 1: return k_cos(y0, y1);
    case 2: return -k_sin(y0, y1, 1);
    default: return -k_cos(y0, y1);
  }
}
mjtNum ora_cos(mjtNum x) {
  double y0, y1;
  int n;
  ORA_FLOP_TRANS();
  if (fabs(x) < PIO4) return k_cos((double)x, 0.0);
  n = rem_pio2((double)x, &y0, &y1);
  switch (n & 3) {
    case 0: return k_cos(y0, y1);
    case 1: return -k_sin(y0, y1, 1);
    case 2: return -k_cos(y0, y1);
    default: return k_sin(y0, y1, 1);
  }
}

/* ---- small vector / quaternion algebra (MuJoCo engine_util_* semantics) */
static inline mjtNum dot3(const mjtNum* a, const mjtNum* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
static inline mjtNum dotn(const mjtNum* a, const mjtNum* b, int n) {
  mjtNum r = 0;
  for (int i = 0; i < n; i++) r += a[i] * b[i];
  return r;
}
static inline void cross3(mjtNum* r, const mjtNum* a, const mjtNum* b) {
  mjtNum t0 = a[1] * b[2] - a[2] * b[1];
  mjtNum t1 = a[2] * b[0] - a[0] * b[2];
  mjtNum t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static mjtNum normalize3(mjtNum* v) {
  mjtNum norm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (norm < mjMINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0;
  } else {
    mjtNum inv = 1 / norm;
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
  }
  return norm;
}
static void normalize4(mjtNum* q) {
  mjtNum norm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (norm < mjMINVAL) {
    q[0] = 1; q[1] = 0; q[2] = 0; q[3] = 0;
  } else if (fabs(norm - 1) > mjMINVAL) {
    mjtNum inv = 1 / norm;
    q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
  }
}
static void quat_mul(mjtNum* r, const mjtNum* a, const mjtNum* b) {
  mjtNum t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  mjtNum t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  mjtNum t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  mjtNum t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
static void rot_vec_quat(mjtNum* r, const mjtNum* v, const mjtNum* q) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) {
    r[0] = r[1] = r[2] = 0;
  } else if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2];
  } else {
    mjtNum t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
    mjtNum t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
    mjtNum t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
    mjtNum r0 = v[0] + 2 * (q[2] * t2 - q[3] * t1);
    mjtNum r1 = v[1] + 2 * (q[3] * t0 - q[1] * t2);
    mjtNum r2 = v[2] + 2 * (q[1] * t1 - q[2] * t0);
    r[0] = r0; r[1] = r1; r[2] = r2;
  }
}
static void quat2mat(mjtNum* r, const mjtNum* q) {
  if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = 1; r[1] = 0; r[2] = 0; r[3] = 0; r[4] = 1; r[5] = 0; r[6] = 0; r[7] = 0; r[8] = 1;
    return;
  }
  mjtNum q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  mjtNum q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  mjtNum q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  r[0] = q00 + q11 - q22 - q33;
  r[4] = q00 - q11 + q22 - q33;
  r[8] = q00 - q11 - q22 + q33;
  r[1] = 2 * (q12 - q03);
  r[2] = 2 * (q13 + q02);
  r[3] = 2 * (q12 + q03);
  r[5] = 2 * (q23 - q01);
  r[6] = 2 * (q13 - q02);
  r[7] = 2 * (q23 + q01);
}
static void axis_angle2quat(mjtNum* r, const mjtNum* axis, mjtNum angle) {
  if (angle == 0) {
    r[0] = 1; r[1] = 0; r[2] = 0; r[3] = 0;
  } else {
    mjtNum s = ora_sin(angle * 0.5);
    r[0] = ora_cos(angle * 0.5);
    r[1] = axis[0] * s; r[2] = axis[1] * s; r[3] = axis[2] * s;
  }
}
static void rot_vec_mat(mjtNum* r, const mjtNum* v, const mjtNum* m) {
  mjtNum r0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  mjtNum r1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  mjtNum r2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
void mju_quatIntegrate(mjtNum quat[4], const mjtNum vel[3], mjtNum scale) {
  mjtNum tmp[3] = {vel[0], vel[1], vel[2]}, qrot[4];
  mjtNum angle = scale * normalize3(tmp);
  axis_angle2quat(qrot, tmp, angle);
  normalize4(quat);
  quat_mul(quat, quat, qrot);
}
/* contact frame from its normal (first row), MuJoCo mju_makeFrame */
static void make_frame(mjtNum* f) {
  mjtNum tmp[3], d;
  normalize3(f);
  f[3] = f[4] = f[5] = 0;
  if (fabs(f[1]) < 0.5) f[4] = 1; else f[5] = 1;
  d = dot3(f, f + 3);
  tmp[0] = f[0] * d; tmp[1] = f[1] * d; tmp[2] = f[2] * d;
  f[3] -= tmp[0]; f[4] -= tmp[1]; f[5] -= tmp[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}
/* spatial algebra: cinert 10-vector, motion/force 6-vectors [ang, lin] */
static void inert_com(mjtNum* res, const mjtNum* in, const mjtNum* mat, const mjtNum* dif, mjtNum mass) {
  mjtNum tmp[9] = {mat[0] * in[0], mat[3] * in[0], mat[6] * in[0],
                   mat[1] * in[1], mat[4] * in[1], mat[7] * in[1],
                   mat[2] * in[2], mat[5] * in[2], mat[8] * in[2]};
  res[0] = mat[0] * tmp[0] + mat[1] * tmp[3] + mat[2] * tmp[6];
  res[1] = mat[3] * tmp[1] + mat[4] * tmp[4] + mat[5] * tmp[7];
  res[2] = mat[6] * tmp[2] + mat[7] * tmp[5] + mat[8] * tmp[8];
  res[3] = mat[0] * tmp[1] + mat[1] * tmp[4] + mat[2] * tmp[7];
  res[4] = mat[0] * tmp[2] + mat[1] * tmp[5] + mat[2] * tmp[8];
  res[5] = mat[3] * tmp[2] + mat[4] * tmp[5] + mat[5] * tmp[8];
  res[0] += mass * (dif[1] * dif[1] + dif[2] * dif[2]);
  res[1] += mass * (dif[0] * dif[0] + dif[2] * dif[2]);
  res[2] += mass * (dif[0] * dif[0] + dif[1] * dif[1]);
  res[3] -= mass * dif[0] * dif[1];
  res[4] -= mass * dif[0] * dif[2];
  res[5] -= mass * dif[1] * dif[2];
  res[6] = mass * dif[0];
  res[7] = mass * dif[1];
  res[8] = mass * dif[2];
  res[9] = mass;
}
static void mul_inert_vec(mjtNum* r, const mjtNum* i, const mjtNum* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
static void cross_motion(mjtNum* r, const mjtNum* vel, const mjtNum* v) {
  r[0] = -vel[2] * v[1] + vel[1] * v[2];
  r[1] = vel[2] * v[0] - vel[0] * v[2];
  r[2] = -vel[1] * v[0] + vel[0] * v[1];
  r[3] = -vel[2] * v[4] + vel[1] * v[5];
  r[4] = vel[2] * v[3] - vel[0] * v[5];
  r[5] = -vel[1] * v[3] + vel[0] * v[4];
  r[3] += -vel[5] * v[1] + vel[4] * v[2];
  r[4] += vel[5] * v[0] - vel[3] * v[2];
  r[5] += -vel[4] * v[0] + vel[3] * v[1];
}
static void cross_force(mjtNum* r, const mjtNum* vel, const mjtNum* f) {
  r[0] = -vel[2] * f[1] + vel[1] * f[2];
  r[1] = vel[2] * f[0] - vel[0] * f[2];
  r[2] = -vel[1] * f[0] + vel[0] * f[1];
  r[3] = -vel[2] * f[4] + vel[1] * f[5];
  r[4] = vel[2] * f[3] - vel[0] * f[5];
  r[5] = -vel[1] * f[3] + vel[0] * f[4];
  r[0] += -vel[5] * f[4] + vel[4] * f[5];
  r[1] += vel[5] * f[3] - vel[3] * f[5];
  r[2] += -vel[4] * f[3] + vel[3] * f[4];
}
static void dof_com(mjtNum* r, const mjtNum* axis, const mjtNum* offset) {
  if (offset) {
    r[0] = axis[0]; r[1] = axis[1]; r[2] = axis[2];
    cross3(r + 3, axis, offset);
  } else {
    r[0] = r[1] = r[2] = 0;
    r[3] = axis[0]; r[4] = axis[1]; r[5] = axis[2];
  }
}
/* res = sum_j mat[6j..6j+5]*vec[j], j ascending */
static void mul_dof_vec(mjtNum* r, const mjtNum* mat, const mjtNum* vec, int n) {
  for (int k = 0; k < 6; k++) {
    mjtNum s = 0;
    for (int j = 0; j < n; j++) s += mat[6 * j + k] * vec[j];
    r[k] = s;
  }
}

/* ------------------------------------------------------------------------- */
/* model record -> mjModel                                                    */

typedef struct { const char* name; int dtype; int count; const void* data; } blob_field;

static const blob_field* find_field(const blob_field* f, int n, const char* name) {
  for (int i = 0; i < n; i++)
    if (!strcmp(f[i].name, name)) return f + i;
  return NULL;
}

mjModel* mj_loadBlob(const void* blob, size_t nbytes, char* error, int error_sz) {
  const unsigned char* p = (const unsigned char*)blob;
  const unsigned char* end = p + nbytes;
  int32_t nfield;
  blob_field* fields;
  mjModel* m;
  size_t total = 0, off = 0;
  char* arena;
  if (nbytes < 16 || memcmp(p, ILQG_BLOB_MAGIC, 8)) {
    snprintf(error, error_sz, "bad model record magic");
    return NULL;
  }
  memcpy(&nfield, p + 8, 4);
  p += 16;
  fields = (blob_field*)calloc((size_t)nfield, sizeof(blob_field));
  for (int i = 0; i < nfield; i++) {
    ilqg_blob_field_hdr h;
    size_t sz;
    if (p + sizeof(h) > end) { snprintf(error, error_sz, "truncated record"); free(fields); return NULL; }
    memcpy(&h, p, sizeof(h));
    p += sizeof(h);
    sz = (size_t)h.count * (h.dtype == ILQG_BLOB_F64 ? 8 : 4);
    fields[i].name = (const char*)(p - sizeof(h));
    fields[i].dtype = h.dtype;
    fields[i].count = h.count;
    fields[i].data = p;
    p += (sz + 7) & ~(size_t)7;
  }
  m = (mjModel*)calloc(1, sizeof(mjModel));

#define GET_I32(nm) do { const blob_field* f_ = find_field(fields, nfield, #nm); \
    if (!f_ || f_->dtype != ILQG_BLOB_I32 || f_->count != 1) { snprintf(error, error_sz, "missing %s", #nm); goto fail; } \
    memcpy(&i32_##nm, f_->data, 4); } while (0)
#define GET_F64(nm) do { const blob_field* f_ = find_field(fields, nfield, #nm); \
    if (!f_ || f_->dtype != ILQG_BLOB_F64 || f_->count != 1) { snprintf(error, error_sz, "missing %s", #nm); goto fail; } \
    memcpy(&f64_##nm, f_->data, 8); } while (0)
#define DECL_I32(nm) int32_t i32_##nm = 0;
#define DECL_F64(nm) double f64_##nm = 0;
  {
    ILQG_MODEL_I32_SCALARS(DECL_I32)
    ILQG_MODEL_F64_SCALARS(DECL_F64)
#define DO_I32(nm) GET_I32(nm);
#define DO_F64(nm) GET_F64(nm);
    ILQG_MODEL_I32_SCALARS(DO_I32)
    ILQG_MODEL_F64_SCALARS(DO_F64)
    m->nq = i32_nq; m->nv = i32_nv; m->nu = i32_nu; m->na = 0;
    m->nbody = i32_nbody; m->njnt = i32_njnt; m->ngeom = i32_ngeom;
    m->nconmax = i32_nconmax; m->njmax = i32_njmax; m->nstack = i32_nstack;
    m->opt.integrator = i32_opt_integrator; m->opt.cone = i32_opt_cone;
    m->opt.solver = i32_opt_solver; m->opt.iterations = i32_opt_iterations;
    m->opt.disableflags = i32_opt_disableflags; m->opt.enableflags = i32_opt_enableflags;
    m->opt.timestep = f64_opt_timestep; m->opt.impratio = f64_opt_impratio;
    m->opt.tolerance = f64_opt_tolerance;
    m->opt.gravity[0] = f64_opt_gravity0; m->opt.gravity[1] = f64_opt_gravity1;
    m->opt.gravity[2] = f64_opt_gravity2;
    m->stat.meaninertia = f64_stat_meaninertia;
  }
  {
    int nq = m->nq, nv = m->nv, nu = m->nu, nbody = m->nbody, njnt = m->njnt, ngeom = m->ngeom;
#define SZ_F(nm, cnt) total += (size_t)(cnt) * 8;
#define SZ_I(nm, cnt) total += (((size_t)(cnt) * 4 + 7) & ~(size_t)7);
    ILQG_MODEL_F64_ARRAYS(SZ_F)
    ILQG_MODEL_I32_ARRAYS(SZ_I)
    arena = (char*)calloc(1, total + 8);
    m->_arena = arena;
#define LD_F(nm, cnt) do { const blob_field* f_ = find_field(fields, nfield, #nm); \
      if (!f_ || f_->dtype != ILQG_BLOB_F64 || f_->count != (int)(cnt)) { snprintf(error, error_sz, "bad field %s", #nm); goto fail; } \
      m->nm = (mjtNum*)(arena + off); memcpy(m->nm, f_->data, (size_t)(cnt) * 8); off += (size_t)(cnt) * 8; } while (0);
#define LD_I(nm, cnt) do { const blob_field* f_ = find_field(fields, nfield, #nm); \
      if (!f_ || f_->dtype != ILQG_BLOB_I32 || f_->count != (int)(cnt)) { snprintf(error, error_sz, "bad field %s", #nm); goto fail; } \
      m->nm = (int*)(arena + off); memcpy(m->nm, f_->data, (size_t)(cnt) * 4); off += (((size_t)(cnt) * 4 + 7) & ~(size_t)7); } while (0);
    ILQG_MODEL_F64_ARRAYS(LD_F)
    ILQG_MODEL_I32_ARRAYS(LD_I)
    (void)nq; (void)nv; (void)nu; (void)nbody; (void)njnt; (void)ngeom;
  }
  free(fields);
  /* arena size of mjData, computed by the same layout routine makeData uses */
  {
    extern size_t ora_data_layout(const mjModel* m, mjData* d, char* base);
    m->nbuffer = (int)ora_data_layout(m, NULL, NULL);
  }
  return m;
fail:
  free(fields);
  free(m->_arena);
  free(m);
  return NULL;
}

void mj_deleteModel(mjModel* m) {
  if (!m) return;
  free(m->_arena);
  free(m);
}

/* ------------------------------------------------------------------------- */
/* mjData arena: one buffer, zeroed on reset (MuJoCo 2.0 mj_makeData/resetData) */

size_t ora_data_layout(const mjModel* m, mjData* d, char* base) {
  size_t off = 0;
  int nq = m->nq, nv = m->nv, nu = m->nu, nb = m->nbody, nj = m->njnt, ng = m->ngeom;
  int nc = m->nconmax, ne = m->njmax;
#define AL(field, type, cnt) do { if (d) d->field = (type*)(base + off); \
    off += (((size_t)(cnt) * sizeof(type)) + 63) & ~(size_t)63; } while (0)
  /* qpos, qvel, act contiguous (MuJoCo layout; ilqr.h:90 relies on it) */
  if (d) {
    d->qpos = (mjtNum*)(base + off);
    d->qvel = d->qpos + nq;
    d->act = d->qvel + nv;
  }
  off += (((size_t)(nq + nv) * 8) + 63) & ~(size_t)63;
  AL(qacc_warmstart, mjtNum, nv);
  AL(ctrl, mjtNum, nu);
  AL(qfrc_applied, mjtNum, nv);
  AL(xfrc_applied, mjtNum, 6 * nb);
  AL(qacc, mjtNum, nv);
  AL(xpos, mjtNum, 3 * nb); AL(xquat, mjtNum, 4 * nb); AL(xmat, mjtNum, 9 * nb);
  AL(xipos, mjtNum, 3 * nb); AL(ximat, mjtNum, 9 * nb);
  AL(xanchor, mjtNum, 3 * nj); AL(xaxis, mjtNum, 3 * nj);
  AL(geom_xpos, mjtNum, 3 * ng); AL(geom_xmat, mjtNum, 9 * ng);
  AL(subtree_com, mjtNum, 3 * nb);
  AL(cdof, mjtNum, 6 * nv);
  AL(cinert, mjtNum, 10 * nb);
  AL(crb, mjtNum, 10 * nb);
  AL(qM, mjtNum, nv * nv);
  AL(qLD, mjtNum, nv * nv);
  AL(qLDiagInv, mjtNum, nv);
  AL(actuator_moment, mjtNum, nu * nv);
  AL(actuator_length, mjtNum, nu);
  AL(contact, mjContact, nc);
  AL(efc_type, int, ne); AL(efc_id, int, ne);
  AL(efc_J, mjtNum, (size_t)ne * nv);
  AL(efc_pos, mjtNum, ne); AL(efc_margin, mjtNum, ne); AL(efc_diagApprox, mjtNum, ne);
  AL(efc_R, mjtNum, ne); AL(efc_D, mjtNum, ne); AL(efc_KBIP, mjtNum, 4 * ne);
  AL(efc_AR, mjtNum, (size_t)ne * ne);
  AL(cvel, mjtNum, 6 * nb); AL(cdof_dot, mjtNum, 6 * nv);
  AL(qfrc_passive, mjtNum, nv); AL(qfrc_bias, mjtNum, nv);
  AL(efc_vel, mjtNum, ne); AL(efc_aref, mjtNum, ne);
  AL(actuator_force, mjtNum, nu); AL(qfrc_actuator, mjtNum, nv);
  AL(qfrc_smooth, mjtNum, nv); AL(qacc_smooth, mjtNum, nv); AL(qfrc_constraint, mjtNum, nv);
  AL(efc_force, mjtNum, ne); AL(efc_b, mjtNum, ne); AL(efc_state, int, ne);
  AL(stack, mjtNum, m->nstack);
#undef AL
  return off;
}

void mj_resetData(const mjModel* m, mjData* d) {
  memset(d->buffer, 0, (size_t)m->nbuffer);
  d->pstack = 0;
  d->maxuse_stack = 0;
  d->ncon = 0;
  d->nefc = 0;
  d->solver_iter = 0;
  d->time = 0;
  mju_copy(d->qpos, m->qpos0, m->nq);
}

mjData* mj_makeData(const mjModel* m) {
  mjData* d = (mjData*)calloc(1, sizeof(mjData));
  d->nstack = m->nstack;
  d->nbuffer = m->nbuffer;
  d->buffer = mju_malloc((size_t)m->nbuffer);
  ora_data_layout(m, d, (char*)d->buffer);
  mj_resetData(m, d);
  return d;
}

void mj_deleteData(mjData* d) {
  if (!d) return;
  mju_free(d->buffer);
  free(d);
}

mjtNum* mj_stackAlloc(mjData* d, int size) {
  mjtNum* r;
  if (!size) return 0;
  if (d->pstack + size > d->nstack) mju_error("mj_stackAlloc: stack overflow");
  r = d->stack + d->pstack;
  d->pstack += size;
  if (d->pstack > d->maxuse_stack) d->maxuse_stack = d->pstack;
  return r;
}

/* ------------------------------------------------------------------------- */
/* position stage                                                             */

static void kinematics(const mjModel* m, mjData* d) {
  d->xpos[0] = d->xpos[1] = d->xpos[2] = 0;
  d->xquat[0] = 1; d->xquat[1] = d->xquat[2] = d->xquat[3] = 0;
  quat2mat(d->xmat, d->xquat);
  d->xipos[0] = d->xipos[1] = d->xipos[2] = 0;
  quat2mat(d->ximat, d->xquat);

  for (int i = 1; i < m->nbody; i++) {
    int pid = m->body_parentid[i];
    mjtNum xpos[3], xquat[4], tmp[3], qloc[4];
    rot_vec_quat(tmp, m->body_pos + 3 * i, d->xquat + 4 * pid);
    xpos[0] = d->xpos[3 * pid] + tmp[0];
    xpos[1] = d->xpos[3 * pid + 1] + tmp[1];
    xpos[2] = d->xpos[3 * pid + 2] + tmp[2];
    quat_mul(xquat, d->xquat + 4 * pid, m->body_quat + 4 * i);

    for (int j = 0; j < m->body_jntnum[i]; j++) {
      int jid = m->body_jntadr[i] + j;
      int qadr = m->jnt_qposadr[jid];
      int type = m->jnt_type[jid];
      mjtNum* xanchor = d->xanchor + 3 * jid;
      mjtNum* xaxis = d->xaxis + 3 * jid;
      if (type == mjJNT_FREE) {
        xpos[0] = d->qpos[qadr]; xpos[1] = d->qpos[qadr + 1]; xpos[2] = d->qpos[qadr + 2];
        xquat[0] = d->qpos[qadr + 3]; xquat[1] = d->qpos[qadr + 4];
        xquat[2] = d->qpos[qadr + 5]; xquat[3] = d->qpos[qadr + 6];
        normalize4(xquat);
        xanchor[0] = xpos[0]; xanchor[1] = xpos[1]; xanchor[2] = xpos[2];
        xaxis[0] = m->jnt_axis[3 * jid]; xaxis[1] = m->jnt_axis[3 * jid + 1];
        xaxis[2] = m->jnt_axis[3 * jid + 2];
        continue;
      }
      rot_vec_quat(xanchor, m->jnt_pos + 3 * jid, xquat);
      xanchor[0] += xpos[0]; xanchor[1] += xpos[1]; xanchor[2] += xpos[2];
      rot_vec_quat(xaxis, m->jnt_axis + 3 * jid, xquat);
      if (type == mjJNT_SLIDE) {
        mjtNum dq = d->qpos[qadr] - m->qpos0[qadr];
        xpos[0] += xaxis[0] * dq; xpos[1] += xaxis[1] * dq; xpos[2] += xaxis[2] * dq;
      } else {
        if (type == mjJNT_BALL) {
          qloc[0] = d->qpos[qadr]; qloc[1] = d->qpos[qadr + 1];
          qloc[2] = d->qpos[qadr + 2]; qloc[3] = d->qpos[qadr + 3];
          normalize4(qloc);
        } else {
          axis_angle2quat(qloc, m->jnt_axis + 3 * jid, d->qpos[qadr] - m->qpos0[qadr]);
        }
        quat_mul(xquat, xquat, qloc);
        rot_vec_quat(tmp, m->jnt_pos + 3 * jid, xquat);
        xpos[0] = xanchor[0] - tmp[0];
        xpos[1] = xanchor[1] - tmp[1];
        xpos[2] = xanchor[2] - tmp[2];
      }
    }
    normalize4(xquat);
    mju_copy(d->xpos + 3 * i, xpos, 3);
    mju_copy(d->xquat + 4 * i, xquat, 4);
    quat2mat(d->xmat + 9 * i, xquat);
    /* inertial frame */
    rot_vec_mat(tmp, m->body_ipos + 3 * i, d->xmat + 9 * i);
    d->xipos[3 * i] = tmp[0] + xpos[0];
    d->xipos[3 * i + 1] = tmp[1] + xpos[1];
    d->xipos[3 * i + 2] = tmp[2] + xpos[2];
    quat_mul(qloc, xquat, m->body_iquat + 4 * i);
    quat2mat(d->ximat + 9 * i, qloc);
  }
  for (int g = 0; g < m->ngeom; g++) {
    int b = m->geom_bodyid[g];
    mjtNum tmp[3], q[4];
    rot_vec_mat(tmp, m->geom_pos + 3 * g, d->xmat + 9 * b);
    d->geom_xpos[3 * g] = tmp[0] + d->xpos[3 * b];
    d->geom_xpos[3 * g + 1] = tmp[1] + d->xpos[3 * b + 1];
    d->geom_xpos[3 * g + 2] = tmp[2] + d->xpos[3 * b + 2];
    quat_mul(q, d->xquat + 4 * b, m->geom_quat + 4 * g);
    quat2mat(d->geom_xmat + 9 * g, q);
  }
}

static void com_pos(const mjModel* m, mjData* d) {
  int nb = m->nbody;
  for (int i = 0; i < nb; i++) {
    d->subtree_com[3 * i] = d->xipos[3 * i] * m->body_mass[i];
    d->subtree_com[3 * i + 1] = d->xipos[3 * i + 1] * m->body_mass[i];
    d->subtree_com[3 * i + 2] = d->xipos[3 * i + 2] * m->body_mass[i];
  }
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    d->subtree_com[3 * p] += d->subtree_com[3 * i];
    d->subtree_com[3 * p + 1] += d->subtree_com[3 * i + 1];
    d->subtree_com[3 * p + 2] += d->subtree_com[3 * i + 2];
  }
  for (int i = 0; i < nb; i++) {
    if (m->body_subtreemass[i] < mjMINVAL) {
      mju_copy(d->subtree_com + 3 * i, d->xipos + 3 * i, 3);
    } else {
      mjtNum inv = 1 / m->body_subtreemass[i];
      d->subtree_com[3 * i] *= inv;
      d->subtree_com[3 * i + 1] *= inv;
      d->subtree_com[3 * i + 2] *= inv;
    }
  }
  mju_zero(d->cinert, 10);
  for (int i = 1; i < nb; i++) {
    mjtNum off[3];
    const mjtNum* rc = d->subtree_com + 3 * m->body_rootid[i];
    off[0] = d->xipos[3 * i] - rc[0];
    off[1] = d->xipos[3 * i + 1] - rc[1];
    off[2] = d->xipos[3 * i + 2] - rc[2];
    inert_com(d->cinert + 10 * i, m->body_inertia + 3 * i, d->ximat + 9 * i, off, m->body_mass[i]);
  }
  for (int j = 0; j < m->njnt; j++) {
    int da = 6 * m->jnt_dofadr[j];
    int bi = m->jnt_bodyid[j];
    const mjtNum* rc = d->subtree_com + 3 * m->body_rootid[bi];
    mjtNum off[3] = {rc[0] - d->xanchor[3 * j], rc[1] - d->xanchor[3 * j + 1],
                     rc[2] - d->xanchor[3 * j + 2]};
    int skip = 0;
    switch (m->jnt_type[j]) {
      case mjJNT_FREE:
        mju_zero(d->cdof + da, 18);
        for (int i = 0; i < 3; i++) d->cdof[da + 3 + 7 * i] = 1;
        skip = 18;
        /* fall through */
      case mjJNT_BALL:
        for (int i = 0; i < 3; i++) {
          mjtNum axis[3] = {d->xmat[9 * bi + i], d->xmat[9 * bi + i + 3], d->xmat[9 * bi + i + 6]};
          dof_com(d->cdof + da + skip + 6 * i, axis, off);
        }
        break;
      case mjJNT_SLIDE:
        dof_com(d->cdof + da, d->xaxis + 3 * j, NULL);
        break;
      default:
        dof_com(d->cdof + da, d->xaxis + 3 * j, off);
        break;
    }
  }
}

/* composite rigid body: dense qM (both triangles) */
static void crb(const mjModel* m, mjData* d) {
  int nv = m->nv;
  mju_copy(d->crb, d->cinert, 10 * m->nbody);
  for (int i = m->nbody - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[10 * p + k] += d->crb[10 * i + k];
  }
  mju_zero(d->qM, nv * nv);
  for (int i = 0; i < nv; i++) {
    mjtNum buf[6];
    d->qM[i * nv + i] = m->dof_armature[i];
    mul_inert_vec(buf, d->crb + 10 * m->dof_bodyid[i], d->cdof + 6 * i);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) d->qM[i * nv + j] += dotn(d->cdof + 6 * j, buf, 6);
  }
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < i; j++) d->qM[j * nv + i] = d->qM[i * nv + j];
}

/* MuJoCo's tree L'DL factorization (mj_factorI) on a dense matrix; only the
   lower triangle of `mat` over ancestor pairs is used. */
static void factor_ld(const mjModel* m, const mjtNum* mat, mjtNum* LD, mjtNum* diaginv) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) LD[i * nv + j] = (j <= i) ? mat[i * nv + j] : 0;
  for (int k = nv - 1; k >= 0; k--) {
    if (LD[k * nv + k] < mjMINVAL) LD[k * nv + k] = mjMINVAL;
    for (int i = m->dof_parentid[k]; i >= 0; i = m->dof_parentid[i]) {
      mjtNum tmp = LD[k * nv + i] / LD[k * nv + k];
      for (int j = i; j >= 0; j = m->dof_parentid[j]) LD[i * nv + j] -= tmp * LD[k * nv + j];
      LD[k * nv + i] = tmp;
    }
  }
  for (int i = 0; i < nv; i++) diaginv[i] = 1 / LD[i * nv + i];
}

/* x <- inv(L'DL) x, MuJoCo mj_solveLD */
static void solve_ld(const mjModel* m, const mjtNum* LD, const mjtNum* diaginv, mjtNum* x) {
  int nv = m->nv;
  for (int i = nv - 1; i >= 0; i--) {
    mjtNum tmp = x[i];
    if (tmp != 0)
      for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) x[j] -= LD[i * nv + j] * tmp;
  }
  for (int i = 0; i < nv; i++) x[i] *= diaginv[i];
  for (int i = 0; i < nv; i++)
    for (int j = m->dof_parentid[i]; j >= 0; j = m->dof_parentid[j]) x[i] -= LD[i * nv + j] * x[j];
}

static void mul_m(int nv, const mjtNum* M, const mjtNum* vec, mjtNum* res) {
  for (int i = 0; i < nv; i++) res[i] = dotn(M + i * nv, vec, nv);
}

/* point jacobian (3 x nv, row major) of `point` attached to `body` */
static void jac_point(const mjModel* m, const mjData* d, mjtNum* jacp, const mjtNum* point, int body) {
  int nv = m->nv;
  mjtNum off[3];
  const mjtNum* rc = d->subtree_com + 3 * m->body_rootid[body];
  mju_zero(jacp, 3 * nv);
  off[0] = point[0] - rc[0]; off[1] = point[1] - rc[1]; off[2] = point[2] - rc[2];
  while (body && !m->body_dofnum[body]) body = m->body_parentid[body];
  if (!body) return;
  for (int i = m->body_dofadr[body] + m->body_dofnum[body] - 1; i >= 0; i = m->dof_parentid[i]) {
    mjtNum tmp[3];
    const mjtNum* cd = d->cdof + 6 * i;
    cross3(tmp, cd, off);
    jacp[i] = cd[3] + tmp[0];
    jacp[nv + i] = cd[4] + tmp[1];
    jacp[2 * nv + i] = cd[5] + tmp[2];
  }
}
static void jac_rot(const mjModel* m, const mjData* d, mjtNum* jacr, int body) {
  int nv = m->nv;
  mju_zero(jacr, 3 * nv);
  while (body && !m->body_dofnum[body]) body = m->body_parentid[body];
  if (!body) return;
  for (int i = m->body_dofadr[body] + m->body_dofnum[body] - 1; i >= 0; i = m->dof_parentid[i]) {
    jacr[i] = d->cdof[6 * i];
    jacr[nv + i] = d->cdof[6 * i + 1];
    jacr[2 * nv + i] = d->cdof[6 * i + 2];
  }
}

/* ---- collision: narrow phase ---- */
static int sphere_sphere(mjContact* c, mjtNum margin, const mjtNum* p1, mjtNum r1,
                         const mjtNum* p2, mjtNum r2) {
  mjtNum axis[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  mjtNum dist = normalize3(axis) - r1 - r2;
  mjtNum s;
  if (dist > margin) return 0;
  c->dist = dist;
  c->frame[0] = axis[0]; c->frame[1] = axis[1]; c->frame[2] = axis[2];
  s = r1 + dist / 2;
  c->pos[0] = p1[0] + axis[0] * s;
  c->pos[1] = p1[1] + axis[1] * s;
  c->pos[2] = p1[2] + axis[2] * s;
  return 1;
}
static int plane_sphere(mjContact* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                        const mjtNum* p2, mjtNum r2) {
  mjtNum n[3] = {mat1[2], mat1[5], mat1[8]};
  mjtNum tmp[3] = {p2[0] - pos1[0], p2[1] - pos1[1], p2[2] - pos1[2]};
  mjtNum cdist = dot3(tmp, n), s;
  if (cdist > margin + r2) return 0;
  c->dist = cdist - r2;
  c->frame[0] = n[0]; c->frame[1] = n[1]; c->frame[2] = n[2];
  s = -c->dist / 2 - r2;
  c->pos[0] = p2[0] + n[0] * s;
  c->pos[1] = p2[1] + n[1] * s;
  c->pos[2] = p2[2] + n[2] * s;
  return 1;
}
static mjtNum clip(mjtNum x, mjtNum lo, mjtNum hi) { return x < lo ? lo : (x > hi ? hi : x); }

static int narrow(const mjModel* m, const mjData* d, int g1, int g2, mjtNum margin, mjContact* con) {
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const mjtNum *pos1 = d->geom_xpos + 3 * g1, *mat1 = d->geom_xmat + 9 * g1, *sz1 = m->geom_size + 3 * g1;
  const mjtNum *pos2 = d->geom_xpos + 3 * g2, *mat2 = d->geom_xmat + 9 * g2, *sz2 = m->geom_size + 3 * g2;
  if (t1 == mjGEOM_PLANE && t2 == mjGEOM_SPHERE) return plane_sphere(con, margin, pos1, mat1, pos2, sz2[0]);
  if (t1 == mjGEOM_PLANE && t2 == mjGEOM_CAPSULE) {
    mjtNum seg[3] = {mat2[2] * sz2[1], mat2[5] * sz2[1], mat2[8] * sz2[1]}, p[3];
    int n1, n2;
    p[0] = pos2[0] + seg[0]; p[1] = pos2[1] + seg[1]; p[2] = pos2[2] + seg[2];
    n1 = plane_sphere(con, margin, pos1, mat1, p, sz2[0]);
    p[0] = pos2[0] - seg[0]; p[1] = pos2[1] - seg[1]; p[2] = pos2[2] - seg[2];
    n2 = plane_sphere(con + n1, margin, pos1, mat1, p, sz2[0]);
    return n1 + n2;
  }
  if (t1 == mjGEOM_SPHERE && t2 == mjGEOM_SPHERE) return sphere_sphere(con, margin, pos1, sz1[0], pos2, sz2[0]);
  if (t1 == mjGEOM_SPHERE && t2 == mjGEOM_CAPSULE) {
    mjtNum ax[3] = {mat2[2], mat2[5], mat2[8]}, dif[3], p[3], x;
    dif[0] = pos1[0] - pos2[0]; dif[1] = pos1[1] - pos2[1]; dif[2] = pos1[2] - pos2[2];
    x = clip(dot3(ax, dif), -sz2[1], sz2[1]);
    p[0] = pos2[0] + ax[0] * x; p[1] = pos2[1] + ax[1] * x; p[2] = pos2[2] + ax[2] * x;
    return sphere_sphere(con, margin, pos1, sz1[0], p, sz2[0]);
  }
  if (t1 == mjGEOM_CAPSULE && t2 == mjGEOM_CAPSULE) {
    mjtNum a1[3] = {mat1[2] * sz1[1], mat1[5] * sz1[1], mat1[8] * sz1[1]};
    mjtNum a2[3] = {mat2[2] * sz2[1], mat2[5] * sz2[1], mat2[8] * sz2[1]};
    mjtNum dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
    mjtNum ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    mjtNum u = -dot3(a1, dif), v = dot3(a2, dif);
    mjtNum det = ma * mc - mb * mb;
    mjtNum v1[3], v2[3], x1, x2;
    if (fabs(det) >= mjMINVAL) {
      x1 = (mc * u - mb * v) / det;
      x2 = (ma * v - mb * u) / det;
      if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
      else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
      if (x2 > 1) { x2 = 1; x1 = clip((u - mb) / ma, -1, 1); }
      else if (x2 < -1) { x2 = -1; x1 = clip((u + mb) / ma, -1, 1); }
      v1[0] = pos1[0] + a1[0] * x1; v1[1] = pos1[1] + a1[1] * x1; v1[2] = pos1[2] + a1[2] * x1;
      v2[0] = pos2[0] + a2[0] * x2; v2[1] = pos2[1] + a2[1] * x2; v2[2] = pos2[2] + a2[2] * x2;
      return sphere_sphere(con, margin, v1, sz1[0], v2, sz2[0]);
    } else {
      int n1, n2;
      v1[0] = pos1[0] + a1[0]; v1[1] = pos1[1] + a1[1]; v1[2] = pos1[2] + a1[2];
      x2 = clip((v - mb) / mc, -1, 1);
      v2[0] = pos2[0] + a2[0] * x2; v2[1] = pos2[1] + a2[1] * x2; v2[2] = pos2[2] + a2[2] * x2;
      n1 = sphere_sphere(con, margin, v1, sz1[0], v2, sz2[0]);
      v1[0] = pos1[0] - a1[0]; v1[1] = pos1[1] - a1[1]; v1[2] = pos1[2] - a1[2];
      x2 = clip((v + mb) / mc, -1, 1);
      v2[0] = pos2[0] + a2[0] * x2; v2[1] = pos2[1] + a2[1] * x2; v2[2] = pos2[2] + a2[2] * x2;
      n2 = sphere_sphere(con + n1, margin, v1, sz1[0], v2, sz2[0]);
      return n1 + n2;
    }
  }
  return 0; /* pair type not needed by the supported models */
}

static void collision(const mjModel* m, mjData* d) {
  int ng = m->ngeom;
  d->ncon = 0;
  for (int g1 = 0; g1 < ng; g1++)
    for (int g2 = g1 + 1; g2 < ng; g2++) {
      int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
      int w1 = m->body_weldid[b1], w2 = m->body_weldid[b2];
      int wp1 = m->body_weldid[m->body_parentid[w1]], wp2 = m->body_weldid[m->body_parentid[w2]];
      int ga = g1, gb = g2, n;
      mjtNum margin, gap, mix, s1, s2;
      mjContact tmp[4];
      if (w1 == w2) continue;
      if (w1 != 0 && w2 != 0 && (w1 == wp2 || w2 == wp1)) continue;
      if (!((m->geom_contype[g1] & m->geom_conaffinity[g2]) ||
            (m->geom_contype[g2] & m->geom_conaffinity[g1])))
        continue;
      margin = mjMAX(m->geom_margin[g1], m->geom_margin[g2]);
      if (m->geom_rbound[g1] > 0 && m->geom_rbound[g2] > 0) {
        const mjtNum *p1 = d->geom_xpos + 3 * g1, *p2 = d->geom_xpos + 3 * g2;
        mjtNum dd[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
        if (sqrt(dot3(dd, dd)) > m->geom_rbound[g1] + m->geom_rbound[g2] + margin) continue;
      }
      if (m->geom_type[g1] > m->geom_type[g2]) { ga = g2; gb = g1; }
      n = narrow(m, d, ga, gb, margin, tmp);
      if (!n) continue;
      gap = mjMAX(m->geom_gap[ga], m->geom_gap[gb]);
      s1 = m->geom_solmix[ga]; s2 = m->geom_solmix[gb];
      if (s1 < mjMINVAL && s2 < mjMINVAL) mix = 0.5;
      else if (s1 < mjMINVAL) mix = 0;
      else if (s2 < mjMINVAL) mix = 1;
      else mix = s1 / (s1 + s2);
      for (int k = 0; k < n; k++) {
        mjContact* c;
        const mjtNum *f1 = m->geom_friction + 3 * ga, *f2 = m->geom_friction + 3 * gb;
        if (d->ncon >= m->nconmax) break;
        c = d->contact + d->ncon;
        *c = tmp[k];
        c->geom1 = ga;
        c->geom2 = gb;
        c->dim = mjMAX(m->geom_condim[ga], m->geom_condim[gb]);
        c->includemargin = margin - gap;
        c->friction[0] = mjMAX(f1[0], f2[0]);
        c->friction[1] = c->friction[0];
        c->friction[2] = mjMAX(f1[1], f2[1]);
        c->friction[3] = mjMAX(f1[2], f2[2]);
        c->friction[4] = c->friction[3];
        for (int r = 0; r < mjNREF; r++)
          c->solref[r] = mix * m->geom_solref[2 * ga + r] + (1 - mix) * m->geom_solref[2 * gb + r];
        for (int r = 0; r < mjNIMP; r++)
          c->solimp[r] = mix * m->geom_solimp[5 * ga + r] + (1 - mix) * m->geom_solimp[5 * gb + r];
        make_frame(c->frame);
        c->efc_address = -1;
        d->ncon++;
      }
    }
}

/* ---- constraints ---- */
static mjtNum get_impedance(const mjtNum* solimp, mjtNum pos, mjtNum margin) {
  mjtNum dmin = clip(solimp[0], mjMINIMP, mjMAXIMP), dmax = clip(solimp[1], mjMINIMP, mjMAXIMP);
  mjtNum width = solimp[2], mid = solimp[3], power = solimp[4], x, y, imp;
  if (dmin == dmax || width <= mjMINVAL) return 0.5 * (dmin + dmax);
  x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  {
    /* integer powers by repeated multiplication (power 2 is the MuJoCo default) */
    int p = (int)(double)power;
    mjtNum xp = 1, mp = 1;
    if ((mjtNum)p != power || p < 1 || p > 8) mju_error("solimp power must be an integer in [1,8]");
    if (x <= mid) {
      for (int k = 0; k < p; k++) xp *= x;
      for (int k = 0; k < p - 1; k++) mp *= mid;
      y = xp / mp;
    } else {
      mjtNum xm = 1 - x, mm = 1 - mid;
      for (int k = 0; k < p; k++) xp *= xm;
      for (int k = 0; k < p - 1; k++) mp *= mm;
      y = 1 - xp / mp;
    }
  }
  imp = dmin + y * (dmax - dmin);
  return clip(imp, mjMINIMP, mjMAXIMP);
}

static int add_row(const mjModel* m, mjData* d, const mjtNum* jac, mjtNum pos, mjtNum margin,
                   int type, int id) {
  int r = d->nefc;
  mju_copy(d->efc_J + (size_t)r * m->nv, jac, m->nv);
  d->efc_pos[r] = pos;
  d->efc_margin[r] = margin;
  d->efc_type[r] = type;
  d->efc_id[r] = id;
  d->nefc++;
  return r;
}

static void make_constraint(const mjModel* m, mjData* d) {
  int nv = m->nv;
  mjMARKSTACK
  mjtNum* jac = mj_stackAlloc(d, nv);
  mjtNum* j1 = mj_stackAlloc(d, 3 * nv);
  mjtNum* j2 = mj_stackAlloc(d, 3 * nv);
  mjtNum* jc = mj_stackAlloc(d, 3 * nv);
  d->nefc = 0;
  /* joint limits */
  for (int j = 0; j < m->njnt; j++) {
      int type = m->jnt_type[j];
      mjtNum value;
      if (!m->jnt_limited[j] || (type != mjJNT_SLIDE && type != mjJNT_HINGE)) continue;
      value = d->qpos[m->jnt_qposadr[j]];
      for (int side = -1; side <= 1; side += 2) {
        mjtNum dist = side * (m->jnt_range[2 * j + (side + 1) / 2] - value);
        if (dist < m->jnt_margin[j]) {
          if (d->nefc + 1 > m->njmax) break;
          mju_zero(jac, nv);
          jac[m->jnt_dofadr[j]] = -side;
          add_row(m, d, jac, dist, m->jnt_margin[j], mjCNSTR_LIMIT_JOINT, j);
        }
      }
    }
  /* contacts */
  for (int c = 0; c < d->ncon; c++) {
    mjContact* con = d->contact + c;
    int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
    int nrow = con->dim == 1 ? 1 : 2 * (con->dim - 1);
    if (d->nefc + nrow > m->njmax) continue;
    jac_point(m, d, j1, con->pos, b1);
    jac_point(m, d, j2, con->pos, b2);
    for (int k = 0; k < 3 * nv; k++) j2[k] -= j1[k];
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < nv; k++)
        jc[r * nv + k] = con->frame[3 * r] * j2[k] + con->frame[3 * r + 1] * j2[nv + k] +
                         con->frame[3 * r + 2] * j2[2 * nv + k];
    con->efc_address = d->nefc;
    if (con->dim == 1) {
      add_row(m, d, jc, con->dist, con->includemargin, mjCNSTR_CONTACT_FRICTIONLESS, c);
    } else {
      for (int k = 1; k < con->dim; k++) {
        mjtNum fr = con->friction[k - 1];
        for (int i = 0; i < nv; i++) jac[i] = jc[i] + fr * jc[k * nv + i];
        add_row(m, d, jac, con->dist, con->includemargin, mjCNSTR_CONTACT_PYRAMIDAL, c);
        for (int i = 0; i < nv; i++) jac[i] = jc[i] + (-fr) * jc[k * nv + i];
        add_row(m, d, jac, con->dist, con->includemargin, mjCNSTR_CONTACT_PYRAMIDAL, c);
      }
    }
  }
  /* impedance, reference-acceleration gains, regularizer */
  for (int i = 0; i < d->nefc; i++) {
    const mjtNum *solref, *solimp;
    mjtNum dA, imp, tc, dr, dmax, K, B;
    int id = d->efc_id[i];
    if (d->efc_type[i] == mjCNSTR_LIMIT_JOINT) {
      solref = m->jnt_solref + 2 * id;
      solimp = m->jnt_solimp + 5 * id;
      dA = m->dof_invweight0[m->jnt_dofadr[id]];
    } else {
      mjContact* con = d->contact + id;
      int b1 = m->geom_bodyid[con->geom1], b2 = m->geom_bodyid[con->geom2];
      mjtNum tran = m->body_invweight0[2 * b1] + m->body_invweight0[2 * b2];
      solref = con->solref;
      solimp = con->solimp;
      if (d->efc_type[i] == mjCNSTR_CONTACT_FRICTIONLESS) {
        dA = tran;
      } else {
        int k = (i - con->efc_address) / 2; /* friction dimension of this pyramid edge */
        mjtNum fr = con->friction[k];
        dA = tran + fr * fr * tran;
      }
    }
    imp = get_impedance(solimp, d->efc_pos[i], d->efc_margin[i]);
    dmax = clip(solimp[1], mjMINIMP, mjMAXIMP);
    tc = solref[0];
    dr = solref[1];
    if (tc > 0) {
      if (tc < 2 * m->opt.timestep) tc = 2 * m->opt.timestep;
      K = 1 / (dmax * dmax * tc * tc * dr * dr);
      B = 2 / (dmax * tc);
    } else {
      K = -tc / (dmax * dmax);
      B = -dr / dmax;
    }
    d->efc_KBIP[4 * i] = K;
    d->efc_KBIP[4 * i + 1] = B;
    d->efc_KBIP[4 * i + 2] = imp;
    d->efc_KBIP[4 * i + 3] = 0;
    d->efc_diagApprox[i] = dA;
    d->efc_R[i] = mjMAX(mjMINVAL, (1 - imp) * dA / imp);
    d->efc_D[i] = 1 / d->efc_R[i];
  }
  mjFREESTACK
}

static void transmission(const mjModel* m, mjData* d) {
  int nv = m->nv;
  mju_zero(d->actuator_moment, m->nu * nv);
  for (int i = 0; i < m->nu; i++) {
    int j = m->actuator_trnid[i];
    d->actuator_moment[i * nv + m->jnt_dofadr[j]] = m->actuator_gear[i];
    d->actuator_length[i] = d->qpos[m->jnt_qposadr[j]] * m->actuator_gear[i];
  }
}

static void fwd_position(const mjModel* m, mjData* d) {
  kinematics(m, d);
  com_pos(m, d);
  transmission(m, d);
  crb(m, d);
  factor_ld(m, d->qM, d->qLD, d->qLDiagInv);
  collision(m, d);
  make_constraint(m, d);
}

/* ------------------------------------------------------------------------- */
/* velocity stage                                                             */

static void com_vel(const mjModel* m, mjData* d) {
  mju_zero(d->cvel, 6);
  for (int i = 1; i < m->nbody; i++) {
    int bda = m->body_dofadr[i];
    mjtNum cvel[6], tmp[6];
    mju_copy(cvel, d->cvel + 6 * m->body_parentid[i], 6);
    for (int j = 0; j < m->body_dofnum[i]; j++) {
      switch (m->jnt_type[m->dof_jntid[bda + j]]) {
        case mjJNT_FREE:
          mju_zero(d->cdof_dot + 6 * (bda + j), 18);
          mul_dof_vec(tmp, d->cdof + 6 * bda, d->qvel + bda, 3);
          for (int k = 0; k < 6; k++) cvel[k] += tmp[k];
          j += 3;
          /* fall through */
        case mjJNT_BALL:
          for (int k = 0; k < 3; k++)
            cross_motion(d->cdof_dot + 6 * (bda + j + k), cvel, d->cdof + 6 * (bda + j + k));
          mul_dof_vec(tmp, d->cdof + 6 * (bda + j), d->qvel + bda + j, 3);
          for (int k = 0; k < 6; k++) cvel[k] += tmp[k];
          j += 2;
          break;
        default:
          cross_motion(d->cdof_dot + 6 * (bda + j), cvel, d->cdof + 6 * (bda + j));
          mul_dof_vec(tmp, d->cdof + 6 * (bda + j), d->qvel + bda + j, 1);
          for (int k = 0; k < 6; k++) cvel[k] += tmp[k];
      }
    }
    mju_copy(d->cvel + 6 * i, cvel, 6);
  }
}

static void sub_quat(mjtNum* res, const mjtNum* qa, const mjtNum* qb) {
  /* res = 3D rotation vector of qb^-1 * qa */
  mjtNum qneg[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, qdif[4], s, ang;
  quat_mul(qdif, qneg, qa);
  res[0] = qdif[1]; res[1] = qdif[2]; res[2] = qdif[3];
  s = normalize3(res);
  ang = 2 * atan2(s, qdif[0]);
  if (ang > mjPI) ang -= 2 * mjPI;
  res[0] *= ang; res[1] *= ang; res[2] *= ang;
}

static void passive(const mjModel* m, mjData* d) {
  mju_zero(d->qfrc_passive, m->nv);
  for (int j = 0; j < m->njnt; j++) {
    mjtNum k = m->jnt_stiffness[j], dif[3];
    int pa = m->jnt_qposadr[j], da = m->jnt_dofadr[j];
    if (k == 0) continue;
    switch (m->jnt_type[j]) {
      case mjJNT_FREE:
        for (int i = 0; i < 3; i++)
          d->qfrc_passive[da + i] = -k * (d->qpos[pa + i] - m->qpos_spring[pa + i]);
        pa += 3; da += 3;
        /* fall through */
      case mjJNT_BALL:
        sub_quat(dif, d->qpos + pa, m->qpos_spring + pa);
        for (int i = 0; i < 3; i++) d->qfrc_passive[da + i] = -k * dif[i];
        break;
      default:
        d->qfrc_passive[da] = -k * (d->qpos[pa] - m->qpos_spring[pa]);
    }
  }
  for (int i = 0; i < m->nv; i++) d->qfrc_passive[i] -= m->dof_damping[i] * d->qvel[i];
}

static void reference_constraint(const mjModel* m, mjData* d) {
  for (int i = 0; i < d->nefc; i++) {
    const mjtNum* k = d->efc_KBIP + 4 * i;
    d->efc_vel[i] = dotn(d->efc_J + (size_t)i * m->nv, d->qvel, m->nv);
    d->efc_aref[i] = -k[1] * d->efc_vel[i] - k[0] * k[2] * (d->efc_pos[i] - d->efc_margin[i]);
  }
}

static void rne(const mjModel* m, mjData* d, mjtNum* result) {
  int nb = m->nbody;
  mjMARKSTACK
  mjtNum* cacc = mj_stackAlloc(d, 6 * nb);
  mjtNum* cfrc = mj_stackAlloc(d, 6 * nb);
  mjtNum tmp[6], tmp1[6];
  mju_zero(cacc, 6);
  cacc[3] = -m->opt.gravity[0];
  cacc[4] = -m->opt.gravity[1];
  cacc[5] = -m->opt.gravity[2];
  for (int i = 1; i < nb; i++) {
    int bda = m->body_dofadr[i];
    int p = m->body_parentid[i];
    if (m->body_dofnum[i])
      mul_dof_vec(tmp, d->cdof_dot + 6 * bda, d->qvel + bda, m->body_dofnum[i]);
    else
      mju_zero(tmp, 6);
    for (int k = 0; k < 6; k++) cacc[6 * i + k] = cacc[6 * p + k] + tmp[k];
    mul_inert_vec(cfrc + 6 * i, d->cinert + 10 * i, cacc + 6 * i);
    mul_inert_vec(tmp, d->cinert + 10 * i, d->cvel + 6 * i);
    cross_force(tmp1, d->cvel + 6 * i, tmp);
    for (int k = 0; k < 6; k++) cfrc[6 * i + k] += tmp1[k];
  }
  mju_zero(cfrc, 6);
  for (int i = nb - 1; i > 0; i--) {
    int p = m->body_parentid[i];
    if (p)
      for (int k = 0; k < 6; k++) cfrc[6 * p + k] += cfrc[6 * i + k];
  }
  for (int i = 0; i < m->nv; i++) result[i] = dotn(d->cdof + 6 * i, cfrc + 6 * m->dof_bodyid[i], 6);
  mjFREESTACK
}

static void fwd_velocity(const mjModel* m, mjData* d) {
  com_vel(m, d);
  passive(m, d);
  reference_constraint(m, d);
  rne(m, d, d->qfrc_bias);
}

/* ------------------------------------------------------------------------- */
/* acceleration stage                                                         */

static void fwd_actuation(const mjModel* m, mjData* d) {
  int nv = m->nv, nu = m->nu;
  for (int i = 0; i < nu; i++) {
    mjtNum c = d->ctrl[i], f;
    if (m->actuator_ctrllimited[i]) c = clip(c, m->actuator_ctrlrange[2 * i], m->actuator_ctrlrange[2 * i + 1]);
    f = m->actuator_gainprm[i] * c;
    if (m->actuator_forcelimited[i])
      f = clip(f, m->actuator_forcerange[2 * i], m->actuator_forcerange[2 * i + 1]);
    d->actuator_force[i] = f;
  }
  for (int j = 0; j < nv; j++) {
    mjtNum s = 0;
    for (int i = 0; i < nu; i++) s += d->actuator_moment[i * nv + j] * d->actuator_force[i];
    d->qfrc_actuator[j] = s;
  }
}

static void xfrc_accumulate(const mjModel* m, mjData* d, mjtNum* qfrc) {
  int nv = m->nv;
  mjMARKSTACK
  mjtNum* jp = mj_stackAlloc(d, 3 * nv);
  mjtNum* jr = mj_stackAlloc(d, 3 * nv);
  for (int b = 1; b < m->nbody; b++) {
    const mjtNum* f = d->xfrc_applied + 6 * b;
    if (f[0] == 0 && f[1] == 0 && f[2] == 0 && f[3] == 0 && f[4] == 0 && f[5] == 0) continue;
    jac_point(m, d, jp, d->xipos + 3 * b, b);
    jac_rot(m, d, jr, b);
    for (int j = 0; j < nv; j++) {
      mjtNum t1 = jp[j] * f[0] + jp[nv + j] * f[1] + jp[2 * nv + j] * f[2];
      mjtNum t2 = jr[j] * f[3] + jr[nv + j] * f[4] + jr[2 * nv + j] * f[5];
      qfrc[j] += t1 + t2;
    }
  }
  mjFREESTACK
}

static void fwd_acceleration(const mjModel* m, mjData* d) {
  int nv = m->nv;
  for (int i = 0; i < nv; i++) d->qfrc_smooth[i] = d->qfrc_passive[i] - d->qfrc_bias[i];
  for (int i = 0; i < nv; i++) d->qfrc_smooth[i] += d->qfrc_applied[i];
  for (int i = 0; i < nv; i++) d->qfrc_smooth[i] += d->qfrc_actuator[i];
  xfrc_accumulate(m, d, d->qfrc_smooth);
  mju_copy(d->qacc_smooth, d->qfrc_smooth, nv);
  solve_ld(m, d->qLD, d->qLDiagInv, d->qacc_smooth);
}

/* constraint cost of residuals jar; sets efc_force/efc_state and
   qfrc_constraint = J'*force */
static mjtNum constraint_update(const mjModel* m, mjData* d, const mjtNum* jar) {
  int nv = m->nv, ne = d->nefc;
  mjtNum cost = 0;
  for (int i = 0; i < ne; i++) {
    if (jar[i] < 0) {
      d->efc_force[i] = -d->efc_D[i] * jar[i];
      d->efc_state[i] = 1;
      cost += 0.5 * d->efc_D[i] * jar[i] * jar[i];
    } else {
      d->efc_force[i] = 0;
      d->efc_state[i] = 0;
    }
  }
  for (int j = 0; j < nv; j++) {
    mjtNum s = 0;
    for (int i = 0; i < ne; i++) s += d->efc_J[(size_t)i * nv + j] * d->efc_force[i];
    d->qfrc_constraint[j] = s;
  }
  return cost;
}
static mjtNum gauss_cost(int nv, const mjtNum* Ma, const mjtNum* qfrc_smooth, const mjtNum* qacc,
                         const mjtNum* qacc_smooth) {
  mjtNum s = 0;
  for (int j = 0; j < nv; j++) s += (Ma[j] - qfrc_smooth[j]) * (qacc[j] - qacc_smooth[j]);
  return 0.5 * s;
}
/* H = M + J' diag(D*active) J (lower), then dense Cholesky L L' in place */
static void hessian_factor(const mjModel* m, mjData* d, mjtNum* H) {
  int nv = m->nv, ne = d->nefc;
  for (int r = 0; r < nv; r++)
    for (int c = 0; c <= r; c++) {
      mjtNum h = 0;
      for (int i = 0; i < ne; i++)
        if (d->efc_state[i]) {
          const mjtNum* J = d->efc_J + (size_t)i * nv;
          h += J[r] * d->efc_D[i] * J[c];
        }
      H[r * nv + c] = d->qM[r * nv + c] + h;
    }
  for (int j = 0; j < nv; j++) {
    mjtNum t = H[j * nv + j];
    if (j) t -= dotn(H + j * nv, H + j * nv, j);
    if (t < mjMINVAL) t = mjMINVAL;
    H[j * nv + j] = sqrt(t);
    t = 1 / H[j * nv + j];
    for (int i = j + 1; i < nv; i++) H[i * nv + j] = (H[i * nv + j] - dotn(H + i * nv, H + j * nv, j)) * t;
  }
}
static void chol_solve(int nv, const mjtNum* L, const mjtNum* b, mjtNum* x) {
  mju_copy(x, b, nv);
  for (int i = 0; i < nv; i++) {
    if (i) x[i] -= dotn(L + i * nv, x, i);
    x[i] /= L[i * nv + i];
  }
  for (int i = nv - 1; i >= 0; i--) {
    for (int j = i + 1; j < nv; j++) x[i] -= L[j * nv + i] * x[j];
    x[i] /= L[i * nv + i];
  }
}

/* exact line search on the convex piecewise quadratic along `search` */
static mjtNum linesearch(const mjModel* m, mjData* d, const mjtNum* search, const mjtNum* Ma,
                         const mjtNum* jar, mjtNum* Mv, mjtNum* Jv) {
  int nv = m->nv, ne = d->nefc;
  mjtNum snorm = sqrt(dotn(search, search, nv)), g1 = 0, g2 = 0;
  mjtNum alpha = 0, d1, d2, lo = 0, hi = -1, gtol;
  if (snorm < mjMINVAL) return 0;
  mul_m(nv, d->qM, search, Mv);
  for (int i = 0; i < ne; i++) Jv[i] = dotn(d->efc_J + (size_t)i * nv, search, nv);
  for (int j = 0; j < nv; j++) g1 += search[j] * (Ma[j] - d->qfrc_smooth[j]);
  for (int j = 0; j < nv; j++) g2 += search[j] * Mv[j];
#define LS_EVAL(a)                                               \
  do {                                                           \
    d1 = g1 + g2 * (a);                                          \
    d2 = g2;                                                     \
    for (int i_ = 0; i_ < ne; i_++) {                            \
      mjtNum x_ = jar[i_] + (a) * Jv[i_];                        \
      if (x_ < 0) {                                              \
        d1 += d->efc_D[i_] * x_ * Jv[i_];                        \
        d2 += d->efc_D[i_] * Jv[i_] * Jv[i_];                    \
      }                                                          \
    }                                                            \
  } while (0)
  LS_EVAL(0.0);
  if (d1 >= 0) return 0;
  gtol = ORA_LS_TOL * fabs(d1);
#ifdef ORA_LS_STUDY /* tools/ls_study: the line search's iterations, observed (never in liboracle.so) */
  ora_ls_study_begin(ne, Jv, jar, d->efc_D, g1, g2, d1, d2, gtol);
#endif
  for (int it = 0; it < ORA_LS_ITER; it++) {
    mjtNum anew = alpha - d1 / d2;
    int bis = 0;
    if (hi >= 0 && !(anew > lo && anew < hi)) anew = 0.5 * (lo + hi), bis = 1;
    alpha = anew;
    LS_EVAL(alpha);
#ifdef ORA_LS_STUDY
    ora_ls_study_iter(it, bis, lo, hi, alpha, d1, d2);
#endif
    (void)bis;
    if (fabs(d1) < gtol) break;
    if (d1 < 0) lo = alpha; else hi = alpha;
  }
#ifdef ORA_LS_STUDY
  ora_ls_study_end();
#endif
#undef LS_EVAL
  return alpha;
}

static void solver_newton(const mjModel* m, mjData* d, int maxiter, mjtNum tol) {
  int nv = m->nv, ne = d->nefc, iter = 0;
  mjtNum scale = 1 / (m->stat.meaninertia * (nv > 1 ? nv : 1));
  mjtNum cost, oldcost, improvement, gradient;
  mjMARKSTACK
  mjtNum* Ma = mj_stackAlloc(d, nv);
  mjtNum* grad = mj_stackAlloc(d, nv);
  mjtNum* search = mj_stackAlloc(d, nv);
  mjtNum* Mv = mj_stackAlloc(d, nv);
  mjtNum* H = mj_stackAlloc(d, nv * nv);
  mjtNum* jar = mj_stackAlloc(d, ne);
  mjtNum* Jv = mj_stackAlloc(d, ne);

  mul_m(nv, d->qM, d->qacc, Ma);
  for (int i = 0; i < ne; i++) jar[i] = dotn(d->efc_J + (size_t)i * nv, d->qacc, nv) - d->efc_aref[i];
  cost = gauss_cost(nv, Ma, d->qfrc_smooth, d->qacc, d->qacc_smooth) + constraint_update(m, d, jar);
  for (int j = 0; j < nv; j++) grad[j] = (Ma[j] - d->qfrc_smooth[j]) - d->qfrc_constraint[j];
  hessian_factor(m, d, H);
  while (iter < maxiter) {
    mjtNum alpha;
    chol_solve(nv, H, grad, search);
    for (int j = 0; j < nv; j++) search[j] = -search[j];
    alpha = linesearch(m, d, search, Ma, jar, Mv, Jv);
#ifdef ORA_NT_STUDY /* tools/ls_study: would the active set at alpha = 1 predict the next factor's? */
    ora_nt_study_iter(ne, jar, Jv, alpha, d->efc_state);
#endif
    if (alpha == 0) break;
    for (int j = 0; j < nv; j++) d->qacc[j] += alpha * search[j];
    for (int j = 0; j < nv; j++) Ma[j] += alpha * Mv[j];
    for (int i = 0; i < ne; i++) jar[i] += alpha * Jv[i];
    iter++;
    oldcost = cost;
    cost = gauss_cost(nv, Ma, d->qfrc_smooth, d->qacc, d->qacc_smooth) + constraint_update(m, d, jar);
    for (int j = 0; j < nv; j++) grad[j] = (Ma[j] - d->qfrc_smooth[j]) - d->qfrc_constraint[j];
    improvement = scale * (oldcost - cost);
    gradient = scale * sqrt(dotn(grad, grad, nv));
    if (improvement < tol || gradient < tol) break;
    hessian_factor(m, d, H);
  }
  d->solver_iter = iter;
  mjFREESTACK
}

static void fwd_constraint(const mjModel* m, mjData* d) {
  int nv = m->nv, ne = d->nefc;
  if (!ne) {
    mju_copy(d->qacc, d->qacc_smooth, nv);
    mju_copy(d->qacc_warmstart, d->qacc_smooth, nv);
    mju_zero(d->qfrc_constraint, nv);
    d->solver_iter = 0;
    return;
  }
  {
    mjMARKSTACK
    mjtNum* Ma = mj_stackAlloc(d, nv);
    mjtNum* jar = mj_stackAlloc(d, ne);
    mjtNum cost_warm, cost_smooth;
    for (int i = 0; i < ne; i++)
      d->efc_b[i] = dotn(d->efc_J + (size_t)i * nv, d->qacc_smooth, nv) - d->efc_aref[i];
    cost_smooth = constraint_update(m, d, d->efc_b);
    mul_m(nv, d->qM, d->qacc_warmstart, Ma);
    for (int i = 0; i < ne; i++)
      jar[i] = dotn(d->efc_J + (size_t)i * nv, d->qacc_warmstart, nv) - d->efc_aref[i];
    cost_warm = gauss_cost(nv, Ma, d->qfrc_smooth, d->qacc_warmstart, d->qacc_smooth) +
                constraint_update(m, d, jar);
    if (cost_warm > cost_smooth)
      mju_copy(d->qacc, d->qacc_smooth, nv);
    else
      mju_copy(d->qacc, d->qacc_warmstart, nv);
    mjFREESTACK
  }
  solver_newton(m, d, m->opt.iterations, m->opt.tolerance);
  mju_copy(d->qacc_warmstart, d->qacc, nv);
}

/* ------------------------------------------------------------------------- */
/* top level                                                                  */

void mj_forwardSkip(const mjModel* m, mjData* d, int skipstage, int skipsensor) {
  (void)skipsensor; /* no sensors in the supported models */
  if (skipstage < mjSTAGE_POS) fwd_position(m, d);
  if (skipstage < mjSTAGE_VEL) fwd_velocity(m, d);
  fwd_actuation(m, d);
  fwd_acceleration(m, d);
  fwd_constraint(m, d);
}

void mj_forward(const mjModel* m, mjData* d) { mj_forwardSkip(m, d, mjSTAGE_NONE, 0); }

static int is_bad(mjtNum x) { return x != x || x > mjMAXVAL || x < -mjMAXVAL; }

static void integrate_pos(const mjModel* m, mjtNum* qpos, const mjtNum* qvel, mjtNum dt) {
  for (int j = 0; j < m->njnt; j++) {
    int pa = m->jnt_qposadr[j], va = m->jnt_dofadr[j];
    switch (m->jnt_type[j]) {
      case mjJNT_FREE:
        for (int i = 0; i < 3; i++) qpos[pa + i] += dt * qvel[va + i];
        mju_quatIntegrate(qpos + pa + 3, qvel + va + 3, dt);
        break;
      case mjJNT_BALL:
        mju_quatIntegrate(qpos + pa, qvel + va, dt);
        break;
      default:
        qpos[pa] += dt * qvel[va];
    }
  }
}

static void advance(const mjModel* m, mjData* d, const mjtNum* qacc, const mjtNum* qvel) {
  mjtNum h = m->opt.timestep;
  for (int i = 0; i < m->nv; i++) d->qvel[i] += qacc[i] * h;
  integrate_pos(m, d->qpos, qvel ? qvel : d->qvel, h);
  d->time += h;
}

void mj_Euler(const mjModel* m, mjData* d) {
  int nv = m->nv, dmp = 0;
  mjMARKSTACK
  mjtNum* qacc = mj_stackAlloc(d, nv);
  for (int i = 0; i < nv; i++)
    if (m->dof_damping[i] > 0) { dmp = 1; break; }
  if (!dmp) {
    mju_copy(qacc, d->qacc, nv);
  } else {
    mjtNum* qH = mj_stackAlloc(d, nv * nv);
    mjtNum* qHLD = mj_stackAlloc(d, nv * nv);
    mjtNum* qHinv = mj_stackAlloc(d, nv);
    mul_m(nv, d->qM, d->qacc, qacc);
    mju_copy(qH, d->qM, nv * nv);
    for (int i = 0; i < nv; i++) qH[i * nv + i] += m->opt.timestep * m->dof_damping[i];
    factor_ld(m, qH, qHLD, qHinv);
    solve_ld(m, qHLD, qHinv, qacc);
  }
  advance(m, d, qacc, NULL);
  mjFREESTACK
}

void mj_RungeKutta(const mjModel* m, mjData* d, int N) {
  static const mjtNum RK4_A[9] = {0.5, 0, 0, 0, 0.5, 0, 0, 0, 1};
  static const mjtNum RK4_B[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6};
  int nv = m->nv, nq = m->nq;
  mjtNum h = m->opt.timestep, time = d->time, C[3], T[3];
  mjtNum *X[4], *F[4], *dX;
  mjMARKSTACK
  if (N != 4) mju_error("only RK4 is supported");
  dX = mj_stackAlloc(d, 2 * nv);
  for (int i = 0; i < N; i++) {
    X[i] = mj_stackAlloc(d, nq + nv);
    F[i] = mj_stackAlloc(d, nv);
  }
  for (int i = 1; i < N; i++) {
    C[i - 1] = 0;
    for (int j = 0; j < i; j++) C[i - 1] += RK4_A[(i - 1) * (N - 1) + j];
    T[i - 1] = d->time + C[i - 1] * h;
  }
  mju_copy(X[0], d->qpos, nq);
  mju_copy(X[0] + nq, d->qvel, nv);
  mju_copy(F[0], d->qacc, nv);
  for (int i = 1; i < N; i++) {
    mju_zero(dX, 2 * nv);
    for (int j = 0; j < i; j++) {
      mjtNum a = RK4_A[(i - 1) * (N - 1) + j];
      for (int k = 0; k < nv; k++) dX[k] += X[j][nq + k] * a;
      for (int k = 0; k < nv; k++) dX[nv + k] += F[j][k] * a;
    }
    mju_copy(X[i], X[0], nq + nv);
    integrate_pos(m, X[i], dX, h);
    for (int k = 0; k < nv; k++) X[i][nq + k] += dX[nv + k] * h;
    mju_copy(d->qpos, X[i], nq + nv); /* qpos, qvel contiguous */
    d->time = T[i - 1];
    mj_forwardSkip(m, d, mjSTAGE_NONE, 1);
    mju_copy(F[i], d->qacc, nv);
  }
  mju_zero(dX, 2 * nv);
  for (int j = 0; j < N; j++) {
    for (int k = 0; k < nv; k++) dX[k] += X[j][nq + k] * RK4_B[j];
    for (int k = 0; k < nv; k++) dX[nv + k] += F[j][k] * RK4_B[j];
  }
  d->time = time;
  mju_copy(d->qpos, X[0], nq + nv);
  advance(m, d, dX + nv, dX);
  mjFREESTACK
}

void mj_step(const mjModel* m, mjData* d) {
  for (int i = 0; i < m->nq; i++)
    if (is_bad(d->qpos[i])) { mj_resetData(m, d); break; }
  for (int i = 0; i < m->nv; i++)
    if (is_bad(d->qvel[i])) { mj_resetData(m, d); break; }
  mj_forward(m, d);
  for (int i = 0; i < m->nv; i++)
    if (is_bad(d->qacc[i])) { mj_resetData(m, d); mj_forward(m, d); break; }
  if (m->opt.integrator == mjINT_RK4)
    mj_RungeKutta(m, d, 4);
  else
    mj_Euler(m, d);
}
