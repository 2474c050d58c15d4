// Scalar building blocks of the device physics (gfx950, fp64): constants,
// fdlibm sin/cos, quaternion/rotation/spatial-algebra helpers, the narrow
// phase and the constraint impedance.  The cooperative pipeline (dcoop.h) --
// the MuJoCo-2.0 mj_forward / mj_forwardSkip / mj_step that the reference
// reaches through libmujoco200 (src/mjderivative.cpp:64,68,92,103,124,134,178,198,
// inc/ilqr.h:86,128) -- is written on top of these.
// Arithmetic contract: identical operation order to the CPU oracle
// (oracle/mjsub.c) with FMA contraction disabled (-ffp-contract=off),
// sums in ascending index order, fdlibm sin/cos, correctly rounded sqrt and
// division -- so every result is bit-identical to the oracle's.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

#include "dmodel.h"

namespace ilqg {
namespace dev {

constexpr double MINVAL = 1e-15;
constexpr double MAXVAL = 1e10;
constexpr double MINIMP = 0.0001;
constexpr double MAXIMP = 0.9999;
constexpr int LS_ITER = 50;
constexpr double LS_TOL = 0.01;
enum { JNT_FREE = 0, JNT_BALL, JNT_SLIDE, JNT_HINGE };
enum { GEOM_PLANE = 0, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE };
enum { STAGE_NONE = 0, STAGE_POS, STAGE_VEL };
enum { C_LIMIT = 3, C_FRICTIONLESS = 5, C_PYRAMIDAL = 6 };

// ------------------------------------------------------------ math -------
__device__ __forceinline__ double clipd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }
__device__ __forceinline__ double maxd(double a, double b) { return a > b ? a : b; }

// fdlibm/musl kernels, same constants and order as oracle/mjsub.c ora_sin/ora_cos
__device__ inline double k_sin(double x, double y, int iy) {
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  double z = x * x, w = z * z;
  double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
  double v = z * x;
  if (iy == 0) return x + v * (S1 + z * r);
  return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
__device__ inline double k_cos(double x, double y) {
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double z = x * x, w = z * z;
  double r = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
  double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}
__device__ inline int rem_pio2(double x, double* y0, double* y1) {
  const double INVPIO2 = 6.36619772367581382433e-01, PIO2_1 = 1.57079632673412561417e+00,
               PIO2_1T = 6.07710050650619224932e-11;
  double fn = floor(x * INVPIO2 + 0.5);
  double r = x - fn * PIO2_1;
  double w = fn * PIO2_1T;
  *y0 = r - w;
  *y1 = (r - *y0) - w;
  return (int)fn;
}
__device__ inline double det_sin(double x) {
  const double PIO4 = 7.85398163397448278999e-01;
  double y0, y1;
  if (fabs(x) < PIO4) return x == 0 ? x : k_sin(x, 0.0, 0);
  int n = rem_pio2(x, &y0, &y1);
  switch (n & 3) {
    case 0: return k_sin(y0, y1, 1);
    case 1: return k_cos(y0, y1);
    case 2: return -k_sin(y0, y1, 1);
    default: return -k_cos(y0, y1);
  }
}
__device__ inline double det_cos(double x) {
  const double PIO4 = 7.85398163397448278999e-01;
  double y0, y1;
  if (fabs(x) < PIO4) return k_cos(x, 0.0);
  int n = rem_pio2(x, &y0, &y1);
  switch (n & 3) {
    case 0: return k_cos(y0, y1);
    case 1: return -k_sin(y0, y1, 1);
    case 2: return -k_cos(y0, y1);
    default: return k_sin(y0, y1, 1);
  }
}

// det_sin(x) and det_cos(x) at once, without branches: the four kernel
// evaluations either function may return (small-angle k_sin / k_cos of x, and
// k_sin / k_cos of the reduced argument) are all formed -- independent chains,
// so they overlap -- and each result selects the one its branch would take,
// with its sign.  Every returned double is the expression det_sin / det_cos
// evaluate, so the values are identical; what goes is the divergent control
// flow (two tests and a four-way switch per function, in series).
__device__ inline void det_sincos(double x, double* s, double* c) {
  const double PIO4 = 7.85398163397448278999e-01;
  // every active lane within pi/4 (the common case for joint half-angles): the
  // small-angle kernels are all either function evaluates
  if (__ballot(!(fabs(x) < PIO4)) == 0ull) {
    *s = x == 0 ? x : k_sin(x, 0.0, 0);
    *c = k_cos(x, 0.0);
    return;
  }
  double y0, y1;
  const int n = rem_pio2(x, &y0, &y1);
  const double s0 = k_sin(x, 0.0, 0), c0 = k_cos(x, 0.0);
  const double sr = k_sin(y0, y1, 1), cr = k_cos(y0, y1);
  const bool small = fabs(x) < PIO4;
  const int q = n & 3;
  const double sl = (q & 1) ? cr : sr;  // sin: q 0 sr, 1 cr, 2 -sr, 3 -cr
  const double cl = (q & 1) ? sr : cr;  // cos: q 0 cr, 1 -sr, 2 -cr, 3 sr
  const double sv = (q & 2) ? -sl : sl;
  const double cv = (q == 1 || q == 2) ? -cl : cl;
  *s = small ? (x == 0 ? x : s0) : sv;
  *c = small ? c0 : cv;
}

template <class A, class B>
__device__ __forceinline__ auto dot3(const A* a, const B* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <class R, class A, class B>
__device__ __forceinline__ void cross3(R* r, const A* a, const B* b) {
  R t0 = a[1] * b[2] - a[2] * b[1];
  R t1 = a[2] * b[0] - a[0] * b[2];
  R t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
template <class R>
__device__ inline R normalize3(R* v) {
  R norm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (norm < MINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0;
  } else {
    R inv = 1 / norm;
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
  }
  return norm;
}
template <class R>
__device__ inline void normalize4(R* q) {
  R norm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (norm < MINVAL) {
    q[0] = 1; q[1] = 0; q[2] = 0; q[3] = 0;
  } else if (fabs(norm - 1) > MINVAL) {
    R inv = 1 / norm;
    q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
  }
}
template <class R, class A, class B>
__device__ __forceinline__ void quat_mul(R* r, const A* a, const B* b) {
  R t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  R t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  R t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  R t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
// dof j of x_a (-) x_b (oracle ora_state_diff): plain difference for
// slide/hinge dofs and free-joint translations; quaternion dofs use the
// first-order log map 2 sign(w) v of conj(q_b) q_a.  For models without
// ball/free joints this is exactly qpos_a[j] - qpos_b[j].
template <class M, class PA, class PB>
__device__ inline auto state_diff_dof(const M& m, int j, const PA& qa, const PB& qb) {
  using R = std::remove_cvref_t<decltype(qa[0])>;
  const int jid = m.dof_jntid[j], t = m.jnt_type[jid], qadr = m.jnt_qposadr[jid], dadr = m.jnt_dofadr[jid];
  if ((t == JNT_FREE && j >= dadr + 3) || t == JNT_BALL) {
    const int qo = qadr + (t == JNT_FREE ? 3 : 0), k = j - dadr - (t == JNT_FREE ? 3 : 0);
    const R c[4] = {qb[qo], -qb[qo + 1], -qb[qo + 2], -qb[qo + 3]};
    const R a[4] = {qa[qo], qa[qo + 1], qa[qo + 2], qa[qo + 3]};
    R q[4];
    quat_mul(q, c, a);
    const R sg = q[0] < 0 ? -2.0 : 2.0;
    return (R)(sg * q[1 + k]);
  }
  return (R)(qa[qadr + j - dadr] - qb[qadr + j - dadr]);
}
template <class R, class V, class Q>
__device__ inline void rot_vec_quat(R* r, const V* v, const Q* q) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) {
    r[0] = r[1] = r[2] = 0;
  } else if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2];
  } else {
    R t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
    R t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
    R t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
    R r0 = v[0] + 2 * (q[2] * t2 - q[3] * t1);
    R r1 = v[1] + 2 * (q[3] * t0 - q[1] * t2);
    R r2 = v[2] + 2 * (q[1] * t1 - q[2] * t0);
    r[0] = r0; r[1] = r1; r[2] = r2;
  }
}
template <class R, class Q>
__device__ inline void quat2mat(R* r, const Q* q) {
  // MuJoCo's identity shortcut is omitted: for q == (1,0,0,0) the general
  // formula yields exactly the same doubles, and the branch forced r to scratch.
  R q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  R q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  R q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
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
template <class R, class A, class G>
__device__ inline void axis_angle2quat(R* r, const A* axis, G angle) {
  if (angle == 0) {
    r[0] = 1; r[1] = 0; r[2] = 0; r[3] = 0;
  } else {
    double sd, cd;
    det_sincos(angle * 0.5, &sd, &cd);
    R s = sd;
    r[0] = cd;
    r[1] = axis[0] * s; r[2] = axis[1] * s; r[3] = axis[2] * s;
  }
}
template <class R, class V, class X>
__device__ __forceinline__ void rot_vec_mat(R* r, const V* v, const X* m) {
  R r0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  R r1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  R r2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
template <class R, class V, class G>
__device__ inline void quat_integrate(R* quat, const V* vel, G scale) {
  R tmp[3] = {vel[0], vel[1], vel[2]}, qrot[4];
  R angle = scale * normalize3(tmp);
  axis_angle2quat(qrot, tmp, angle);
  normalize4(quat);
  quat_mul(quat, quat, qrot);
}
template <class R>
__device__ inline void make_frame(R* f) {
  R tmp[3], d;
  normalize3(f);
  f[3] = f[4] = f[5] = 0;
  if (fabs(f[1]) < 0.5) f[4] = 1; else f[5] = 1;
  d = dot3(f, f + 3);
  tmp[0] = f[0] * d; tmp[1] = f[1] * d; tmp[2] = f[2] * d;
  f[3] -= tmp[0]; f[4] -= tmp[1]; f[5] -= tmp[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}
template <class R, class I, class X, class D, class G>
__device__ inline void inert_com(R* res, const I* in, const X* mat, const D* dif, G mass) {
  R tmp[9] = {mat[0] * in[0], mat[3] * in[0], mat[6] * in[0],
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
template <class R, class I, class V>
__device__ inline void mul_inert_vec(R* r, const I* i, const V* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
template <class R, class A, class V>
__device__ inline void cross_motion(R* r, const A* vel, const V* v) {
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
template <class R, class A, class V>
__device__ inline void cross_force(R* r, const A* vel, const V* f) {
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

// load a small vector into registers
template <int N, class R, class A>
__device__ __forceinline__ void ldm(R* r, const A* a) {
#pragma unroll
  for (int k = 0; k < N; k++) r[k] = a[k];
}

template <class R>
struct LdsConSinkT {
  R* rec;  // contact k at rec + 7k: dist, pos[3], n[3]
  template <class P, class N>
  __device__ __forceinline__ void put(int k, R d, const P* p, const N* n) const {
    R* r = rec + 7 * k;
    r[0] = d;
    r[1] = p[0]; r[2] = p[1]; r[3] = p[2];
    r[4] = n[0]; r[5] = n[1]; r[6] = n[2];
  }
};
using LdsConSink = LdsConSinkT<double>;
template <class S>
__device__ __forceinline__ int sphere_sphere(const S& out, int k, double margin, const auto* p1, double r1,
                                             const auto* p2, double r2) {
  using R = std::remove_cvref_t<decltype(*out.rec)>;
  R axis[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  R dist = normalize3(axis) - r1 - r2;
  if (dist > margin) return 0;
  const R s = r1 + dist / 2;
  const R pos[3] = {p1[0] + axis[0] * s, p1[1] + axis[1] * s, p1[2] + axis[2] * s};
  out.put(k, dist, pos, axis);
  return 1;
}
template <class S>
__device__ __forceinline__ int plane_sphere(const S& out, int k, double margin, const auto* pos1,
                                            const auto* mat1, const auto* p2, double r2) {
  using R = std::remove_cvref_t<decltype(*out.rec)>;
  R n[3] = {mat1[2], mat1[5], mat1[8]};
  R tmp[3] = {p2[0] - pos1[0], p2[1] - pos1[1], p2[2] - pos1[2]};
  R cdist = dot3(tmp, n);
  if (cdist > margin + r2) return 0;
  const R dist = cdist - r2;
  const R s = -dist / 2 - r2;
  const R pos[3] = {p2[0] + n[0] * s, p2[1] + n[1] * s, p2[2] + n[2] * s};
  out.put(k, dist, pos, n);
  return 1;
}
template <class M, class S>
__device__ __forceinline__ int narrow(const M& m, int t1, int t2, const auto* pos1, const auto* mat1,
                                      const auto* sz1, const auto* pos2, const auto* mat2, const auto* sz2,
                                      double margin, const S& out) {
  using R = std::remove_cvref_t<decltype(*out.rec)>;
  if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) return plane_sphere(out, 0, margin, pos1, mat1, pos2, sz2[0]);
  if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
    R seg[3] = {mat2[2] * sz2[1], mat2[5] * sz2[1], mat2[8] * sz2[1]}, p[3];
    int n1, n2;
    p[0] = pos2[0] + seg[0]; p[1] = pos2[1] + seg[1]; p[2] = pos2[2] + seg[2];
    n1 = plane_sphere(out, 0, margin, pos1, mat1, p, sz2[0]);
    p[0] = pos2[0] - seg[0]; p[1] = pos2[1] - seg[1]; p[2] = pos2[2] - seg[2];
    n2 = plane_sphere(out, n1, margin, pos1, mat1, p, sz2[0]);
    return n1 + n2;
  }
  if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) return sphere_sphere(out, 0, margin, pos1, sz1[0], pos2, sz2[0]);
  if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
    R ax[3] = {mat2[2], mat2[5], mat2[8]}, dif[3], p[3], x;
    dif[0] = pos1[0] - pos2[0]; dif[1] = pos1[1] - pos2[1]; dif[2] = pos1[2] - pos2[2];
    x = clipd(dot3(ax, dif), -sz2[1], sz2[1]);
    p[0] = pos2[0] + ax[0] * x; p[1] = pos2[1] + ax[1] * x; p[2] = pos2[2] + ax[2] * x;
    return sphere_sphere(out, 0, margin, pos1, sz1[0], p, sz2[0]);
  }
  if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
    R a1[3] = {mat1[2] * sz1[1], mat1[5] * sz1[1], mat1[8] * sz1[1]};
    R a2[3] = {mat2[2] * sz2[1], mat2[5] * sz2[1], mat2[8] * sz2[1]};
    R dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
    R ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    R u = -dot3(a1, dif), v = dot3(a2, dif);
    R det = ma * mc - mb * mb;
    R v1[3], v2[3], x1, x2;
    if (fabs(det) >= MINVAL) {
      x1 = (mc * u - mb * v) / det;
      x2 = (ma * v - mb * u) / det;
      if (x1 > 1) { x1 = 1; x2 = (v - mb) / mc; }
      else if (x1 < -1) { x1 = -1; x2 = (v + mb) / mc; }
      if (x2 > 1) { x2 = 1; x1 = clipd((u - mb) / ma, -1, 1); }
      else if (x2 < -1) { x2 = -1; x1 = clipd((u + mb) / ma, -1, 1); }
      v1[0] = pos1[0] + a1[0] * x1; v1[1] = pos1[1] + a1[1] * x1; v1[2] = pos1[2] + a1[2] * x1;
      v2[0] = pos2[0] + a2[0] * x2; v2[1] = pos2[1] + a2[1] * x2; v2[2] = pos2[2] + a2[2] * x2;
      return sphere_sphere(out, 0, margin, v1, sz1[0], v2, sz2[0]);
    } else {
      int n1, n2;
      v1[0] = pos1[0] + a1[0]; v1[1] = pos1[1] + a1[1]; v1[2] = pos1[2] + a1[2];
      x2 = clipd((v - mb) / mc, -1, 1);
      v2[0] = pos2[0] + a2[0] * x2; v2[1] = pos2[1] + a2[1] * x2; v2[2] = pos2[2] + a2[2] * x2;
      n1 = sphere_sphere(out, 0, margin, v1, sz1[0], v2, sz2[0]);
      v1[0] = pos1[0] - a1[0]; v1[1] = pos1[1] - a1[1]; v1[2] = pos1[2] - a1[2];
      x2 = clipd((v + mb) / mc, -1, 1);
      v2[0] = pos2[0] + a2[0] * x2; v2[1] = pos2[1] + a2[1] * x2; v2[2] = pos2[2] + a2[2] * x2;
      n2 = sphere_sphere(out, n1, margin, v1, sz1[0], v2, sz2[0]);
      return n1 + n2;
    }
  }
  return 0;
}

template <class S>
__device__ inline double get_impedance(const S* solimp, double pos, double margin) {
  double dmin = clipd(solimp[0], MINIMP, MAXIMP), dmax = clipd(solimp[1], MINIMP, MAXIMP);
  double width = solimp[2], mid = solimp[3], power = solimp[4], x, y, imp;
  if (dmin == dmax || width <= MINVAL) return 0.5 * (dmin + dmax);
  x = (pos - margin) / width;
  if (x < 0) x = -x;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  int p = (int)power;
  double xp = 1, mp = 1;
  if (x <= mid) {
    for (int k = 0; k < p; k++) xp *= x;
    for (int k = 0; k < p - 1; k++) mp *= mid;
    y = xp / mp;
  } else {
    double xm = 1 - x, mm = 1 - mid;
    for (int k = 0; k < p; k++) xp *= xm;
    for (int k = 0; k < p - 1; k++) mp *= mm;
    y = 1 - xp / mp;
  }
  imp = dmin + y * (dmax - dmin);
  return clipd(imp, MINIMP, MAXIMP);
}

__device__ inline bool is_bad(double x) { return x != x || x > MAXVAL || x < -MAXVAL; }

}  // namespace dev
}  // namespace ilqg
