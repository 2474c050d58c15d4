// Device forward dynamics for one evaluation per lane (gfx950, fp64).
//
// This is the MuJoCo-2.0 pipeline that the reference reaches through
// libmujoco200 on every mj_forward / mj_forwardSkip / mj_step call
// (src/mjderivative.cpp:64,68,92,103,124,134,178,198, inc/ilqr.h:86,128).
// Arithmetic contract: identical operation order to the CPU oracle
// (oracle/mjsub.c) with FMA contraction disabled (-ffp-contract=off),
// sums in ascending index order, fdlibm sin/cos, correctly rounded sqrt and
// division -- so every result is bit-identical to the oracle's.
#pragma once

#include <hip/hip_runtime.h>

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

// strided views into the lane workspace
struct SPd {
  double* p;
  size_t s;
  __device__ __forceinline__ double& operator[](int i) const { return p[(size_t)i * s]; }
  __device__ __forceinline__ SPd operator+(int k) const { return SPd{p + (size_t)k * s, s}; }
};
struct SPi {
  int* p;
  size_t s;
  __device__ __forceinline__ int& operator[](int i) const { return p[(size_t)i * s]; }
};
struct Lane {
  double* d;
  int* i;
  size_t s;
  __device__ __forceinline__ SPd D(int off) const { return SPd{d + (size_t)off * s, s}; }
  __device__ __forceinline__ SPi I(int off) const { return SPi{i + (size_t)off * s, s}; }
};

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

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ void cross3(double* r, const double* a, const double* b) {
  double t0 = a[1] * b[2] - a[2] * b[1];
  double t1 = a[2] * b[0] - a[0] * b[2];
  double t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
__device__ inline double normalize3(double* v) {
  double norm = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (norm < MINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0;
  } else {
    double inv = 1 / norm;
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
  }
  return norm;
}
__device__ inline void normalize4(double* q) {
  double norm = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (norm < MINVAL) {
    q[0] = 1; q[1] = 0; q[2] = 0; q[3] = 0;
  } else if (fabs(norm - 1) > MINVAL) {
    double inv = 1 / norm;
    q[0] *= inv; q[1] *= inv; q[2] *= inv; q[3] *= inv;
  }
}
__device__ __forceinline__ void quat_mul(double* r, const double* a, const double* b) {
  double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}
// dof j of x_a (-) x_b (oracle ora_state_diff): plain difference for
// slide/hinge dofs and free-joint translations; quaternion dofs use the
// first-order log map 2 sign(w) v of conj(q_b) q_a.  For models without
// ball/free joints this is exactly qpos_a[j] - qpos_b[j].
template <class M, class PA, class PB>
__device__ inline double state_diff_dof(const M& m, int j, const PA& qa, const PB& qb) {
  const int jid = m.dof_jntid[j], t = m.jnt_type[jid], qadr = m.jnt_qposadr[jid], dadr = m.jnt_dofadr[jid];
  if ((t == JNT_FREE && j >= dadr + 3) || t == JNT_BALL) {
    const int qo = qadr + (t == JNT_FREE ? 3 : 0), k = j - dadr - (t == JNT_FREE ? 3 : 0);
    const double c[4] = {qb[qo], -qb[qo + 1], -qb[qo + 2], -qb[qo + 3]};
    const double a[4] = {qa[qo], qa[qo + 1], qa[qo + 2], qa[qo + 3]};
    double q[4];
    quat_mul(q, c, a);
    const double sg = q[0] < 0 ? -2.0 : 2.0;
    return sg * q[1 + k];
  }
  return qa[qadr + j - dadr] - qb[qadr + j - dadr];
}
__device__ inline void rot_vec_quat(double* r, const double* v, const double* q) {
  if (v[0] == 0 && v[1] == 0 && v[2] == 0) {
    r[0] = r[1] = r[2] = 0;
  } else if (q[0] == 1 && q[1] == 0 && q[2] == 0 && q[3] == 0) {
    r[0] = v[0]; r[1] = v[1]; r[2] = v[2];
  } else {
    double t0 = q[0] * v[0] + q[2] * v[2] - q[3] * v[1];
    double t1 = q[0] * v[1] + q[3] * v[0] - q[1] * v[2];
    double t2 = q[0] * v[2] + q[1] * v[1] - q[2] * v[0];
    double r0 = v[0] + 2 * (q[2] * t2 - q[3] * t1);
    double r1 = v[1] + 2 * (q[3] * t0 - q[1] * t2);
    double r2 = v[2] + 2 * (q[1] * t1 - q[2] * t0);
    r[0] = r0; r[1] = r1; r[2] = r2;
  }
}
__device__ inline void quat2mat(double* r, const double* q) {
  // MuJoCo's identity shortcut is omitted: for q == (1,0,0,0) the general
  // formula yields exactly the same doubles, and the branch forced r to scratch.
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
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
__device__ inline void axis_angle2quat(double* r, const double* axis, double angle) {
  if (angle == 0) {
    r[0] = 1; r[1] = 0; r[2] = 0; r[3] = 0;
  } else {
    double s = det_sin(angle * 0.5);
    r[0] = det_cos(angle * 0.5);
    r[1] = axis[0] * s; r[2] = axis[1] * s; r[3] = axis[2] * s;
  }
}
__device__ __forceinline__ void rot_vec_mat(double* r, const double* v, const double* m) {
  double r0 = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
  double r1 = m[3] * v[0] + m[4] * v[1] + m[5] * v[2];
  double r2 = m[6] * v[0] + m[7] * v[1] + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
__device__ inline void quat_integrate(double* quat, const double* vel, double scale) {
  double tmp[3] = {vel[0], vel[1], vel[2]}, qrot[4];
  double angle = scale * normalize3(tmp);
  axis_angle2quat(qrot, tmp, angle);
  normalize4(quat);
  quat_mul(quat, quat, qrot);
}
__device__ inline void make_frame(double* f) {
  double tmp[3], d;
  normalize3(f);
  f[3] = f[4] = f[5] = 0;
  if (fabs(f[1]) < 0.5) f[4] = 1; else f[5] = 1;
  d = dot3(f, f + 3);
  tmp[0] = f[0] * d; tmp[1] = f[1] * d; tmp[2] = f[2] * d;
  f[3] -= tmp[0]; f[4] -= tmp[1]; f[5] -= tmp[2];
  normalize3(f + 3);
  cross3(f + 6, f, f + 3);
}
__device__ inline void inert_com(double* res, const double* in, const double* mat, const double* dif, double mass) {
  double tmp[9] = {mat[0] * in[0], mat[3] * in[0], mat[6] * in[0],
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
__device__ inline void mul_inert_vec(double* r, const double* i, const double* v) {
  r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
}
__device__ inline void cross_motion(double* r, const double* vel, const double* v) {
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
__device__ inline void cross_force(double* r, const double* vel, const double* f) {
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

// load/store small vectors between registers and the strided workspace
template <int N>
__device__ __forceinline__ void ld(double* r, SPd a) {
#pragma unroll
  for (int k = 0; k < N; k++) r[k] = a[k];
}
template <int N>
__device__ __forceinline__ void st(SPd a, const double* r) {
#pragma unroll
  for (int k = 0; k < N; k++) a[k] = r[k];
}
template <int N>
__device__ __forceinline__ void ldm(double* r, const double* a) {
#pragma unroll
  for (int k = 0; k < N; k++) r[k] = a[k];
}
__device__ __forceinline__ double dotn(SPd a, SPd b, int n) {
  double r = 0;
  for (int i = 0; i < n; i++) r += a[i] * b[i];
  return r;
}

// ------------------------------------------------------ position stage ---
__device__ inline void kinematics(const DevModel& m, const WsLayout& L, const Lane& ln) {
  SPd qpos = ln.D(L.qpos), xpos = ln.D(L.xpos), xquat = ln.D(L.xquat), xmat = ln.D(L.xmat);
  SPd xipos = ln.D(L.xipos), ximat = ln.D(L.ximat), xanchor = ln.D(L.xanchor), xaxis = ln.D(L.xaxis);
  {
    double q0[4] = {1, 0, 0, 0}, m0[9];
    xpos[0] = xpos[1] = xpos[2] = 0;
    st<4>(xquat, q0);
    quat2mat(m0, q0);
    st<9>(xmat, m0);
    xipos[0] = xipos[1] = xipos[2] = 0;
    st<9>(ximat, m0);
  }
  for (int i = 1; i < m.nbody; i++) {
    int pid = m.body_parentid[i];
    double xp[3], xq[4], tmp[3], qloc[4], pq[4], pp[3], bp[3], bq[4];
    ld<4>(pq, xquat + 4 * pid);
    ld<3>(pp, xpos + 3 * pid);
    ldm<3>(bp, m.body_pos + 3 * i);
    ldm<4>(bq, m.body_quat + 4 * i);
    rot_vec_quat(tmp, bp, pq);
    xp[0] = pp[0] + tmp[0];
    xp[1] = pp[1] + tmp[1];
    xp[2] = pp[2] + tmp[2];
    quat_mul(xq, pq, bq);
    for (int j = 0; j < m.body_jntnum[i]; j++) {
      int jid = m.body_jntadr[i] + j;
      int qadr = m.jnt_qposadr[jid];
      int type = m.jnt_type[jid];
      double anc[3], ax[3], jp[3], ja[3];
      ldm<3>(jp, m.jnt_pos + 3 * jid);
      ldm<3>(ja, m.jnt_axis + 3 * jid);
      if (type == JNT_FREE) {
        xp[0] = qpos[qadr]; xp[1] = qpos[qadr + 1]; xp[2] = qpos[qadr + 2];
        xq[0] = qpos[qadr + 3]; xq[1] = qpos[qadr + 4]; xq[2] = qpos[qadr + 5]; xq[3] = qpos[qadr + 6];
        normalize4(xq);
        st<3>(xanchor + 3 * jid, xp);
        st<3>(xaxis + 3 * jid, ja);
        continue;
      }
      rot_vec_quat(anc, jp, xq);
      anc[0] += xp[0]; anc[1] += xp[1]; anc[2] += xp[2];
      rot_vec_quat(ax, ja, xq);
      if (type == JNT_SLIDE) {
        double dq = qpos[qadr] - m.qpos0[qadr];
        xp[0] += ax[0] * dq; xp[1] += ax[1] * dq; xp[2] += ax[2] * dq;
      } else {
        if (type == JNT_BALL) {
          qloc[0] = qpos[qadr]; qloc[1] = qpos[qadr + 1]; qloc[2] = qpos[qadr + 2]; qloc[3] = qpos[qadr + 3];
          normalize4(qloc);
        } else {
          axis_angle2quat(qloc, ja, qpos[qadr] - m.qpos0[qadr]);
        }
        quat_mul(xq, xq, qloc);
        rot_vec_quat(tmp, jp, xq);
        xp[0] = anc[0] - tmp[0];
        xp[1] = anc[1] - tmp[1];
        xp[2] = anc[2] - tmp[2];
      }
      st<3>(xanchor + 3 * jid, anc);
      st<3>(xaxis + 3 * jid, ax);
    }
    normalize4(xq);
    st<3>(xpos + 3 * i, xp);
    st<4>(xquat + 4 * i, xq);
    double mat[9], ip[3], iq[4];
    quat2mat(mat, xq);
    st<9>(xmat + 9 * i, mat);
    ldm<3>(ip, m.body_ipos + 3 * i);
    ldm<4>(iq, m.body_iquat + 4 * i);
    rot_vec_mat(tmp, ip, mat);
    double xi[3] = {tmp[0] + xp[0], tmp[1] + xp[1], tmp[2] + xp[2]};
    st<3>(xipos + 3 * i, xi);
    quat_mul(qloc, xq, iq);
    quat2mat(mat, qloc);
    st<9>(ximat + 9 * i, mat);
  }
  SPd gxpos = ln.D(L.gxpos), gxmat = ln.D(L.gxmat);
  for (int g = 0; g < m.ngeom; g++) {
    int b = m.geom_bodyid[g];
    double tmp[3], q[4], bm[9], bx[3], bq[4], gp[3], gq[4], mat[9];
    ld<9>(bm, xmat + 9 * b);
    ld<3>(bx, xpos + 3 * b);
    ld<4>(bq, xquat + 4 * b);
    ldm<3>(gp, m.geom_pos + 3 * g);
    ldm<4>(gq, m.geom_quat + 4 * g);
    rot_vec_mat(tmp, gp, bm);
    double o[3] = {tmp[0] + bx[0], tmp[1] + bx[1], tmp[2] + bx[2]};
    st<3>(gxpos + 3 * g, o);
    quat_mul(q, bq, gq);
    quat2mat(mat, q);
    st<9>(gxmat + 9 * g, mat);
  }
}

__device__ inline void com_pos(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nb = m.nbody;
  SPd xipos = ln.D(L.xipos), scom = ln.D(L.scom), cinert = ln.D(L.cinert), ximat = ln.D(L.ximat);
  SPd cdof = ln.D(L.cdof), xanchor = ln.D(L.xanchor), xaxis = ln.D(L.xaxis), xmat = ln.D(L.xmat);
  for (int i = 0; i < nb; i++) {
    double ms = m.body_mass[i];
    scom[3 * i] = xipos[3 * i] * ms;
    scom[3 * i + 1] = xipos[3 * i + 1] * ms;
    scom[3 * i + 2] = xipos[3 * i + 2] * ms;
  }
  for (int i = nb - 1; i > 0; i--) {
    int p = m.body_parentid[i];
    scom[3 * p] += scom[3 * i];
    scom[3 * p + 1] += scom[3 * i + 1];
    scom[3 * p + 2] += scom[3 * i + 2];
  }
  for (int i = 0; i < nb; i++) {
    if (m.body_subtreemass[i] < MINVAL) {
      scom[3 * i] = xipos[3 * i];
      scom[3 * i + 1] = xipos[3 * i + 1];
      scom[3 * i + 2] = xipos[3 * i + 2];
    } else {
      double inv = 1 / m.body_subtreemass[i];
      scom[3 * i] *= inv;
      scom[3 * i + 1] *= inv;
      scom[3 * i + 2] *= inv;
    }
  }
  for (int k = 0; k < 10; k++) cinert[k] = 0;
  for (int i = 1; i < nb; i++) {
    double off[3], rc[3], xi[3], mat[9], in[3], res[10];
    ld<3>(rc, scom + 3 * m.body_rootid[i]);
    ld<3>(xi, xipos + 3 * i);
    off[0] = xi[0] - rc[0]; off[1] = xi[1] - rc[1]; off[2] = xi[2] - rc[2];
    ld<9>(mat, ximat + 9 * i);
    ldm<3>(in, m.body_inertia + 3 * i);
    inert_com(res, in, mat, off, m.body_mass[i]);
    st<10>(cinert + 10 * i, res);
  }
  for (int j = 0; j < m.njnt; j++) {
    int da = 6 * m.jnt_dofadr[j];
    int bi = m.jnt_bodyid[j];
    double rc[3], an[3], out[6];
    ld<3>(rc, scom + 3 * m.body_rootid[bi]);
    ld<3>(an, xanchor + 3 * j);
    double off[3] = {rc[0] - an[0], rc[1] - an[1], rc[2] - an[2]};
    int type = m.jnt_type[j];
    int skip = 0;
    if (type == JNT_FREE) {
      for (int k = 0; k < 18; k++) cdof[da + k] = 0;
      for (int i = 0; i < 3; i++) cdof[da + 3 + 7 * i] = 1;
      skip = 18;
    }
    if (type == JNT_FREE || type == JNT_BALL) {
      for (int i = 0; i < 3; i++) {
        double axis[3] = {xmat[9 * bi + i], xmat[9 * bi + i + 3], xmat[9 * bi + i + 6]};
        out[0] = axis[0]; out[1] = axis[1]; out[2] = axis[2];
        cross3(out + 3, axis, off);
        st<6>(cdof + da + skip + 6 * i, out);
      }
    } else if (type == JNT_SLIDE) {
      double ax[3];
      ld<3>(ax, xaxis + 3 * j);
      out[0] = out[1] = out[2] = 0;
      out[3] = ax[0]; out[4] = ax[1]; out[5] = ax[2];
      st<6>(cdof + da, out);
    } else {
      double ax[3];
      ld<3>(ax, xaxis + 3 * j);
      out[0] = ax[0]; out[1] = ax[1]; out[2] = ax[2];
      cross3(out + 3, ax, off);
      st<6>(cdof + da, out);
    }
  }
}

__device__ inline void crb(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nv = m.nv;
  SPd crbv = ln.D(L.crb), cinert = ln.D(L.cinert), qM = ln.D(L.qM), cdof = ln.D(L.cdof);
  for (int k = 0; k < 10 * m.nbody; k++) crbv[k] = cinert[k];
  for (int i = m.nbody - 1; i > 0; i--) {
    int p = m.body_parentid[i];
    if (p > 0)
      for (int k = 0; k < 10; k++) crbv[10 * p + k] += crbv[10 * i + k];
  }
  for (int k = 0; k < nv * nv; k++) qM[k] = 0;
  for (int i = 0; i < nv; i++) {
    double buf[6], ci[10], cd[6];
    qM[i * nv + i] = m.dof_armature[i];
    ld<10>(ci, crbv + 10 * m.dof_bodyid[i]);
    ld<6>(cd, cdof + 6 * i);
    mul_inert_vec(buf, ci, cd);
    for (int j = i; j >= 0; j = m.dof_parentid[j]) {
      double cj[6], r = 0;
      ld<6>(cj, cdof + 6 * j);
      for (int k = 0; k < 6; k++) r += cj[k] * buf[k];
      qM[i * nv + j] += r;
    }
  }
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < i; j++) qM[j * nv + i] = qM[i * nv + j];
}

__device__ inline void factor_ld(const DevModel& m, SPd mat, SPd LD, SPd diaginv) {
  const int nv = m.nv;
  for (int i = 0; i < nv; i++)
    for (int j = 0; j < nv; j++) LD[i * nv + j] = (j <= i) ? mat[i * nv + j] : 0;
  for (int k = nv - 1; k >= 0; k--) {
    if (LD[k * nv + k] < MINVAL) LD[k * nv + k] = MINVAL;
    for (int i = m.dof_parentid[k]; i >= 0; i = m.dof_parentid[i]) {
      double tmp = LD[k * nv + i] / LD[k * nv + k];
      for (int j = i; j >= 0; j = m.dof_parentid[j]) LD[i * nv + j] -= tmp * LD[k * nv + j];
      LD[k * nv + i] = tmp;
    }
  }
  for (int i = 0; i < nv; i++) diaginv[i] = 1 / LD[i * nv + i];
}
__device__ inline void solve_ld(const DevModel& m, SPd LD, SPd diaginv, SPd x) {
  const int nv = m.nv;
  for (int i = nv - 1; i >= 0; i--) {
    double tmp = x[i];
    if (tmp != 0)
      for (int j = m.dof_parentid[i]; j >= 0; j = m.dof_parentid[j]) x[j] -= LD[i * nv + j] * tmp;
  }
  for (int i = 0; i < nv; i++) x[i] *= diaginv[i];
  for (int i = 0; i < nv; i++)
    for (int j = m.dof_parentid[i]; j >= 0; j = m.dof_parentid[j]) x[i] -= LD[i * nv + j] * x[j];
}
__device__ inline void mul_m(int nv, SPd M, SPd vec, SPd res) {
  for (int i = 0; i < nv; i++) res[i] = dotn(M + i * nv, vec, nv);
}

__device__ inline void jac_point(const DevModel& m, const WsLayout& L, const Lane& ln, SPd jacp,
                                 const double* point, int body) {
  const int nv = m.nv;
  SPd scom = ln.D(L.scom), cdof = ln.D(L.cdof);
  double rc[3], off[3];
  ld<3>(rc, scom + 3 * m.body_rootid[body]);
  for (int k = 0; k < 3 * nv; k++) jacp[k] = 0;
  off[0] = point[0] - rc[0]; off[1] = point[1] - rc[1]; off[2] = point[2] - rc[2];
  while (body && !m.body_dofnum[body]) body = m.body_parentid[body];
  if (!body) return;
  for (int i = m.body_dofadr[body] + m.body_dofnum[body] - 1; i >= 0; i = m.dof_parentid[i]) {
    double tmp[3], cd[6];
    ld<6>(cd, cdof + 6 * i);
    cross3(tmp, cd, off);
    jacp[i] = cd[3] + tmp[0];
    jacp[nv + i] = cd[4] + tmp[1];
    jacp[2 * nv + i] = cd[5] + tmp[2];
  }
}
__device__ inline void jac_rot(const DevModel& m, const WsLayout& L, const Lane& ln, SPd jacr, int body) {
  const int nv = m.nv;
  SPd cdof = ln.D(L.cdof);
  for (int k = 0; k < 3 * nv; k++) jacr[k] = 0;
  while (body && !m.body_dofnum[body]) body = m.body_parentid[body];
  if (!body) return;
  for (int i = m.body_dofadr[body] + m.body_dofnum[body] - 1; i >= 0; i = m.dof_parentid[i]) {
    jacr[i] = cdof[6 * i];
    jacr[nv + i] = cdof[6 * i + 1];
    jacr[2 * nv + i] = cdof[6 * i + 2];
  }
}

// ---- narrow phase (contacts: dist, pos[3], frame[0..2]) ----
// Contact k goes to a sink: RConSink (a private array, lane kernels) or
// LdsConSink (7-double records in LDS, cooperative kernels -- a runtime
// contact index into a private array would put it in scratch memory).
struct RCon {
  double dist, pos[3], n[3];
};
struct RConSink {
  RCon* c;
  __device__ __forceinline__ void put(int k, double d, const double* p, const double* n) const {
    c[k].dist = d;
    c[k].pos[0] = p[0]; c[k].pos[1] = p[1]; c[k].pos[2] = p[2];
    c[k].n[0] = n[0]; c[k].n[1] = n[1]; c[k].n[2] = n[2];
  }
};
struct LdsConSink {
  double* rec;  // contact k at rec + 7k: dist, pos[3], n[3]
  __device__ __forceinline__ void put(int k, double d, const double* p, const double* n) const {
    double* r = rec + 7 * k;
    r[0] = d;
    r[1] = p[0]; r[2] = p[1]; r[3] = p[2];
    r[4] = n[0]; r[5] = n[1]; r[6] = n[2];
  }
};
template <class S>
__device__ __forceinline__ int sphere_sphere(const S& out, int k, double margin, const double* p1, double r1,
                                             const double* p2, double r2) {
  double axis[3] = {p2[0] - p1[0], p2[1] - p1[1], p2[2] - p1[2]};
  double dist = normalize3(axis) - r1 - r2;
  if (dist > margin) return 0;
  const double s = r1 + dist / 2;
  const double pos[3] = {p1[0] + axis[0] * s, p1[1] + axis[1] * s, p1[2] + axis[2] * s};
  out.put(k, dist, pos, axis);
  return 1;
}
template <class S>
__device__ __forceinline__ int plane_sphere(const S& out, int k, double margin, const double* pos1,
                                            const double* mat1, const double* p2, double r2) {
  double n[3] = {mat1[2], mat1[5], mat1[8]};
  double tmp[3] = {p2[0] - pos1[0], p2[1] - pos1[1], p2[2] - pos1[2]};
  double cdist = dot3(tmp, n);
  if (cdist > margin + r2) return 0;
  const double dist = cdist - r2;
  const double s = -dist / 2 - r2;
  const double pos[3] = {p2[0] + n[0] * s, p2[1] + n[1] * s, p2[2] + n[2] * s};
  out.put(k, dist, pos, n);
  return 1;
}
template <class M, class S>
__device__ __forceinline__ int narrow(const M& m, int t1, int t2, const double* pos1, const double* mat1,
                                      const double* sz1, const double* pos2, const double* mat2, const double* sz2,
                                      double margin, const S& out) {
  if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) return plane_sphere(out, 0, margin, pos1, mat1, pos2, sz2[0]);
  if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
    double seg[3] = {mat2[2] * sz2[1], mat2[5] * sz2[1], mat2[8] * sz2[1]}, p[3];
    int n1, n2;
    p[0] = pos2[0] + seg[0]; p[1] = pos2[1] + seg[1]; p[2] = pos2[2] + seg[2];
    n1 = plane_sphere(out, 0, margin, pos1, mat1, p, sz2[0]);
    p[0] = pos2[0] - seg[0]; p[1] = pos2[1] - seg[1]; p[2] = pos2[2] - seg[2];
    n2 = plane_sphere(out, n1, margin, pos1, mat1, p, sz2[0]);
    return n1 + n2;
  }
  if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) return sphere_sphere(out, 0, margin, pos1, sz1[0], pos2, sz2[0]);
  if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
    double ax[3] = {mat2[2], mat2[5], mat2[8]}, dif[3], p[3], x;
    dif[0] = pos1[0] - pos2[0]; dif[1] = pos1[1] - pos2[1]; dif[2] = pos1[2] - pos2[2];
    x = clipd(dot3(ax, dif), -sz2[1], sz2[1]);
    p[0] = pos2[0] + ax[0] * x; p[1] = pos2[1] + ax[1] * x; p[2] = pos2[2] + ax[2] * x;
    return sphere_sphere(out, 0, margin, pos1, sz1[0], p, sz2[0]);
  }
  if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
    double a1[3] = {mat1[2] * sz1[1], mat1[5] * sz1[1], mat1[8] * sz1[1]};
    double a2[3] = {mat2[2] * sz2[1], mat2[5] * sz2[1], mat2[8] * sz2[1]};
    double dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
    double ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    double u = -dot3(a1, dif), v = dot3(a2, dif);
    double det = ma * mc - mb * mb;
    double v1[3], v2[3], x1, x2;
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

__device__ inline void collision(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int ng = m.ngeom;
  SPd gxpos = ln.D(L.gxpos), gxmat = ln.D(L.gxmat), con = ln.D(L.con);
  SPi coni = ln.I(L.coni);
  int ncon = 0;
  for (int g1 = 0; g1 < ng; g1++)
    for (int g2 = g1 + 1; g2 < ng; g2++) {
      int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
      int w1 = m.body_weldid[b1], w2 = m.body_weldid[b2];
      int wp1 = m.body_weldid[m.body_parentid[w1]], wp2 = m.body_weldid[m.body_parentid[w2]];
      if (w1 == w2) continue;
      if (w1 != 0 && w2 != 0 && (w1 == wp2 || w2 == wp1)) continue;
      if (!((m.geom_contype[g1] & m.geom_conaffinity[g2]) || (m.geom_contype[g2] & m.geom_conaffinity[g1])))
        continue;
      double margin = maxd(m.geom_margin[g1], m.geom_margin[g2]);
      if (m.geom_rbound[g1] > 0 && m.geom_rbound[g2] > 0) {
        double p1[3], p2[3];
        ld<3>(p1, gxpos + 3 * g1);
        ld<3>(p2, gxpos + 3 * g2);
        double dd[3] = {p1[0] - p2[0], p1[1] - p2[1], p1[2] - p2[2]};
        if (sqrt(dot3(dd, dd)) > m.geom_rbound[g1] + m.geom_rbound[g2] + margin) continue;
      }
      int ga = g1, gb = g2;
      if (m.geom_type[g1] > m.geom_type[g2]) { ga = g2; gb = g1; }
      double pos1[3], mat1[9], sz1[3], pos2[3], mat2[9], sz2[3];
      ld<3>(pos1, gxpos + 3 * ga);
      ld<9>(mat1, gxmat + 9 * ga);
      ldm<3>(sz1, m.geom_size + 3 * ga);
      ld<3>(pos2, gxpos + 3 * gb);
      ld<9>(mat2, gxmat + 9 * gb);
      ldm<3>(sz2, m.geom_size + 3 * gb);
      RCon tmp[2];
      int n = narrow(m, m.geom_type[ga], m.geom_type[gb], pos1, mat1, sz1, pos2, mat2, sz2, margin, RConSink{tmp});
      if (!n) continue;
      double gap = maxd(m.geom_gap[ga], m.geom_gap[gb]);
      double s1 = m.geom_solmix[ga], s2 = m.geom_solmix[gb], mix;
      if (s1 < MINVAL && s2 < MINVAL) mix = 0.5;
      else if (s1 < MINVAL) mix = 0;
      else if (s2 < MINVAL) mix = 1;
      else mix = s1 / (s1 + s2);
      for (int k = 0; k < n; k++) {
        if (ncon >= m.nconmax || ncon >= m.maxcon) break;
        SPd c = con + CON_ND * ncon;
        double fr[9];
        fr[0] = tmp[k].n[0]; fr[1] = tmp[k].n[1]; fr[2] = tmp[k].n[2];
        make_frame(fr);
        c[CON_DIST] = tmp[k].dist;
        c[CON_POS] = tmp[k].pos[0]; c[CON_POS + 1] = tmp[k].pos[1]; c[CON_POS + 2] = tmp[k].pos[2];
        for (int r = 0; r < 9; r++) c[CON_FRAME + r] = fr[r];
        c[CON_INCLM] = margin - gap;
        double f0 = maxd(m.geom_friction[3 * ga], m.geom_friction[3 * gb]);
        double f1 = maxd(m.geom_friction[3 * ga + 1], m.geom_friction[3 * gb + 1]);
        double f2 = maxd(m.geom_friction[3 * ga + 2], m.geom_friction[3 * gb + 2]);
        c[CON_FRIC] = f0; c[CON_FRIC + 1] = f0; c[CON_FRIC + 2] = f1; c[CON_FRIC + 3] = f2; c[CON_FRIC + 4] = f2;
        for (int r = 0; r < 2; r++)
          c[CON_SOLREF + r] = mix * m.geom_solref[2 * ga + r] + (1 - mix) * m.geom_solref[2 * gb + r];
        for (int r = 0; r < 5; r++)
          c[CON_SOLIMP + r] = mix * m.geom_solimp[5 * ga + r] + (1 - mix) * m.geom_solimp[5 * gb + r];
        int cd1 = m.geom_condim[ga], cd2 = m.geom_condim[gb];
        coni[CON_NI * ncon + CONI_DIM] = cd1 > cd2 ? cd1 : cd2;
        coni[CON_NI * ncon + CONI_G1] = ga;
        coni[CON_NI * ncon + CONI_G2] = gb;
        coni[CON_NI * ncon + CONI_EFCADR] = -1;
        ncon++;
      }
    }
  ln.I(L.ncon)[0] = ncon;
}

__device__ inline double get_impedance(const double* solimp, double pos, double margin) {
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

__device__ inline void make_constraint(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nv = m.nv;
  SPd qpos = ln.D(L.qpos), con = ln.D(L.con), efcJ = ln.D(L.efc_J), efc_pos = ln.D(L.efc_pos);
  SPd efc_margin = ln.D(L.efc_margin), efc_D = ln.D(L.efc_D), KBIP = ln.D(L.efc_KBIP);
  SPi coni = ln.I(L.coni), efc_type = ln.I(L.efc_type), efc_id = ln.I(L.efc_id);
  SPd sc = ln.D(L.s_con);
  SPd j1 = sc + nv, j2 = sc + 4 * nv, jc = sc + 7 * nv;
  const int ncon = ln.I(L.ncon)[0];
  const int njmax = m.njmax < m.maxefc ? m.njmax : m.maxefc;
  int nefc = 0;
  for (int j = 0; j < m.njnt; j++) {
    int type = m.jnt_type[j];
    if (!m.jnt_limited[j] || (type != JNT_SLIDE && type != JNT_HINGE)) continue;
    double value = qpos[m.jnt_qposadr[j]];
    for (int side = -1; side <= 1; side += 2) {
      double dist = side * (m.jnt_range[2 * j + (side + 1) / 2] - value);
      if (dist < m.jnt_margin[j]) {
        if (nefc + 1 > njmax) break;
        SPd row = efcJ + nefc * nv;
        for (int k = 0; k < nv; k++) row[k] = 0;
        row[m.jnt_dofadr[j]] = -side;
        efc_pos[nefc] = dist;
        efc_margin[nefc] = m.jnt_margin[j];
        efc_type[nefc] = C_LIMIT;
        efc_id[nefc] = j;
        nefc++;
      }
    }
  }
  for (int c = 0; c < ncon; c++) {
    SPd cc = con + CON_ND * c;
    int dim = coni[CON_NI * c + CONI_DIM];
    int b1 = m.geom_bodyid[coni[CON_NI * c + CONI_G1]], b2 = m.geom_bodyid[coni[CON_NI * c + CONI_G2]];
    int nrow = dim == 1 ? 1 : 2 * (dim - 1);
    if (nefc + nrow > njmax) continue;
    double pos[3], fr[9];
    ld<3>(pos, cc + CON_POS);
    ld<9>(fr, cc + CON_FRAME);
    jac_point(m, L, ln, j1, pos, b1);
    jac_point(m, L, ln, j2, pos, b2);
    for (int k = 0; k < 3 * nv; k++) j2[k] -= j1[k];
    for (int r = 0; r < 3; r++)
      for (int k = 0; k < nv; k++)
        jc[r * nv + k] = fr[3 * r] * j2[k] + fr[3 * r + 1] * j2[nv + k] + fr[3 * r + 2] * j2[2 * nv + k];
    coni[CON_NI * c + CONI_EFCADR] = nefc;
    double dist = cc[CON_DIST], inclm = cc[CON_INCLM];
    if (dim == 1) {
      SPd row = efcJ + nefc * nv;
      for (int i = 0; i < nv; i++) row[i] = jc[i];
      efc_pos[nefc] = dist; efc_margin[nefc] = inclm; efc_type[nefc] = C_FRICTIONLESS; efc_id[nefc] = c;
      nefc++;
    } else {
      for (int k = 1; k < dim; k++) {
        double f = cc[CON_FRIC + k - 1];
        SPd row = efcJ + nefc * nv;
        for (int i = 0; i < nv; i++) row[i] = jc[i] + f * jc[k * nv + i];
        efc_pos[nefc] = dist; efc_margin[nefc] = inclm; efc_type[nefc] = C_PYRAMIDAL; efc_id[nefc] = c;
        nefc++;
        row = efcJ + nefc * nv;
        for (int i = 0; i < nv; i++) row[i] = jc[i] + (-f) * jc[k * nv + i];
        efc_pos[nefc] = dist; efc_margin[nefc] = inclm; efc_type[nefc] = C_PYRAMIDAL; efc_id[nefc] = c;
        nefc++;
      }
    }
  }
  for (int i = 0; i < nefc; i++) {
    double solref[2], solimp[5], dA, imp, tc, dr, dmax, K, B;
    int id = efc_id[i];
    if (efc_type[i] == C_LIMIT) {
      ldm<2>(solref, m.jnt_solref + 2 * id);
      ldm<5>(solimp, m.jnt_solimp + 5 * id);
      dA = m.dof_invweight0[m.jnt_dofadr[id]];
    } else {
      SPd cc = con + CON_ND * id;
      int b1 = m.geom_bodyid[coni[CON_NI * id + CONI_G1]], b2 = m.geom_bodyid[coni[CON_NI * id + CONI_G2]];
      double tran = m.body_invweight0[2 * b1] + m.body_invweight0[2 * b2];
      ld<2>(solref, cc + CON_SOLREF);
      ld<5>(solimp, cc + CON_SOLIMP);
      if (efc_type[i] == C_FRICTIONLESS) {
        dA = tran;
      } else {
        int k = (i - coni[CON_NI * id + CONI_EFCADR]) / 2;
        double f = cc[CON_FRIC + k];
        dA = tran + f * f * tran;
      }
    }
    imp = get_impedance(solimp, efc_pos[i], efc_margin[i]);
    dmax = clipd(solimp[1], MINIMP, MAXIMP);
    tc = solref[0];
    dr = solref[1];
    if (tc > 0) {
      if (tc < 2 * m.opt_timestep) tc = 2 * m.opt_timestep;
      K = 1 / (dmax * dmax * tc * tc * dr * dr);
      B = 2 / (dmax * tc);
    } else {
      K = -tc / (dmax * dmax);
      B = -dr / dmax;
    }
    KBIP[4 * i] = K;
    KBIP[4 * i + 1] = B;
    KBIP[4 * i + 2] = imp;
    KBIP[4 * i + 3] = 0;
    double R = maxd(MINVAL, (1 - imp) * dA / imp);
    efc_D[i] = 1 / R;
  }
  ln.I(L.nefc)[0] = nefc;
}

__device__ inline void transmission(const DevModel& m, const WsLayout& L, const Lane& ln) {
  SPd amom = ln.D(L.amom);
  const int nv = m.nv;
  for (int k = 0; k < m.nu * nv; k++) amom[k] = 0;
  for (int i = 0; i < m.nu; i++) {
    int j = m.actuator_trnid[i];
    amom[i * nv + m.jnt_dofadr[j]] = m.actuator_gear[i];
  }
}

__device__ inline void fwd_position(const DevModel& m, const WsLayout& L, const Lane& ln) {
  kinematics(m, L, ln);
  com_pos(m, L, ln);
  transmission(m, L, ln);
  crb(m, L, ln);
  factor_ld(m, ln.D(L.qM), ln.D(L.qLD), ln.D(L.qLDinv));
  collision(m, L, ln);
  make_constraint(m, L, ln);
}

// ------------------------------------------------------ velocity stage ---
__device__ inline void com_vel(const DevModel& m, const WsLayout& L, const Lane& ln) {
  SPd cvelw = ln.D(L.cvel), cdof = ln.D(L.cdof), cdd = ln.D(L.cdof_dot), qvel = ln.D(L.qvel);
  for (int k = 0; k < 6; k++) cvelw[k] = 0;
  for (int i = 1; i < m.nbody; i++) {
    int bda = m.body_dofadr[i];
    double cvel[6], tmp[6], cd[6], r[6];
    ld<6>(cvel, cvelw + 6 * m.body_parentid[i]);
    for (int j = 0; j < m.body_dofnum[i]; j++) {
      int type = m.jnt_type[m.dof_jntid[bda + j]];
      if (type == JNT_FREE) {
        for (int k = 0; k < 18; k++) cdd[6 * (bda + j) + k] = 0;
        for (int k = 0; k < 6; k++) {
          double s = 0;
          for (int q = 0; q < 3; q++) s += cdof[6 * (bda + q) + k] * qvel[bda + q];
          tmp[k] = s;
        }
        for (int k = 0; k < 6; k++) cvel[k] += tmp[k];
        j += 3;
      }
      if (type == JNT_FREE || type == JNT_BALL) {
        for (int k = 0; k < 3; k++) {
          ld<6>(cd, cdof + 6 * (bda + j + k));
          cross_motion(r, cvel, cd);
          st<6>(cdd + 6 * (bda + j + k), r);
        }
        for (int k = 0; k < 6; k++) {
          double s = 0;
          for (int q = 0; q < 3; q++) s += cdof[6 * (bda + j + q) + k] * qvel[bda + j + q];
          tmp[k] = s;
        }
        for (int k = 0; k < 6; k++) cvel[k] += tmp[k];
        j += 2;
      } else {
        ld<6>(cd, cdof + 6 * (bda + j));
        cross_motion(r, cvel, cd);
        st<6>(cdd + 6 * (bda + j), r);
        double qv = qvel[bda + j];
        for (int k = 0; k < 6; k++) {
          double s = 0;
          s += cd[k] * qv;
          tmp[k] = s;
        }
        for (int k = 0; k < 6; k++) cvel[k] += tmp[k];
      }
    }
    st<6>(cvelw + 6 * i, cvel);
  }
}

__device__ inline void passive(const DevModel& m, const WsLayout& L, const Lane& ln) {
  SPd qp = ln.D(L.qfrc_passive), qpos = ln.D(L.qpos), qvel = ln.D(L.qvel);
  for (int i = 0; i < m.nv; i++) qp[i] = 0;
  for (int j = 0; j < m.njnt; j++) {
    double k = m.jnt_stiffness[j];
    int pa = m.jnt_qposadr[j], da = m.jnt_dofadr[j];
    if (k == 0) continue;
    // ball/free springs are rejected at solver creation (need atan2)
    qp[da] = -k * (qpos[pa] - m.qpos_spring[pa]);
  }
  for (int i = 0; i < m.nv; i++) qp[i] -= m.dof_damping[i] * qvel[i];
}

__device__ inline void reference_constraint(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nefc = ln.I(L.nefc)[0], nv = m.nv;
  SPd KBIP = ln.D(L.efc_KBIP), vel = ln.D(L.efc_vel), aref = ln.D(L.efc_aref), J = ln.D(L.efc_J);
  SPd pos = ln.D(L.efc_pos), mar = ln.D(L.efc_margin), qvel = ln.D(L.qvel);
  for (int i = 0; i < nefc; i++) {
    double k0 = KBIP[4 * i], k1 = KBIP[4 * i + 1], k2 = KBIP[4 * i + 2];
    double v = dotn(J + i * nv, qvel, nv);
    vel[i] = v;
    aref[i] = -k1 * v - k0 * k2 * (pos[i] - mar[i]);
  }
}

__device__ inline void rne(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nb = m.nbody;
  SPd s = ln.D(L.s_rne), cacc = s, cfrc = s + 6 * nb;
  SPd cdd = ln.D(L.cdof_dot), qvel = ln.D(L.qvel), cinert = ln.D(L.cinert), cvel = ln.D(L.cvel);
  SPd cdof = ln.D(L.cdof), bias = ln.D(L.qfrc_bias);
  for (int k = 0; k < 6; k++) cacc[k] = 0;
  cacc[3] = -m.opt_gravity0;
  cacc[4] = -m.opt_gravity1;
  cacc[5] = -m.opt_gravity2;
  for (int i = 1; i < nb; i++) {
    int bda = m.body_dofadr[i], nd = m.body_dofnum[i];
    int p = m.body_parentid[i];
    double tmp[6], tmp1[6], ci[10], a[6], f[6], cv[6];
    for (int k = 0; k < 6; k++) {
      double sum = 0;
      for (int j = 0; j < nd; j++) sum += cdd[6 * (bda + j) + k] * qvel[bda + j];
      tmp[k] = nd ? sum : 0;
    }
    for (int k = 0; k < 6; k++) a[k] = cacc[6 * p + k] + tmp[k];
    st<6>(cacc + 6 * i, a);
    ld<10>(ci, cinert + 10 * i);
    ld<6>(cv, cvel + 6 * i);
    mul_inert_vec(f, ci, a);
    mul_inert_vec(tmp, ci, cv);
    cross_force(tmp1, cv, tmp);
    for (int k = 0; k < 6; k++) f[k] += tmp1[k];
    st<6>(cfrc + 6 * i, f);
  }
  for (int k = 0; k < 6; k++) cfrc[k] = 0;
  for (int i = nb - 1; i > 0; i--) {
    int p = m.body_parentid[i];
    if (p)
      for (int k = 0; k < 6; k++) cfrc[6 * p + k] += cfrc[6 * i + k];
  }
  for (int i = 0; i < m.nv; i++) bias[i] = dotn(cdof + 6 * i, cfrc + 6 * m.dof_bodyid[i], 6);
}

__device__ inline void fwd_velocity(const DevModel& m, const WsLayout& L, const Lane& ln) {
  com_vel(m, L, ln);
  passive(m, L, ln);
  reference_constraint(m, L, ln);
  rne(m, L, ln);
}

// -------------------------------------------------- acceleration stage ---
__device__ inline void fwd_actuation(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nv = m.nv, nu = m.nu;
  SPd ctrl = ln.D(L.ctrl), af = ln.D(L.afrc), amom = ln.D(L.amom), qa = ln.D(L.qfrc_act);
  for (int i = 0; i < nu; i++) {
    double c = ctrl[i], f;
    if (m.actuator_ctrllimited[i]) c = clipd(c, m.actuator_ctrlrange[2 * i], m.actuator_ctrlrange[2 * i + 1]);
    f = m.actuator_gainprm[i] * c;
    if (m.actuator_forcelimited[i]) f = clipd(f, m.actuator_forcerange[2 * i], m.actuator_forcerange[2 * i + 1]);
    af[i] = f;
  }
  for (int j = 0; j < nv; j++) {
    double s = 0;
    for (int i = 0; i < nu; i++) s += amom[i * nv + j] * af[i];
    qa[j] = s;
  }
}

__device__ inline void xfrc_accumulate(const DevModel& m, const WsLayout& L, const Lane& ln, SPd qfrc) {
  const int nv = m.nv;
  SPd xf = ln.D(L.xfrc_applied), xipos = ln.D(L.xipos);
  SPd sc = ln.D(L.s_con), jp = sc + nv, jr = sc + 4 * nv;
  for (int b = 1; b < m.nbody; b++) {
    double f[6];
    ld<6>(f, xf + 6 * b);
    if (f[0] == 0 && f[1] == 0 && f[2] == 0 && f[3] == 0 && f[4] == 0 && f[5] == 0) continue;
    double p[3];
    ld<3>(p, xipos + 3 * b);
    jac_point(m, L, ln, jp, p, b);
    jac_rot(m, L, ln, jr, b);
    for (int j = 0; j < nv; j++) {
      double t1 = jp[j] * f[0] + jp[nv + j] * f[1] + jp[2 * nv + j] * f[2];
      double t2 = jr[j] * f[3] + jr[nv + j] * f[4] + jr[2 * nv + j] * f[5];
      qfrc[j] += t1 + t2;
    }
  }
}

__device__ inline void fwd_acceleration(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nv = m.nv;
  SPd sm = ln.D(L.qfrc_smooth), qp = ln.D(L.qfrc_passive), qb = ln.D(L.qfrc_bias);
  SPd qap = ln.D(L.qfrc_applied), qac = ln.D(L.qfrc_act), qs = ln.D(L.qacc_smooth);
  for (int i = 0; i < nv; i++) sm[i] = qp[i] - qb[i];
  for (int i = 0; i < nv; i++) sm[i] += qap[i];
  for (int i = 0; i < nv; i++) sm[i] += qac[i];
  xfrc_accumulate(m, L, ln, sm);
  for (int i = 0; i < nv; i++) qs[i] = sm[i];
  solve_ld(m, ln.D(L.qLD), ln.D(L.qLDinv), qs);
}

__device__ inline double constraint_update(const DevModel& m, const WsLayout& L, const Lane& ln, SPd jar) {
  const int nv = m.nv, ne = ln.I(L.nefc)[0];
  SPd D = ln.D(L.efc_D), force = ln.D(L.efc_force), J = ln.D(L.efc_J), qc = ln.D(L.qfrc_con);
  SPi state = ln.I(L.efc_state);
  double cost = 0;
  for (int i = 0; i < ne; i++) {
    double jr = jar[i];
    if (jr < 0) {
      double Di = D[i];
      force[i] = -Di * jr;
      state[i] = 1;
      cost += 0.5 * Di * jr * jr;
    } else {
      force[i] = 0;
      state[i] = 0;
    }
  }
  for (int j = 0; j < nv; j++) {
    double s = 0;
    for (int i = 0; i < ne; i++) s += J[i * nv + j] * force[i];
    qc[j] = s;
  }
  return cost;
}
__device__ inline double gauss_cost(int nv, SPd Ma, SPd qfrc_smooth, SPd qacc, SPd qacc_smooth) {
  double s = 0;
  for (int j = 0; j < nv; j++) s += (Ma[j] - qfrc_smooth[j]) * (qacc[j] - qacc_smooth[j]);
  return 0.5 * s;
}
__device__ inline void hessian_factor(const DevModel& m, const WsLayout& L, const Lane& ln, SPd H) {
  const int nv = m.nv, ne = ln.I(L.nefc)[0];
  SPd J = ln.D(L.efc_J), D = ln.D(L.efc_D), qM = ln.D(L.qM);
  SPi state = ln.I(L.efc_state);
  for (int r = 0; r < nv; r++)
    for (int c = 0; c <= r; c++) {
      double h = 0;
      for (int i = 0; i < ne; i++)
        if (state[i]) h += J[i * nv + r] * D[i] * J[i * nv + c];
      H[r * nv + c] = qM[r * nv + c] + h;
    }
  for (int j = 0; j < nv; j++) {
    double t = H[j * nv + j];
    if (j) t -= dotn(H + j * nv, H + j * nv, j);
    if (t < MINVAL) t = MINVAL;
    H[j * nv + j] = sqrt(t);
    t = 1 / H[j * nv + j];
    for (int i = j + 1; i < nv; i++) H[i * nv + j] = (H[i * nv + j] - dotn(H + i * nv, H + j * nv, j)) * t;
  }
}
__device__ inline void chol_solve(int nv, SPd Lm, SPd b, SPd x) {
  for (int i = 0; i < nv; i++) x[i] = b[i];
  for (int i = 0; i < nv; i++) {
    if (i) x[i] -= dotn(Lm + i * nv, x, i);
    x[i] /= Lm[i * nv + i];
  }
  for (int i = nv - 1; i >= 0; i--) {
    for (int j = i + 1; j < nv; j++) x[i] -= Lm[j * nv + i] * x[j];
    x[i] /= Lm[i * nv + i];
  }
}

__device__ inline double linesearch(const DevModel& m, const WsLayout& L, const Lane& ln, SPd search, SPd Ma,
                                    SPd jar, SPd Mv, SPd Jv) {
  const int nv = m.nv, ne = ln.I(L.nefc)[0];
  SPd qM = ln.D(L.qM), J = ln.D(L.efc_J), D = ln.D(L.efc_D), qs = ln.D(L.qfrc_smooth);
  double snorm = sqrt(dotn(search, search, nv)), g1 = 0, g2 = 0;
  double alpha = 0, d1, d2, lo = 0, hi = -1, gtol;
  if (snorm < MINVAL) return 0;
  mul_m(nv, qM, search, Mv);
  for (int i = 0; i < ne; i++) Jv[i] = dotn(J + i * nv, search, nv);
  for (int j = 0; j < nv; j++) g1 += search[j] * (Ma[j] - qs[j]);
  for (int j = 0; j < nv; j++) g2 += search[j] * Mv[j];
  auto eval = [&](double a) {
    d1 = g1 + g2 * a;
    d2 = g2;
    for (int i = 0; i < ne; i++) {
      double jv = Jv[i];
      double x = jar[i] + a * jv;
      if (x < 0) {
        double Di = D[i];
        d1 += Di * x * jv;
        d2 += Di * jv * jv;
      }
    }
  };
  eval(0.0);
  if (d1 >= 0) return 0;
  gtol = LS_TOL * fabs(d1);
  for (int it = 0; it < LS_ITER; it++) {
    double anew = alpha - d1 / d2;
    if (hi >= 0 && !(anew > lo && anew < hi)) anew = 0.5 * (lo + hi);
    alpha = anew;
    eval(alpha);
    if (fabs(d1) < gtol) break;
    if (d1 < 0) lo = alpha; else hi = alpha;
  }
  return alpha;
}

__device__ inline void solver_newton(const DevModel& m, const WsLayout& L, const Lane& ln, int maxiter, double tol) {
  const int nv = m.nv, ne = ln.I(L.nefc)[0];
  double scale = 1 / (m.stat_meaninertia * (nv > 1 ? nv : 1));
  SPd s = ln.D(L.s_newton);
  SPd Ma = s, grad = s + nv, search = s + 2 * nv, Mv = s + 3 * nv, H = s + 4 * nv;
  SPd jar = s + 4 * nv + nv * nv, Jv = jar + ne;
  SPd qM = ln.D(L.qM), qacc = ln.D(L.qacc), J = ln.D(L.efc_J), aref = ln.D(L.efc_aref);
  SPd qfs = ln.D(L.qfrc_smooth), qas = ln.D(L.qacc_smooth), qc = ln.D(L.qfrc_con);
  double cost, oldcost, improvement, gradient;
  int iter = 0;
  mul_m(nv, qM, qacc, Ma);
  for (int i = 0; i < ne; i++) jar[i] = dotn(J + i * nv, qacc, nv) - aref[i];
  cost = gauss_cost(nv, Ma, qfs, qacc, qas) + constraint_update(m, L, ln, jar);
  for (int j = 0; j < nv; j++) grad[j] = (Ma[j] - qfs[j]) - qc[j];
  hessian_factor(m, L, ln, H);
  while (iter < maxiter) {
    chol_solve(nv, H, grad, search);
    for (int j = 0; j < nv; j++) search[j] = -search[j];
    double alpha = linesearch(m, L, ln, search, Ma, jar, Mv, Jv);
    if (alpha == 0) break;
    for (int j = 0; j < nv; j++) qacc[j] += alpha * search[j];
    for (int j = 0; j < nv; j++) Ma[j] += alpha * Mv[j];
    for (int i = 0; i < ne; i++) jar[i] += alpha * Jv[i];
    iter++;
    oldcost = cost;
    cost = gauss_cost(nv, Ma, qfs, qacc, qas) + constraint_update(m, L, ln, jar);
    for (int j = 0; j < nv; j++) grad[j] = (Ma[j] - qfs[j]) - qc[j];
    improvement = scale * (oldcost - cost);
    gradient = scale * sqrt(dotn(grad, grad, nv));
    if (improvement < tol || gradient < tol) break;
    hessian_factor(m, L, ln, H);
  }
}

__device__ inline void fwd_constraint(const DevModel& m, const WsLayout& L, const Lane& ln, int maxiter, double tol) {
  const int nv = m.nv, ne = ln.I(L.nefc)[0];
  SPd qacc = ln.D(L.qacc), warm = ln.D(L.warm), qas = ln.D(L.qacc_smooth), qc = ln.D(L.qfrc_con);
  if (!ne) {
    for (int i = 0; i < nv; i++) { double v = qas[i]; qacc[i] = v; warm[i] = v; qc[i] = 0; }
    return;
  }
  {
    SPd s = ln.D(L.s_newton);
    SPd Ma = s, jar = s + 4 * nv + nv * nv;
    SPd J = ln.D(L.efc_J), aref = ln.D(L.efc_aref), b = ln.D(L.efc_b), qM = ln.D(L.qM), qfs = ln.D(L.qfrc_smooth);
    for (int i = 0; i < ne; i++) b[i] = dotn(J + i * nv, qas, nv) - aref[i];
    double cost_smooth = constraint_update(m, L, ln, b);
    mul_m(nv, qM, warm, Ma);
    for (int i = 0; i < ne; i++) jar[i] = dotn(J + i * nv, warm, nv) - aref[i];
    double cost_warm = gauss_cost(nv, Ma, qfs, warm, qas) + constraint_update(m, L, ln, jar);
    if (cost_warm > cost_smooth)
      for (int i = 0; i < nv; i++) qacc[i] = qas[i];
    else
      for (int i = 0; i < nv; i++) qacc[i] = warm[i];
  }
  solver_newton(m, L, ln, maxiter, tol);
  for (int i = 0; i < nv; i++) warm[i] = qacc[i];
}

// ----------------------------------------------------------- top level ---
__device__ inline void forward_skip(const DevModel& m, const WsLayout& L, const Lane& ln, int skipstage,
                                    int maxiter, double tol) {
  if (skipstage < STAGE_POS) fwd_position(m, L, ln);
  if (skipstage < STAGE_VEL) fwd_velocity(m, L, ln);
  fwd_actuation(m, L, ln);
  fwd_acceleration(m, L, ln);
  fwd_constraint(m, L, ln, maxiter, tol);
}

__device__ inline void integrate_pos(const DevModel& m, SPd qpos, SPd qvel, double dt) {
  for (int j = 0; j < m.njnt; j++) {
    int pa = m.jnt_qposadr[j], va = m.jnt_dofadr[j];
    int type = m.jnt_type[j];
    if (type == JNT_FREE || type == JNT_BALL) {
      if (type == JNT_FREE) {
        for (int i = 0; i < 3; i++) qpos[pa + i] += dt * qvel[va + i];
        pa += 3; va += 3;
      }
      double q[4], v[3];
      ld<4>(q, qpos + pa);
      ld<3>(v, qvel + va);
      quat_integrate(q, v, dt);
      st<4>(qpos + pa, q);
    } else {
      qpos[pa] += dt * qvel[va];
    }
  }
}

__device__ inline void reset_data(const DevModel& m, const WsLayout& L, const Lane& ln) {
  SPd qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), ctrl = ln.D(L.ctrl), warm = ln.D(L.warm);
  SPd qap = ln.D(L.qfrc_applied), xf = ln.D(L.xfrc_applied);
  for (int i = 0; i < m.nq; i++) qpos[i] = m.qpos0[i];
  for (int i = 0; i < m.nv; i++) { qvel[i] = 0; warm[i] = 0; qap[i] = 0; }
  for (int i = 0; i < m.nu; i++) ctrl[i] = 0;
  for (int i = 0; i < 6 * m.nbody; i++) xf[i] = 0;
  ln.D(L.time)[0] = 0;
}

__device__ inline bool is_bad(double x) { return x != x || x > MAXVAL || x < -MAXVAL; }

__device__ inline void euler(const DevModel& m, const WsLayout& L, const Lane& ln) {
  const int nv = m.nv;
  SPd s = ln.D(L.s_euler), qacc = s, qH = s + nv, qHLD = s + nv + nv * nv, qHinv = s + nv + 2 * nv * nv;
  SPd qM = ln.D(L.qM), dq = ln.D(L.qacc), qvel = ln.D(L.qvel);
  int dmp = 0;
  for (int i = 0; i < nv; i++)
    if (m.dof_damping[i] > 0) { dmp = 1; break; }
  if (!dmp) {
    for (int i = 0; i < nv; i++) qacc[i] = dq[i];
  } else {
    mul_m(nv, qM, dq, qacc);
    for (int k = 0; k < nv * nv; k++) qH[k] = qM[k];
    for (int i = 0; i < nv; i++) qH[i * nv + i] += m.opt_timestep * m.dof_damping[i];
    factor_ld(m, qH, qHLD, qHinv);
    solve_ld(m, qHLD, qHinv, qacc);
  }
  double h = m.opt_timestep;
  for (int i = 0; i < nv; i++) qvel[i] += qacc[i] * h;
  integrate_pos(m, ln.D(L.qpos), qvel, h);
  ln.D(L.time)[0] += h;
}

__device__ inline void rk4(const DevModel& m, const WsLayout& L, const Lane& ln, int maxiter, double tol) {
  const double A[9] = {0.5, 0, 0, 0, 0.5, 0, 0, 0, 1};
  const double Bw[4] = {1.0 / 6, 1.0 / 3, 1.0 / 3, 1.0 / 6};
  const int nv = m.nv, nq = m.nq, N = 4;
  const double h = m.opt_timestep;
  SPd timew = ln.D(L.time), qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), qaccw = ln.D(L.qacc);
  double time = timew[0], C[3], T[3];
  SPd s = ln.D(L.s_rk4), dX = s, X = s + 2 * nv, F = s + 2 * nv + 4 * (nq + nv);
  for (int i = 1; i < N; i++) {
    C[i - 1] = 0;
    for (int j = 0; j < i; j++) C[i - 1] += A[(i - 1) * (N - 1) + j];
    T[i - 1] = time + C[i - 1] * h;
  }
  for (int k = 0; k < nq; k++) X[k] = qpos[k];
  for (int k = 0; k < nv; k++) X[nq + k] = qvel[k];
  for (int k = 0; k < nv; k++) F[k] = qaccw[k];
  for (int i = 1; i < N; i++) {
    SPd Xi = X + i * (nq + nv);
    for (int k = 0; k < 2 * nv; k++) dX[k] = 0;
    for (int j = 0; j < i; j++) {
      double a = A[(i - 1) * (N - 1) + j];
      SPd Xj = X + j * (nq + nv), Fj = F + j * nv;
      for (int k = 0; k < nv; k++) dX[k] += Xj[nq + k] * a;
      for (int k = 0; k < nv; k++) dX[nv + k] += Fj[k] * a;
    }
    for (int k = 0; k < nq + nv; k++) Xi[k] = X[k];
    integrate_pos(m, Xi, dX, h);
    for (int k = 0; k < nv; k++) Xi[nq + k] += dX[nv + k] * h;
    for (int k = 0; k < nq; k++) qpos[k] = Xi[k];
    for (int k = 0; k < nv; k++) qvel[k] = Xi[nq + k];
    timew[0] = T[i - 1];
    forward_skip(m, L, ln, STAGE_NONE, maxiter, tol);
    SPd Fi = F + i * nv;
    for (int k = 0; k < nv; k++) Fi[k] = qaccw[k];
  }
  for (int k = 0; k < 2 * nv; k++) dX[k] = 0;
  for (int j = 0; j < N; j++) {
    SPd Xj = X + j * (nq + nv), Fj = F + j * nv;
    for (int k = 0; k < nv; k++) dX[k] += Xj[nq + k] * Bw[j];
    for (int k = 0; k < nv; k++) dX[nv + k] += Fj[k] * Bw[j];
  }
  timew[0] = time;
  for (int k = 0; k < nq; k++) qpos[k] = X[k];
  for (int k = 0; k < nv; k++) qvel[k] = X[nq + k];
  for (int i = 0; i < nv; i++) qvel[i] += dX[nv + i] * h;
  integrate_pos(m, qpos, dX, h);
  timew[0] += h;
}

// mj_step with the model's own solver settings
__device__ inline void step(const DevModel& m, const WsLayout& L, const Lane& ln) {
  SPd qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), qacc = ln.D(L.qacc);
  for (int i = 0; i < m.nq; i++)
    if (is_bad(qpos[i])) { reset_data(m, L, ln); break; }
  for (int i = 0; i < m.nv; i++)
    if (is_bad(qvel[i])) { reset_data(m, L, ln); break; }
  forward_skip(m, L, ln, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
  for (int i = 0; i < m.nv; i++)
    if (is_bad(qacc[i])) {
      reset_data(m, L, ln);
      forward_skip(m, L, ln, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
      break;
    }
  if (m.opt_integrator == 1)
    rk4(m, L, ln, m.opt_iterations, m.opt_tolerance);
  else
    euler(m, L, ln);
}

}  // namespace dev
}  // namespace ilqg
