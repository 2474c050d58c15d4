// mj_setConst at qpos0 (MuJoCo 2.0 semantics): subtree masses, mean inertia,
// dof/body inverse weights that the constraint regulariser's diagApprox uses.
// Model compilation only (host, runs once per model); not on the hot path.
#include <cmath>
#include <vector>

#include "model.h"

namespace ilqg {
namespace {

void quat_mul(double* r, const double* a, const double* b) {
  double t[4] = {a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                 a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                 a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                 a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]};
  for (int k = 0; k < 4; k++) r[k] = t[k];
}
void quat2mat(double* r, const double* q) {
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  r[0] = q00 + q11 - q22 - q33; r[4] = q00 - q11 + q22 - q33; r[8] = q00 - q11 - q22 + q33;
  r[1] = 2 * (q12 - q03); r[2] = 2 * (q13 + q02); r[3] = 2 * (q12 + q03);
  r[5] = 2 * (q23 - q01); r[6] = 2 * (q13 - q02); r[7] = 2 * (q23 + q01);
}
void mv(double* r, const double* m, const double* v) {
  double t[3] = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                 m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}
void cross(double* r, const double* a, const double* b) {
  double t[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
  r[0] = t[0]; r[1] = t[1]; r[2] = t[2];
}

}  // namespace

void set_const(HostModel& m) {
  const int nb = m.nbody, nv = m.nv;
  std::vector<double> xpos(3 * nb, 0), xquat(4 * nb, 0), xmat(9 * nb, 0), xipos(3 * nb, 0), ximat(9 * nb, 0);
  std::vector<double> xanchor(3 * m.njnt), xaxis(3 * m.njnt);
  xquat[0] = 1;
  quat2mat(&xmat[0], &xquat[0]);
  quat2mat(&ximat[0], &xquat[0]);
  for (int b = 1; b < nb; b++) {
    int p = m.body_parentid[b];
    double R[9], t[3];
    quat2mat(R, &xquat[4 * p]);
    mv(t, R, &m.body_pos[3 * b]);
    for (int k = 0; k < 3; k++) xpos[3 * b + k] = xpos[3 * p + k] + t[k];
    quat_mul(&xquat[4 * b], &xquat[4 * p], &m.body_quat[4 * b]);
    for (int j = m.body_jntadr[b]; j >= 0 && j < m.body_jntadr[b] + m.body_jntnum[b]; j++) {
      if (m.jnt_type[j] == 0) {  // free: pose from qpos0
        for (int k = 0; k < 3; k++) xpos[3 * b + k] = m.qpos0[m.jnt_qposadr[j] + k];
        for (int k = 0; k < 4; k++) xquat[4 * b + k] = m.qpos0[m.jnt_qposadr[j] + 3 + k];
      }
      double Rb[9];
      quat2mat(Rb, &xquat[4 * b]);
      mv(t, Rb, &m.jnt_pos[3 * j]);
      for (int k = 0; k < 3; k++) xanchor[3 * j + k] = xpos[3 * b + k] + t[k];
      mv(&xaxis[3 * j], Rb, &m.jnt_axis[3 * j]);
    }
    quat2mat(&xmat[9 * b], &xquat[4 * b]);
    mv(t, &xmat[9 * b], &m.body_ipos[3 * b]);
    for (int k = 0; k < 3; k++) xipos[3 * b + k] = xpos[3 * b + k] + t[k];
    double qi[4];
    quat_mul(qi, &xquat[4 * b], &m.body_iquat[4 * b]);
    quat2mat(&ximat[9 * b], qi);
  }
  // subtree mass / com
  m.body_subtreemass.assign(nb, 0);
  std::vector<double> scom(3 * nb, 0);
  for (int b = 0; b < nb; b++) {
    m.body_subtreemass[b] = m.body_mass[b];
    for (int k = 0; k < 3; k++) scom[3 * b + k] = m.body_mass[b] * xipos[3 * b + k];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m.body_parentid[b];
    m.body_subtreemass[p] += m.body_subtreemass[b];
    for (int k = 0; k < 3; k++) scom[3 * p + k] += scom[3 * b + k];
  }
  for (int b = 0; b < nb; b++)
    for (int k = 0; k < 3; k++)
      scom[3 * b + k] = m.body_subtreemass[b] > 1e-15 ? scom[3 * b + k] / m.body_subtreemass[b] : xipos[3 * b + k];
  // cdof (6 per dof: [ang, lin] at the root's subtree com)
  std::vector<double> cdof(6 * nv, 0);
  for (int j = 0; j < m.njnt; j++) {
    int b = m.jnt_bodyid[j], da = m.jnt_dofadr[j];
    const double* rc = &scom[3 * m.body_rootid[b]];
    double off[3] = {rc[0] - xanchor[3 * j], rc[1] - xanchor[3 * j + 1], rc[2] - xanchor[3 * j + 2]};
    auto rot_dof = [&](double* out, const double* ax) {
      for (int k = 0; k < 3; k++) out[k] = ax[k];
      cross(out + 3, ax, off);
    };
    switch (m.jnt_type[j]) {
      case 0:
        for (int i = 0; i < 3; i++) cdof[6 * (da + i) + 3 + i] = 1;
        for (int i = 0; i < 3; i++) {
          double ax[3] = {xmat[9 * b + i], xmat[9 * b + 3 + i], xmat[9 * b + 6 + i]};
          rot_dof(&cdof[6 * (da + 3 + i)], ax);
        }
        break;
      case 1:
        for (int i = 0; i < 3; i++) {
          double ax[3] = {xmat[9 * b + i], xmat[9 * b + 3 + i], xmat[9 * b + 6 + i]};
          rot_dof(&cdof[6 * (da + i)], ax);
        }
        break;
      case 2:
        for (int k = 0; k < 3; k++) cdof[6 * da + 3 + k] = xaxis[3 * j + k];
        break;
      default:
        rot_dof(&cdof[6 * da], &xaxis[3 * j]);
    }
  }
  // body spatial inertia at root com -> composite -> M = sum over ancestors
  std::vector<double> crb(10 * nb, 0);
  for (int b = 1; b < nb; b++) {
    const double* R = &ximat[9 * b];
    const double* I = &m.body_inertia[3 * b];
    double mass = m.body_mass[b];
    const double* rc = &scom[3 * m.body_rootid[b]];
    double d[3] = {xipos[3 * b] - rc[0], xipos[3 * b + 1] - rc[1], xipos[3 * b + 2] - rc[2]};
    double Iw[9];
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += R[3 * r + k] * I[k] * R[3 * c + k];
        Iw[3 * r + c] = s;
      }
    double* ci = &crb[10 * b];
    ci[0] = Iw[0] + mass * (d[1] * d[1] + d[2] * d[2]);
    ci[1] = Iw[4] + mass * (d[0] * d[0] + d[2] * d[2]);
    ci[2] = Iw[8] + mass * (d[0] * d[0] + d[1] * d[1]);
    ci[3] = Iw[1] - mass * d[0] * d[1];
    ci[4] = Iw[2] - mass * d[0] * d[2];
    ci[5] = Iw[5] - mass * d[1] * d[2];
    ci[6] = mass * d[0]; ci[7] = mass * d[1]; ci[8] = mass * d[2]; ci[9] = mass;
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = m.body_parentid[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) crb[10 * p + k] += crb[10 * b + k];
  }
  auto inert_vec = [](double* r, const double* i, const double* v) {
    r[0] = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
    r[1] = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
    r[2] = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
    r[3] = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
    r[4] = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
    r[5] = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
  };
  std::vector<double> M(nv * nv, 0);
  for (int i = 0; i < nv; i++) {
    double buf[6];
    inert_vec(buf, &crb[10 * m.dof_bodyid[i]], &cdof[6 * i]);
    for (int j = i; j >= 0; j = m.dof_parentid[j]) {
      double s = 0;
      for (int k = 0; k < 6; k++) s += cdof[6 * j + k] * buf[k];
      M[i * nv + j] += s;
      M[j * nv + i] = M[i * nv + j];
    }
    M[i * nv + i] += m.dof_armature[i];
  }
  // dense inverse via Cholesky
  std::vector<double> L(M), Minv(nv * nv, 0);
  for (int j = 0; j < nv; j++) {
    double s = L[j * nv + j];
    for (int k = 0; k < j; k++) s -= L[j * nv + k] * L[j * nv + k];
    L[j * nv + j] = std::sqrt(s > 1e-15 ? s : 1e-15);
    for (int i = j + 1; i < nv; i++) {
      double t = L[i * nv + j];
      for (int k = 0; k < j; k++) t -= L[i * nv + k] * L[j * nv + k];
      L[i * nv + j] = t / L[j * nv + j];
    }
  }
  for (int c = 0; c < nv; c++) {
    std::vector<double> x(nv, 0);
    x[c] = 1;
    for (int i = 0; i < nv; i++) {
      for (int k = 0; k < i; k++) x[i] -= L[i * nv + k] * x[k];
      x[i] /= L[i * nv + i];
    }
    for (int i = nv - 1; i >= 0; i--) {
      for (int k = i + 1; k < nv; k++) x[i] -= L[k * nv + i] * x[k];
      x[i] /= L[i * nv + i];
    }
    for (int r = 0; r < nv; r++) Minv[r * nv + c] = x[r];
  }
  m.dof_invweight0.assign(nv, 0);
  for (int i = 0; i < nv; i++) m.dof_invweight0[i] = Minv[i * nv + i];
  double tr = 0;
  for (int i = 0; i < nv; i++) tr += M[i * nv + i];
  m.stat_meaninertia = nv ? tr / nv : 1;
  // body invweight0: mean diagonal of J Minv J' (translation / rotation) at xipos
  m.body_invweight0.assign(2 * nb, 0);
  for (int b = 1; b < nb; b++) {
    int bb = b;
    while (bb && !m.body_dofnum[bb]) bb = m.body_parentid[bb];
    if (!bb) continue;
    std::vector<double> J(6 * nv, 0);
    const double* rc = &scom[3 * m.body_rootid[b]];
    double off[3] = {xipos[3 * b] - rc[0], xipos[3 * b + 1] - rc[1], xipos[3 * b + 2] - rc[2]};
    for (int i = m.body_dofadr[bb] + m.body_dofnum[bb] - 1; i >= 0; i = m.dof_parentid[i]) {
      double t[3];
      cross(t, &cdof[6 * i], off);
      for (int k = 0; k < 3; k++) {
        J[k * nv + i] = cdof[6 * i + 3 + k] + t[k];
        J[(3 + k) * nv + i] = cdof[6 * i + k];
      }
    }
    double diag[6];
    for (int r = 0; r < 6; r++) {
      double s = 0;
      for (int a = 0; a < nv; a++)
        for (int c = 0; c < nv; c++) s += J[r * nv + a] * Minv[a * nv + c] * J[r * nv + c];
      diag[r] = s;
    }
    double tran = (diag[0] + diag[1] + diag[2]) / 3, rot = (diag[3] + diag[4] + diag[5]) / 3;
    if (tran < 1e-15 && rot > 1e-15) tran = rot;
    if (rot < 1e-15) rot = tran;
    m.body_invweight0[2 * b] = tran;
    m.body_invweight0[2 * b + 1] = rot;
  }
}

}  // namespace ilqg
