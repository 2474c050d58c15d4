/*
 * ORACLE / TEST INFRASTRUCTURE ONLY -- the checker, never the product.
 *
 * Plain-C restatement of the reference's iLQR hot path:
 *   ora_calcMJDerivatives  <- /root/reference/src/mjderivative.cpp:43-255 (worker + calcMJDerivatives)
 *   ora_cpMjData           <- /root/reference/src/util.cpp:4-14
 *   A/B assembly           <- /root/reference/inc/differentiator.h:52-93 (incl. quirk Q1)
 *   ora_ilqr_*             <- /root/reference/inc/ilqr.h:69-186 (ctor, initV, setDInit,
 *                             forwardPass, backwardPass, iterate; quirks Q10-Q24)
 *   ora_cost_pendulum      <- /root/reference/inc/inverted_pendulum/cost.h:7-17
 *
 * Pinning: ora_calcMJDerivatives is checked bit-for-bit against the
 * reference's own calcMJDerivatives compiled from /root/reference/src by
 * oracle/Makefile (oracle/_ref/libilqg_ref.so), tests/test_oracle_ref.py.
 * ilqr.h needs Eigen (absent), so the Riccati/rollout restatement follows
 * ilqr.h as written, with a fixed, documented summation order (Eigen's
 * vectorised product order is not reproducible without Eigen): parity of this
 * part against Eigen itself is unpinned; the GPU reproduces this file.
 * Documented deviations: K/k zero-initialised (Q12, UB in the reference);
 * one Differentiator per instance (Q19); nthread capped at MAXTHREAD=16 (Q7).
 */
#include "ilqr_ora.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* FD knobs, mjderivative.cpp:32-39 */
#define ORA_MAXTHREAD 16
static int g_nthread_override = 0;
static const int ora_niter = 30;
static const int ora_nwarmup = 3;
static double ora_eps = 1e-6; /* mjderivative.cpp:39; ora_set_fd_eps for the fp32-FD tolerance tests */
void ora_set_fd_eps(double eps) { ora_eps = eps; }

void ora_set_nthread(int n) { g_nthread_override = n; }

int ora_get_nthread(void) {
  int n = 1;
#ifdef _OPENMP
  n = omp_get_num_procs();
#endif
  if (g_nthread_override > 0) n = g_nthread_override;
  if (n > ORA_MAXTHREAD) n = ORA_MAXTHREAD;
  if (n < 1) n = 1;
  return n;
}

/* util.cpp:4-14 */
void ora_cpMjData(const mjModel* m, mjData* dst, const mjData* src) {
  dst->time = src->time;
  mju_copy(dst->qpos, src->qpos, m->nq);
  mju_copy(dst->qvel, src->qvel, m->nv);
  mju_copy(dst->qacc, src->qacc, m->nv);
  mju_copy(dst->qacc_warmstart, src->qacc_warmstart, m->nv);
  mju_copy(dst->qfrc_applied, src->qfrc_applied, m->nv);
  mju_copy(dst->xfrc_applied, src->xfrc_applied, 6 * m->nbody);
  mju_copy(dst->ctrl, src->ctrl, m->nu);
}

/* ---- costs ---- */
mjtNum ora_cost_pendulum(const mjData* d) {
  /* cost.h:7-17 */
  return 1.0 * d->qpos[0] * d->qpos[0] + 10.0 * d->qpos[1] * d->qpos[1] +
         1.0 * d->qvel[0] * d->qvel[0] + 10.0 * d->qvel[1] * d->qvel[1] +
         1.0 * d->ctrl[0] * d->ctrl[0];
}

static ora_cost_desc g_desc;
void ora_set_cost_desc(const ora_cost_desc* desc) { g_desc = *desc; }

static mjtNum desc_terms(mjtNum c, const mjtNum* x, const mjtNum* w, const mjtNum* t,
                         const mjtNum* l, int n) {
  for (int i = 0; i < n; i++) {
    if (w[i] != 0) {
      mjtNum dx = x[i] - t[i];
      c += w[i] * dx * dx;
    }
    if (l[i] != 0) c += l[i] * x[i];
  }
  return c;
}
mjtNum ora_cost_eval_desc(const ora_cost_desc* c, const mjtNum* qpos, const mjtNum* qvel, const mjtNum* ctrl) {
  mjtNum s = 0;
  s = desc_terms(s, qpos, c->wq, c->tq, c->lq, c->nq);
  s = desc_terms(s, qvel, c->wv, c->tv, c->lv, c->nv);
  s = desc_terms(s, ctrl, c->wu, c->tu, c->lu, c->nu);
  return s;
}
mjtNum ora_cost_desc_fn(const mjData* d) { return ora_cost_eval_desc(&g_desc, d->qpos, d->qvel, d->ctrl); }

/* ---- FD worker, mjderivative.cpp:43-209 ---- */
static void ora_worker(const mjModel* m, const mjData* dmain, mjData* d, int id, int nthread,
                       mjtNum* deriv, stepCostFn_t cost) {
  int nv = m->nv, nu = m->nu;
  int chunk = (nv + nthread - 1) / nthread;
  int istart = id * chunk;
  int iend = istart + chunk < nv ? istart + chunk : nv;
  mjtNum costCenter, *output;
  mjMARKSTACK
  mjtNum* temp = mj_stackAlloc(d, nv);
  mjtNum* warmstart = mj_stackAlloc(d, nv);

  ora_cpMjData(m, d, dmain);
  mj_forward(m, d);
  for (int rep = 1; rep < ora_nwarmup; rep++) mj_forwardSkip(m, d, mjSTAGE_VEL, 1);
  output = d->qacc;
  costCenter = cost(dmain);
  mju_copy(warmstart, d->qacc_warmstart, nv);

  /* ctrl columns: skip = VEL */
  for (int i = istart; i < iend; i++) {
    if (i >= nu) break;
    d->ctrl[i] = dmain->ctrl[i] + ora_eps;
    deriv[2 * nv * nv + nv * nu + 2 * nv + i] = (cost(d) - costCenter) / ora_eps;
    mju_copy(d->qacc_warmstart, warmstart, nv);
    mj_forwardSkip(m, d, mjSTAGE_VEL, 1);
    mju_copy(temp, output, nv);
    ora_cpMjData(m, d, dmain);
    d->ctrl[i] = dmain->ctrl[i] - ora_eps;
    mju_copy(d->qacc_warmstart, warmstart, nv);
    mj_forwardSkip(m, d, mjSTAGE_VEL, 1);
    for (int j = 0; j < nv; j++) deriv[2 * nv * nv + i + j * nu] = (temp[j] - output[j]) / (2 * ora_eps);
    ora_cpMjData(m, d, dmain);
  }
  /* qvel columns: skip = POS */
  for (int i = istart; i < iend; i++) {
    d->qvel[i] = dmain->qvel[i] + ora_eps;
    deriv[2 * nv * nv + nv * nu + nv + i] = (cost(d) - costCenter) / ora_eps;
    mju_copy(d->qacc_warmstart, warmstart, nv);
    mj_forwardSkip(m, d, mjSTAGE_POS, 1);
    mju_copy(temp, output, nv);
    d->qvel[i] = dmain->qvel[i] - ora_eps;
    mju_copy(d->qacc_warmstart, warmstart, nv);
    mj_forwardSkip(m, d, mjSTAGE_POS, 1);
    for (int j = 0; j < nv; j++) deriv[nv * nv + i + j * nv] = (temp[j] - output[j]) / (2 * ora_eps);
    ora_cpMjData(m, d, dmain);
  }
  /* qpos columns: skip = NONE, quaternion-aware */
  for (int i = istart; i < iend; i++) {
    int jid = m->dof_jntid[i];
    int quatadr = -1, dofpos = 0;
    if (m->jnt_type[jid] == mjJNT_BALL) {
      quatadr = m->jnt_qposadr[jid];
      dofpos = i - m->jnt_dofadr[jid];
    } else if (m->jnt_type[jid] == mjJNT_FREE && i >= m->jnt_dofadr[jid] + 3) {
      quatadr = m->jnt_qposadr[jid] + 3;
      dofpos = i - m->jnt_dofadr[jid] - 3;
    }
    if (quatadr >= 0) {
      mjtNum angvel[3] = {0, 0, 0};
      angvel[dofpos] = ora_eps;
      mju_quatIntegrate(d->qpos + quatadr, angvel, 1);
    } else {
      d->qpos[m->jnt_qposadr[jid] + i - m->jnt_dofadr[jid]] += ora_eps;
    }
    deriv[2 * nv * nv + nv * nu + i] = (cost(d) - costCenter) / ora_eps;
    mju_copy(d->qacc_warmstart, warmstart, nv);
    mj_forwardSkip(m, d, mjSTAGE_NONE, 1);
    mju_copy(temp, output, nv);
    mju_copy(d->qpos, dmain->qpos, m->nq);
    if (quatadr >= 0) {
      mjtNum angvel[3] = {0, 0, 0};
      angvel[dofpos] = -ora_eps;
      mju_quatIntegrate(d->qpos + quatadr, angvel, 1);
    } else {
      d->qpos[m->jnt_qposadr[jid] + i - m->jnt_dofadr[jid]] -= ora_eps;
    }
    mju_copy(d->qacc_warmstart, warmstart, nv);
    mj_forwardSkip(m, d, mjSTAGE_NONE, 1);
    for (int j = 0; j < nv; j++) deriv[i + j * nv] = (temp[j] - output[j]) / (2 * ora_eps);
    ora_cpMjData(m, d, dmain);
  }
  mjFREESTACK
}

/* mjderivative.cpp:212-255: per-call per-thread mjData, FD solver options
   written into the (shared) model and restored afterwards */
void ora_calcMJDerivatives(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t cost) {
  int nthread = ora_get_nthread();
  mjData* d[ORA_MAXTHREAD];
  int save_iterations = m->opt.iterations;
  mjtNum save_tolerance = m->opt.tolerance;
  for (int n = 0; n < nthread; n++) d[n] = mj_makeData(m);
  m->opt.iterations = ora_niter;
  m->opt.tolerance = 0;
#pragma omp parallel for schedule(static) num_threads(nthread)
  for (int n = 0; n < nthread; n++) ora_worker(m, dmain, d[n], n, nthread, deriv, cost);
  for (int n = 0; n < nthread; n++) mj_deleteData(d[n]);
  m->opt.iterations = save_iterations;
  m->opt.tolerance = save_tolerance;
}

/* "Tuned CPU" variant (reported for honesty, never the
   reference number): persistent per-thread mjData, one centre per point,
   columns spread over threads.  Same arithmetic per column, so bit-identical
   output. */
void ora_calcMJDerivatives_tuned(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t cost,
                                 mjData** pool, int npool) {
  int save_iterations = m->opt.iterations;
  mjtNum save_tolerance = m->opt.tolerance;
  int nv = m->nv;
  m->opt.iterations = ora_niter;
  m->opt.tolerance = 0;
  {
    int nt = npool < nv ? npool : nv;
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int n = 0; n < nt; n++) ora_worker(m, dmain, pool[n], n, nt, deriv, cost);
  }
  m->opt.iterations = save_iterations;
  m->opt.tolerance = save_tolerance;
}

/* ---- A/B assembly, differentiator.h:66-71,89-92 (col-major, quirk Q1) ----
   Layout 0 (reference): the lower blocks are Eigen column-major maps of the
   row-major deriv blocks (differentiator.h:57-59): A lower = dt J^T, B lower a
   permutation of dt J_u when nu > 1.  Layout 1 (corrected, SURVEY.md Appendix A
   Q1's optional mode): the true Jacobians, entry (r, c) of J_q at
   deriv[c + r nv] (mjderivative.cpp:202), of J_u at deriv[2nv^2 + c + r nu]
   (:107). */
static int ora_layout = 0;
void ora_set_layout(int layout) { ora_layout = layout; }
int ora_get_layout(void) { return ora_layout; }

void ora_assemble_AB(int nv, int nu, mjtNum dt, const mjtNum* deriv, mjtNum* A, mjtNum* B) {
  int nx = 2 * nv, L = ora_layout;
  for (int c = 0; c < nx; c++)
    for (int r = 0; r < nx; r++) {
      mjtNum val;
      int rr = r - nv, cc = c < nv ? c : c - nv;
      if (r < nv && c < nv) val = (r == c) ? 1 : 0;
      else if (r < nv) val = (r == c - nv) ? dt : 0;
      else if (c < nv) val = deriv[L ? cc + rr * nv : rr + cc * nv] * dt;
      else val = (rr == cc ? 1 : 0) + deriv[nv * nv + (L ? cc + rr * nv : rr + cc * nv)] * dt;
      A[r + c * nx] = val;
    }
  for (int c = 0; c < nu; c++)
    for (int r = 0; r < nx; r++)
      B[r + c * nx] = (r < nv) ? 0 : deriv[2 * nv * nv + (L ? c + (r - nv) * nu : (r - nv) + c * nv)] * dt;
}

/* ---- Eigen-style pivoted LDLT (Eigen/src/Cholesky/LDLT.h, lower) ---- */
int ora_ldlt_factor(int n, mjtNum* mat, int* transp) {
  mjtNum temp[64];
  for (int k = 0; k < n; k++) {
    int big = k;
    mjtNum bigv = fabs(mat[k + k * n]);
    int rs = n - k - 1;
    for (int i = k + 1; i < n; i++)
      if (fabs(mat[i + i * n]) > bigv) { bigv = fabs(mat[i + i * n]); big = i; }
    transp[k] = big;
    if (k != big) {
      int s = n - big - 1;
      mjtNum t;
      for (int j = 0; j < k; j++) { t = mat[k + j * n]; mat[k + j * n] = mat[big + j * n]; mat[big + j * n] = t; }
      for (int i = 0; i < s; i++) {
        t = mat[(big + 1 + i) + k * n]; mat[(big + 1 + i) + k * n] = mat[(big + 1 + i) + big * n];
        mat[(big + 1 + i) + big * n] = t;
      }
      t = mat[k + k * n]; mat[k + k * n] = mat[big + big * n]; mat[big + big * n] = t;
      for (int i = k + 1; i < big; i++) {
        t = mat[i + k * n]; mat[i + k * n] = mat[big + i * n]; mat[big + i * n] = t;
      }
    }
    if (k > 0) {
      mjtNum s = 0;
      for (int j = 0; j < k; j++) temp[j] = mat[j + j * n] * mat[k + j * n];
      for (int j = 0; j < k; j++) s += mat[k + j * n] * temp[j];
      mat[k + k * n] -= s;
      for (int i = k + 1; i < n; i++) {
        mjtNum si = 0;
        for (int j = 0; j < k; j++) si += mat[i + j * n] * temp[j];
        mat[i + k * n] -= si;
      }
    }
    if (k == 0 && !(fabs(mat[0]) > 0)) {
      for (int j = 0; j < n; j++) transp[j] = j;
      return 0;
    }
    if (rs > 0 && fabs(mat[k + k * n]) > 0)
      for (int i = k + 1; i < n; i++) mat[i + k * n] /= mat[k + k * n];
  }
  return 1;
}
void ora_ldlt_solve(int n, const mjtNum* L, const int* transp, mjtNum* x) {
  const mjtNum tol = 2.2250738585072014e-308; /* numeric_limits<double>::min() */
  for (int k = 0; k < n; k++) {
    mjtNum t = x[k]; x[k] = x[transp[k]]; x[transp[k]] = t;
  }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < i; j++) x[i] -= L[i + j * n] * x[j];
  for (int i = 0; i < n; i++) {
    if (fabs(L[i + i * n]) > tol) x[i] /= L[i + i * n];
    else x[i] = 0;
  }
  for (int i = n - 1; i >= 0; i--)
    for (int j = i + 1; j < n; j++) x[i] -= L[j + i * n] * x[j];
  for (int k = n - 1; k >= 0; k--) {
    mjtNum t = x[k]; x[k] = x[transp[k]]; x[transp[k]] = t;
  }
}

/* ---- one Riccati step, ilqr.h:150-174 (quirks Q13-Q18), fixed order ----
   In: V (nx*nx col-major, updated in place), v (nx), deriv (D), xprev/xcur
   (x*_{n-1}, x*_n, 2nv each), dt, mu.  Out: K (nu*nx col-major), k (nu). */
/* x_a (-) x_b in the tangent space (2nv entries).  Equal, operation for
   operation, to the reference's x_a - x_b on [qpos; qvel] when the model has
   no ball/free joints (nq == nv, inc/ilqr.h:90).  Quaternion blocks (an
   extension: the reference does not support them, quirk Q21) use the
   first-order log map 2 sign(w) v of qdif = conj(q_b) q_a, with no
   transcendental function so host and device agree bit for bit. */
static void ora_quat_diff(mjtNum* d, const mjtNum* qa, const mjtNum* qb) {
  mjtNum c[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, q[4];
  q[0] = c[0] * qa[0] - c[1] * qa[1] - c[2] * qa[2] - c[3] * qa[3];
  q[1] = c[0] * qa[1] + c[1] * qa[0] + c[2] * qa[3] - c[3] * qa[2];
  q[2] = c[0] * qa[2] - c[1] * qa[3] + c[2] * qa[0] + c[3] * qa[1];
  q[3] = c[0] * qa[3] + c[1] * qa[2] - c[2] * qa[1] + c[3] * qa[0];
  mjtNum s = q[0] < 0 ? -2.0 : 2.0;
  d[0] = s * q[1];
  d[1] = s * q[2];
  d[2] = s * q[3];
}
void ora_state_diff(const mjModel* m, const mjtNum* qa, const mjtNum* va, const mjtNum* qb, const mjtNum* vb,
                    mjtNum* dx) {
  int nv = m->nv;
  for (int j = 0; j < m->njnt; j++) {
    int qadr = m->jnt_qposadr[j], dadr = m->jnt_dofadr[j], t = m->jnt_type[j];
    if (t == mjJNT_FREE) {
      for (int k = 0; k < 3; k++) dx[dadr + k] = qa[qadr + k] - qb[qadr + k];
      ora_quat_diff(dx + dadr + 3, qa + qadr + 3, qb + qadr + 3);
    } else if (t == mjJNT_BALL) {
      ora_quat_diff(dx + dadr, qa + qadr, qb + qadr);
    } else {
      dx[dadr] = qa[qadr] - qb[qadr];
    }
  }
  for (int i = 0; i < nv; i++) dx[nv + i] = va[i] - vb[i];
}

void ora_riccati_step(int nv, int nu, mjtNum dt, mjtNum mu, const mjtNum* deriv,
                      const mjtNum* xprev, const mjtNum* xcur, mjtNum* V, mjtNum* v,
                      mjtNum* K, mjtNum* kff) {
  mjtNum c[256];
  for (int i = 0; i < 2 * nv; i++) c[i] = xprev[i] - xcur[i];
  ora_riccati_step_c(nv, nu, dt, mu, deriv, c, V, v, K, kff);
}

/* the step with c = x*_{n-1} (-) x*_n supplied */
void ora_riccati_step_c(int nv, int nu, mjtNum dt, mjtNum mu, const mjtNum* deriv, const mjtNum* cin,
                        mjtNum* V, mjtNum* v, mjtNum* K, mjtNum* kff) {
  int nx = 2 * nv;
  mjtNum *A = malloc(sizeof(mjtNum) * nx * nx), *B = malloc(sizeof(mjtNum) * nx * nu);
  mjtNum *Vs = malloc(sizeof(mjtNum) * nx * nx), *T1 = malloc(sizeof(mjtNum) * nu * nx);
  mjtNum *T2 = malloc(sizeof(mjtNum) * nu * nu), *T3 = malloc(sizeof(mjtNum) * nu * nx);
  mjtNum *ABK = malloc(sizeof(mjtNum) * nx * nx), *T4 = malloc(sizeof(mjtNum) * nx * nx);
  mjtNum *T6 = malloc(sizeof(mjtNum) * nx * nu), *Vn = malloc(sizeof(mjtNum) * nx * nx);
  mjtNum *c = malloc(sizeof(mjtNum) * nx), *w = malloc(sizeof(mjtNum) * nx);
  mjtNum *y = malloc(sizeof(mjtNum) * nx), *z = malloc(sizeof(mjtNum) * nx);
  mjtNum *vn = malloc(sizeof(mjtNum) * nx), *kR = malloc(sizeof(mjtNum) * nu);
  mjtNum *Mm = malloc(sizeof(mjtNum) * nu * nu), *col = malloc(sizeof(mjtNum) * nu);
  int* tr = malloc(sizeof(int) * nu);
  const mjtNum* q = deriv + 2 * nv * nv + nv * nu;
  const mjtNum* r = q + nx;

  /* V = (V + V')/2 */
  for (int j = 0; j < nx; j++)
    for (int i = 0; i < nx; i++) Vs[i + j * nx] = (V[i + j * nx] + V[j + i * nx]) / 2;
  ora_assemble_AB(nv, nu, dt, deriv, A, B);
  for (int i = 0; i < nx; i++) c[i] = cin[i];
  for (int i = 0; i < nx; i++) Vs[i + i * nx] += mu;
  /* T1 = B'V */
  for (int j = 0; j < nx; j++)
    for (int a = 0; a < nu; a++) {
      mjtNum s = 0;
      for (int kk = 0; kk < nx; kk++) s += B[kk + a * nx] * Vs[kk + j * nx];
      T1[a + j * nu] = s;
    }
  /* T2 = T1 B ; Mm = -2 T2 - 2 R */
  for (int b = 0; b < nu; b++)
    for (int a = 0; a < nu; a++) {
      mjtNum s = 0;
      for (int kk = 0; kk < nx; kk++) s += T1[a + kk * nu] * B[kk + b * nx];
      T2[a + b * nu] = s;
      Mm[a + b * nu] = -2 * s - 2 * (r[a] * r[b]);
    }
  /* T3 = T1 A */
  for (int j = 0; j < nx; j++)
    for (int a = 0; a < nu; a++) {
      mjtNum s = 0;
      for (int kk = 0; kk < nx; kk++) s += T1[a + kk * nu] * A[kk + j * nx];
      T3[a + j * nu] = s;
    }
  ora_ldlt_factor(nu, Mm, tr);
  /* K = ldlt.solve(2 T3), column by column */
  for (int j = 0; j < nx; j++) {
    for (int a = 0; a < nu; a++) col[a] = 2 * T3[a + j * nu];
    ora_ldlt_solve(nu, Mm, tr, col);
    for (int a = 0; a < nu; a++) K[a + j * nu] = col[a];
  }
  /* k = ldlt.solve(B'(v' + 2Vc) + r') */
  for (int i = 0; i < nx; i++) {
    mjtNum s = 0;
    for (int j = 0; j < nx; j++) s += Vs[i + j * nx] * c[j];
    w[i] = v[i] + 2 * s;
  }
  for (int a = 0; a < nu; a++) {
    mjtNum s = 0;
    for (int kk = 0; kk < nx; kk++) s += B[kk + a * nx] * w[kk];
    col[a] = s + r[a];
  }
  ora_ldlt_solve(nu, Mm, tr, col);
  for (int a = 0; a < nu; a++) kff[a] = col[a];
  /* ABK = A + B K */
  for (int j = 0; j < nx; j++)
    for (int i = 0; i < nx; i++) {
      mjtNum s = 0;
      for (int a = 0; a < nu; a++) s += B[i + a * nx] * K[a + j * nu];
      ABK[i + j * nx] = A[i + j * nx] + s;
    }
  /* V_new = ABK' V ABK + Q + K' R K */
  for (int j = 0; j < nx; j++)
    for (int i = 0; i < nx; i++) {
      mjtNum s = 0;
      for (int kk = 0; kk < nx; kk++) s += ABK[kk + i * nx] * Vs[kk + j * nx];
      T4[i + j * nx] = s;
    }
  for (int b = 0; b < nu; b++)
    for (int i = 0; i < nx; i++) {
      mjtNum s = 0;
      for (int a = 0; a < nu; a++) s += K[a + i * nu] * (r[a] * r[b]);
      T6[i + b * nx] = s;
    }
  for (int j = 0; j < nx; j++)
    for (int i = 0; i < nx; i++) {
      mjtNum s5 = 0, s7 = 0;
      for (int kk = 0; kk < nx; kk++) s5 += T4[i + kk * nx] * ABK[kk + j * nx];
      for (int b = 0; b < nu; b++) s7 += T6[i + b * nx] * K[b + j * nu];
      Vn[i + j * nx] = (s5 + q[i] * q[j]) + s7;
    }
  /* v_new = 2(k'B' + c')V_new ABK + v ABK + q + 2 k'R K  (reads the NEW V: Q14) */
  for (int i = 0; i < nx; i++) {
    mjtNum s = 0;
    for (int a = 0; a < nu; a++) s += B[i + a * nx] * kff[a];
    y[i] = s + c[i];
  }
  for (int j = 0; j < nx; j++) {
    mjtNum s = 0;
    for (int i = 0; i < nx; i++) s += (2 * y[i]) * Vn[i + j * nx];
    z[j] = s;
  }
  for (int b = 0; b < nu; b++) {
    mjtNum s = 0;
    for (int a = 0; a < nu; a++) s += kff[a] * (r[a] * r[b]);
    kR[b] = s;
  }
  for (int j = 0; j < nx; j++) {
    mjtNum ta = 0, tb = 0, td = 0;
    for (int i = 0; i < nx; i++) ta += z[i] * ABK[i + j * nx];
    for (int i = 0; i < nx; i++) tb += v[i] * ABK[i + j * nx];
    for (int b = 0; b < nu; b++) td += (2 * kR[b]) * K[b + j * nu];
    vn[j] = ((ta + tb) + q[j]) + td;
  }
  memcpy(V, Vn, sizeof(mjtNum) * nx * nx);
  memcpy(v, vn, sizeof(mjtNum) * nx);
  free(A); free(B); free(Vs); free(T1); free(T2); free(T3); free(ABK); free(T4); free(T6);
  free(Vn); free(c); free(w); free(y); free(z); free(vn); free(kR); free(Mm); free(col); free(tr);
}

/* ---- ILQR<nv,nu,N>, ilqr.h:69-186 ---- */
ora_ilqr* ora_ilqr_create(mjModel* m, const mjData* dmain, int N, stepCostFn_t cost,
                          ora_calc_fn calc) {
  ora_ilqr* s = (ora_ilqr*)calloc(1, sizeof(ora_ilqr));
  int nv = m->nv, nu = m->nu, nx = 2 * nv;
  s->m = m; s->N = N; s->nv = nv; s->nu = nu; s->nx = nx;
  s->cost = cost;
  s->calc = calc ? calc : ora_calcMJDerivatives;
  s->mu = 1000.0;
  s->D = nv * (2 * nv + nu) + 2 * nv + nu;
  s->deriv = (mjtNum*)calloc((size_t)(N + 1) * s->D, sizeof(mjtNum));
  s->V = (mjtNum*)calloc((size_t)nx * nx, sizeof(mjtNum));
  s->v = (mjtNum*)calloc((size_t)nx, sizeof(mjtNum));
  s->K = (mjtNum*)calloc((size_t)(N + 1) * nu * nx, sizeof(mjtNum)); /* Q12: zero-init */
  s->k = (mjtNum*)calloc((size_t)(N + 1) * nu, sizeof(mjtNum));
  s->dArray = (mjData**)calloc((size_t)(N + 1), sizeof(mjData*));
  s->d = mj_makeData(m);
  ora_cpMjData(m, s->d, dmain);
  for (int n = N; n >= 0; n--) {
    s->dArray[n] = mj_makeData(m);
    ora_cpMjData(m, s->dArray[n], s->d);
    mj_step(m, s->d);
  }
  return s;
}

void ora_ilqr_free(ora_ilqr* s) {
  if (!s) return;
  for (int n = 0; n <= s->N; n++) mj_deleteData(s->dArray[n]);
  mj_deleteData(s->d);
  free(s->dArray); free(s->deriv); free(s->V); free(s->v); free(s->K); free(s->k);
  free(s);
}

void ora_ilqr_setDInit(ora_ilqr* s, const mjData* dinit) { ora_cpMjData(s->m, s->d, dinit); }

void ora_ilqr_forwardPass(ora_ilqr* s) {
  int nx = s->nx, nu = s->nu;
  mjtNum dx[128];
  for (int n = s->N; n >= 0; n--) {
    const mjtNum* xs = s->dArray[n]->qpos;
    const mjtNum* us = s->dArray[n]->ctrl;
    const mjtNum* K = s->K + (size_t)n * nu * nx;
    const mjtNum* k = s->k + (size_t)n * nu;
    ora_state_diff(s->m, s->d->qpos, s->d->qvel, xs, s->dArray[n]->qvel, dx);
    for (int a = 0; a < nu; a++) {
      mjtNum t = 0;
      for (int j = 0; j < nx; j++) t += K[a + j * nu] * dx[j];
      s->d->ctrl[a] = (t + k[a]) + us[a];
    }
    ora_cpMjData(s->m, s->dArray[n], s->d);
    mj_step(s->m, s->d);
  }
}

/* an FD "driver" that leaves the record as it is: backwardPass over records
   formed elsewhere (the point-sharded sweep's gathered records, tests) */
void ora_calc_none(mjModel* m, mjData* d, mjtNum* deriv, stepCostFn_t cost) {
  (void)m; (void)d; (void)deriv; (void)cost;
}

void ora_ilqr_fd_point(ora_ilqr* s, int n) {
  s->calc(s->m, s->dArray[n], s->deriv + (size_t)n * s->D, s->cost);
}

/* the recursion n = 1..N from the V, v already in s (ilqr.h:144-175) */
static void ora_ilqr_recursion(ora_ilqr* s) {
  int nv = s->nv, nu = s->nu, nx = s->nx;
  mjtNum dt = s->m->opt.timestep;
  for (int n = 1; n <= s->N; n++) {
    s->cout_lines += 2; /* ilqr.h:146-147 -> counted null sink */
    ora_ilqr_fd_point(s, n);
    mjtNum c[256];
    ora_state_diff(s->m, s->dArray[n - 1]->qpos, s->dArray[n - 1]->qvel, s->dArray[n]->qpos,
                   s->dArray[n]->qvel, c);
    ora_riccati_step_c(nv, nu, dt, s->mu, s->deriv + (size_t)n * s->D, c, s->V, s->v,
                       s->K + (size_t)n * nu * nx, s->k + (size_t)n * nu);
  }
}

void ora_ilqr_backwardPass(ora_ilqr* s) {
  int nv = s->nv, nu = s->nu, nx = s->nx;
  /* initV, ilqr.h:100-107 */
  ora_ilqr_fd_point(s, 0);
  {
    const mjtNum* q = s->deriv + 2 * nv * nv + nv * nu;
    for (int i = 0; i < nx; i++) s->v[i] = q[i];
    for (int j = 0; j < nx; j++)
      for (int i = 0; i < nx; i++) s->V[i + j * nx] = s->v[i] * s->v[j];
  }
  ora_ilqr_recursion(s);
}

/* backwardPass with an overridden initV (virtual, ilqr.h:100,142): the
   recursion starts from the caller's V0 (nx x nx col-major) and v0 */
void ora_ilqr_backwardPass_v0(ora_ilqr* s, const mjtNum* V0, const mjtNum* v0) {
  int nx = s->nx;
  ora_ilqr_fd_point(s, 0);
  memcpy(s->V, V0, sizeof(mjtNum) * nx * nx);
  memcpy(s->v, v0, sizeof(mjtNum) * nx);
  ora_ilqr_recursion(s);
}

void ora_ilqr_iterate(ora_ilqr* s) {
  ora_ilqr_forwardPass(s);
  ora_ilqr_setDInit(s, s->dArray[s->N]);
  ora_ilqr_backwardPass(s);
}

/* iterate() of an ILQR subclass whose initV override sets V0, v0 */
void ora_ilqr_iterate_v0(ora_ilqr* s, const mjtNum* V0, const mjtNum* v0) {
  ora_ilqr_forwardPass(s);
  ora_ilqr_setDInit(s, s->dArray[s->N]);
  ora_ilqr_backwardPass_v0(s, V0, v0);
}

/* ---- line-search extension (no reference counterpart,
   quirk Q22): forwardPass (ilqr.h:116-130) rolled out once per candidate with
   the feed-forward scaled, u = K (x - x*) + alpha k + u*, each candidate
   recording its own trajectory and its trajectory cost sum_n cost(d_n) over
   the recorded states (terms in n = N..0 order).  alpha = 1 is exactly the
   reference's forwardPass.  select_mode 0 keeps candidate 0 (reference
   semantics), 1 the lowest cost (first minimum; a NaN cost loses to any
   number).  The selected candidate becomes dArray; the caller's setDInit
   (ilqr.h:183) follows. ---- */
void ora_ilqr_forward_candidates(ora_ilqr* s, int A, const mjtNum* alphas, int select_mode, mjtNum* costs,
                                 int* selected) {
  const mjModel* m = s->m;
  int nq = m->nq, nv = m->nv, nu = s->nu, nx = s->nx, N = s->N, P = N + 1;
  /* per candidate and point: time, qpos, qvel, qacc, warm, ctrl */
  int rec = 1 + nq + 3 * nv + nu;
  mjtNum* tr = (mjtNum*)malloc(sizeof(mjtNum) * (size_t)A * P * rec);
  mjData* d = mj_makeData(s->m);
  mjtNum dx[256];
  for (int a = 0; a < A; a++) {
    mjtNum alpha = alphas ? alphas[a] : 1.0, c = 0;
    ora_cpMjData(m, d, s->d);
    for (int n = N; n >= 0; n--) {
      const mjtNum* xs = s->dArray[n]->qpos;
      const mjtNum* us = s->dArray[n]->ctrl;
      const mjtNum* K = s->K + (size_t)n * nu * nx;
      const mjtNum* k = s->k + (size_t)n * nu;
      ora_state_diff(m, d->qpos, d->qvel, xs, s->dArray[n]->qvel, dx);
      for (int i = 0; i < nu; i++) {
        mjtNum t = 0;
        for (int j = 0; j < nx; j++) t += K[i + j * nu] * dx[j];
        d->ctrl[i] = (t + alpha * k[i]) + us[i];
      }
      mjtNum* r = tr + ((size_t)a * P + n) * rec;
      r[0] = d->time;
      mju_copy(r + 1, d->qpos, nq);
      mju_copy(r + 1 + nq, d->qvel, nv);
      mju_copy(r + 1 + nq + nv, d->qacc, nv);
      mju_copy(r + 1 + nq + 2 * nv, d->qacc_warmstart, nv);
      mju_copy(r + 1 + nq + 3 * nv, d->ctrl, nu);
      c += s->cost(d);
      mj_step(s->m, d);
    }
    if (costs) costs[a] = c;
  }
  int best = 0;
  if (select_mode == 1 && costs) {
    mjtNum bc = costs[0];
    for (int a = 1; a < A; a++)
      if (costs[a] < bc || (bc != bc && costs[a] == costs[a])) { bc = costs[a]; best = a; }
  }
  if (selected) *selected = best;
  /* the selected candidate's records become dArray (cpMjData's fields) and
     the rollout's end state becomes d, as after the reference forwardPass */
  for (int n = N; n >= 0; n--) {
    mjData* dn = s->dArray[n];
    const mjtNum* r = tr + ((size_t)best * P + n) * rec;
    dn->time = r[0];
    mju_copy(dn->qpos, r + 1, nq);
    mju_copy(dn->qvel, r + 1 + nq, nv);
    mju_copy(dn->qacc, r + 1 + nq + nv, nv);
    mju_copy(dn->qacc_warmstart, r + 1 + nq + 2 * nv, nv);
    mju_copy(dn->ctrl, r + 1 + nq + 3 * nv, nu);
    mju_copy(dn->qfrc_applied, s->d->qfrc_applied, nv);
    mju_copy(dn->xfrc_applied, s->d->xfrc_applied, 6 * m->nbody);
  }
  mj_deleteData(d);
  free(tr);
}

/* iterate() with the line search: candidates, selection, setDInit(dArray[N]), backwardPass */
void ora_ilqr_iterate_ls(ora_ilqr* s, int A, const mjtNum* alphas, int select_mode, mjtNum* costs, int* selected) {
  ora_ilqr_forward_candidates(s, A, alphas, select_mode, costs, selected);
  ora_ilqr_setDInit(s, s->dArray[s->N]);
  ora_ilqr_backwardPass(s);
}

/* a rollout with fixed gains: forwardPass alone */
void ora_ilqr_set_gains(ora_ilqr* s, const mjtNum* K, const mjtNum* k) {
  if (K) memcpy(s->K, K, sizeof(mjtNum) * (size_t)(s->N + 1) * s->nu * s->nx);
  if (k) memcpy(s->k, k, sizeof(mjtNum) * (size_t)(s->N + 1) * s->nu);
}

/* trajectory export: per point time, qpos, qvel, qacc_warmstart, ctrl */
void ora_ilqr_get_traj(const ora_ilqr* s, mjtNum* time, mjtNum* qpos, mjtNum* qvel, mjtNum* warm,
                       mjtNum* ctrl) {
  const mjModel* m = s->m;
  for (int n = 0; n <= s->N; n++) {
    const mjData* d = s->dArray[n];
    if (time) time[n] = d->time;
    if (qpos) mju_copy(qpos + (size_t)n * m->nq, d->qpos, m->nq);
    if (qvel) mju_copy(qvel + (size_t)n * m->nv, d->qvel, m->nv);
    if (warm) mju_copy(warm + (size_t)n * m->nv, d->qacc_warmstart, m->nv);
    if (ctrl) mju_copy(ctrl + (size_t)n * m->nu, d->ctrl, m->nu);
  }
}
