// Hot-path kernels for gfx950.
//
//  k_fd_centre   src/mjderivative.cpp:61-75   centre forward + 2 warm-up solves per point
//  k_fd_cols     src/mjderivative.cpp:78-206  one lane per derivative column (+/- sides)
//  k_rollout     inc/ilqr.h:116-130 (+ ctor rollout inc/ilqr.h:82-87), one lane per (seed, alpha)
//  k_select      inc/ilqr.h:183 setDInit(dArray[N]) + line-search candidate selection
//  k_backward    inc/ilqr.h:100-107,133-176, one workgroup per seed, LDS-resident V/A/B
//  k_step/k_fwd  mj_step / mj_forward on independent states (legacy boundary)
//
// Evaluation lanes are independent; the per-lane workspace is SoA across
// lanes (see dmodel.h) so every field access of a wave is one coalesced
// 512-byte transaction.
#include "dphys.h"
#include "kernels.h"

namespace ilqg {
namespace {

using dev::Lane;
using dev::SPd;

constexpr double FD_EPS = 1e-6;  // mjderivative.cpp:39
constexpr int FD_NITER = 30;     // mjderivative.cpp:37
constexpr int FD_NWARMUP = 3;    // mjderivative.cpp:38
constexpr int LANE_BLOCK = 64;   // one wave per workgroup: spreads lanes over all CUs

__device__ inline double cost_terms(double c, SPd x, const double* w, const double* t, const double* l, int n) {
  for (int i = 0; i < n; i++) {
    double xi = x[i];
    if (w[i] != 0) {
      double dx = xi - t[i];
      c += w[i] * dx * dx;
    }
    if (l[i] != 0) c += l[i] * xi;
  }
  return c;
}
__device__ inline double cost_terms_g(double c, const double* x, const double* w, const double* t, const double* l,
                                      int n) {
  for (int i = 0; i < n; i++) {
    double xi = x[i];
    if (w[i] != 0) {
      double dx = xi - t[i];
      c += w[i] * dx * dx;
    }
    if (l[i] != 0) c += l[i] * xi;
  }
  return c;
}
__device__ inline double step_cost_ws(const DevModel& m, const CostDev& c, SPd qpos, SPd qvel, SPd ctrl) {
  double s = 0;
  s = cost_terms(s, qpos, c.wq, c.tq, c.lq, m.nq);
  s = cost_terms(s, qvel, c.wv, c.tv, c.lv, m.nv);
  s = cost_terms(s, ctrl, c.wu, c.tu, c.lu, m.nu);
  return s;
}

// cpMjData(d, dmain) (src/util.cpp:4-14) from the trajectory record of `pt`
__device__ inline void load_state(const DevModel& m, const WsLayout& L, const Lane& ln, const TrajDev& tr, int pt,
                                  int seed, const double* qfrc_applied, const double* xfrc_applied) {
  SPd qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), ctrl = ln.D(L.ctrl), warm = ln.D(L.warm);
  SPd qap = ln.D(L.qfrc_applied), xf = ln.D(L.xfrc_applied);
  for (int i = 0; i < m.nq; i++) qpos[i] = tr.qpos[(size_t)pt * m.nq + i];
  for (int i = 0; i < m.nv; i++) qvel[i] = tr.qvel[(size_t)pt * m.nv + i];
  for (int i = 0; i < m.nv; i++) warm[i] = tr.warm[(size_t)pt * m.nv + i];
  for (int i = 0; i < m.nu; i++) ctrl[i] = tr.ctrl[(size_t)pt * m.nu + i];
  for (int i = 0; i < m.nv; i++) qap[i] = qfrc_applied ? qfrc_applied[(size_t)seed * m.nv + i] : 0.0;
  for (int i = 0; i < 6 * m.nbody; i++) xf[i] = xfrc_applied ? xfrc_applied[(size_t)seed * 6 * m.nbody + i] : 0.0;
  ln.D(L.time)[0] = tr.time[pt];
}

__global__ __launch_bounds__(LANE_BLOCK) void k_fd_centre(DevModel m, WsLayout L, WsDev ws, TrajDev tr, int npts,
                                                          int P, const double* qfrc_applied,
                                                          const double* xfrc_applied, CostDev cost, double* warm_c,
                                                          double* cost_c) {
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= npts) return;
  Lane ln{ws.d + lane, ws.i + lane, (size_t)ws.nlanes};
  int seed = lane / P;
  load_state(m, L, ln, tr, lane, seed, qfrc_applied, xfrc_applied);
  dev::forward_skip(m, L, ln, dev::STAGE_NONE, FD_NITER, 0.0);
  for (int rep = 1; rep < FD_NWARMUP; rep++) dev::forward_skip(m, L, ln, dev::STAGE_VEL, FD_NITER, 0.0);
  SPd warm = ln.D(L.warm);
  for (int i = 0; i < m.nv; i++) warm_c[(size_t)lane * m.nv + i] = warm[i];
  double s = 0;
  s = cost_terms_g(s, tr.qpos + (size_t)lane * m.nq, cost.wq, cost.tq, cost.lq, m.nq);
  s = cost_terms_g(s, tr.qvel + (size_t)lane * m.nv, cost.wv, cost.tv, cost.lv, m.nv);
  s = cost_terms_g(s, tr.ctrl + (size_t)lane * m.nu, cost.wu, cost.tu, cost.lu, m.nu);
  cost_c[lane] = s;
}

__global__ __launch_bounds__(LANE_BLOCK) void k_fd_cols(DevModel m, WsLayout L, WsDev ws, TrajDev tr, int npts,
                                                        int P, const double* qfrc_applied, const double* xfrc_applied,
                                                        CostDev cost, const double* warm_c, const double* cost_c,
                                                        double* deriv) {
  const int nv = m.nv, nu = m.nu;
  const int nctrl = nu < nv ? nu : nv;  // mjderivative.cpp:78-82 (assumes nv >= nu)
  const int ncol = nctrl + 2 * nv;
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= npts * ncol) return;
  int pt = lane / ncol, col = lane % ncol, seed = pt / P;
  Lane ln{ws.d + lane, ws.i + lane, (size_t)ws.nlanes};
  const int D = nv * (2 * nv + nu) + 2 * nv + nu;
  double* dr = deriv + (size_t)pt * D;
  const double* wc = warm_c + (size_t)pt * nv;
  const double costCenter = cost_c[pt];
  SPd qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), ctrl = ln.D(L.ctrl), warm = ln.D(L.warm), qacc = ln.D(L.qacc);
  SPd temp = ln.D(L.s_fd);
  const double* dq = tr.qpos + (size_t)pt * m.nq;
  const double* dv = tr.qvel + (size_t)pt * nv;
  const double* du = tr.ctrl + (size_t)pt * nu;
  load_state(m, L, ln, tr, pt, seed, qfrc_applied, xfrc_applied);
  if (col < nctrl) {
    int i = col;
    ctrl[i] = du[i] + FD_EPS;
    dr[2 * nv * nv + nv * nu + 2 * nv + i] = (step_cost_ws(m, cost, qpos, qvel, ctrl) - costCenter) / FD_EPS;
    for (int j = 0; j < nv; j++) warm[j] = wc[j];
    dev::forward_skip(m, L, ln, dev::STAGE_NONE, FD_NITER, 0.0);
    for (int j = 0; j < nv; j++) temp[j] = qacc[j];
    ctrl[i] = du[i] - FD_EPS;
    for (int j = 0; j < nv; j++) warm[j] = wc[j];
    dev::forward_skip(m, L, ln, dev::STAGE_VEL, FD_NITER, 0.0);
    for (int j = 0; j < nv; j++) dr[2 * nv * nv + i + j * nu] = (temp[j] - qacc[j]) / (2 * FD_EPS);
  } else if (col < nctrl + nv) {
    int i = col - nctrl;
    qvel[i] = dv[i] + FD_EPS;
    dr[2 * nv * nv + nv * nu + nv + i] = (step_cost_ws(m, cost, qpos, qvel, ctrl) - costCenter) / FD_EPS;
    for (int j = 0; j < nv; j++) warm[j] = wc[j];
    dev::forward_skip(m, L, ln, dev::STAGE_NONE, FD_NITER, 0.0);
    for (int j = 0; j < nv; j++) temp[j] = qacc[j];
    qvel[i] = dv[i] - FD_EPS;
    for (int j = 0; j < nv; j++) warm[j] = wc[j];
    dev::forward_skip(m, L, ln, dev::STAGE_POS, FD_NITER, 0.0);
    for (int j = 0; j < nv; j++) dr[nv * nv + i + j * nv] = (temp[j] - qacc[j]) / (2 * FD_EPS);
  } else {
    int i = col - nctrl - nv;
    int jid = m.dof_jntid[i];
    int quatadr = -1, dofpos = 0;
    if (m.jnt_type[jid] == dev::JNT_BALL) {
      quatadr = m.jnt_qposadr[jid];
      dofpos = i - m.jnt_dofadr[jid];
    } else if (m.jnt_type[jid] == dev::JNT_FREE && i >= m.jnt_dofadr[jid] + 3) {
      quatadr = m.jnt_qposadr[jid] + 3;
      dofpos = i - m.jnt_dofadr[jid] - 3;
    }
    for (int side = 0; side < 2; side++) {
      double e = side == 0 ? FD_EPS : -FD_EPS;
      if (side == 1)
        for (int k = 0; k < m.nq; k++) qpos[k] = dq[k];
      if (quatadr >= 0) {
        double angvel[3] = {0, 0, 0}, q[4];
        angvel[dofpos] = e;
        dev::ld<4>(q, qpos + quatadr);
        dev::quat_integrate(q, angvel, 1);
        dev::st<4>(qpos + quatadr, q);
      } else {
        int a = m.jnt_qposadr[jid] + i - m.jnt_dofadr[jid];
        if (side == 0) qpos[a] += FD_EPS; else qpos[a] -= FD_EPS;
      }
      if (side == 0)
        dr[2 * nv * nv + nv * nu + i] = (step_cost_ws(m, cost, qpos, qvel, ctrl) - costCenter) / FD_EPS;
      for (int j = 0; j < nv; j++) warm[j] = wc[j];
      dev::forward_skip(m, L, ln, dev::STAGE_NONE, FD_NITER, 0.0);
      if (side == 0)
        for (int j = 0; j < nv; j++) temp[j] = qacc[j];
    }
    for (int j = 0; j < nv; j++) dr[i + j * nv] = (temp[j] - qacc[j]) / (2 * FD_EPS);
  }
}

__global__ __launch_bounds__(LANE_BLOCK) void k_rollout(DevModel m, WsLayout L, WsDev ws, int S, int A, int P,
                                                        TrajDev nom, TrajDev out, int out_is_cand, const double* K,
                                                        const double* k, const double* alphas, TrajDev dinit,
                                                        const double* qfrc_applied, const double* xfrc_applied,
                                                        int passive, CostDev cost, double* cost_cand) {
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= S * A) return;
  int s = lane / A, a = lane % A;
  const int nq = m.nq, nv = m.nv, nu = m.nu, nx = 2 * nv;
  Lane ln{ws.d + lane, ws.i + lane, (size_t)ws.nlanes};
  load_state(m, L, ln, dinit, s, s, qfrc_applied, xfrc_applied);
  SPd qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), ctrl = ln.D(L.ctrl), warm = ln.D(L.warm), timew = ln.D(L.time);
  SPd dx = ln.D(L.s_fd);
  const double alpha = alphas ? alphas[a] : 1.0;
  const int ob = out_is_cand ? lane : s;
  double c = 0;
  for (int n = P - 1; n >= 0; n--) {
    size_t pn = (size_t)s * P + n;
    if (!passive) {
      const double* xs_q = nom.qpos + pn * nq;
      const double* xs_v = nom.qvel + pn * nv;
      const double* us = nom.ctrl + pn * nu;
      const double* Kn = K + pn * nu * nx;
      const double* kn = k + pn * nu;
      for (int j = 0; j < nv; j++) dx[j] = qpos[j] - xs_q[j];
      for (int j = 0; j < nv; j++) dx[nv + j] = qvel[j] - xs_v[j];
      for (int i = 0; i < nu; i++) {
        double t = 0;
        for (int j = 0; j < nx; j++) t += Kn[i + j * nu] * dx[j];
        ctrl[i] = (t + alpha * kn[i]) + us[i];
      }
    }
    size_t po = (size_t)ob * P + n;
    out.time[po] = timew[0];
    for (int i = 0; i < nq; i++) out.qpos[po * nq + i] = qpos[i];
    for (int i = 0; i < nv; i++) out.qvel[po * nv + i] = qvel[i];
    for (int i = 0; i < nv; i++) out.warm[po * nv + i] = warm[i];
    for (int i = 0; i < nu; i++) out.ctrl[po * nu + i] = ctrl[i];
    c += step_cost_ws(m, cost, qpos, qvel, ctrl);
    dev::step(m, L, ln);
  }
  if (cost_cand) cost_cand[lane] = c;
}

__global__ void k_select(int nq, int nv, int nu, int S, int A, int P, int mode, int copy_cand,
                         const double* cost_cand, int* sel, double* cost_sel, TrajDev cand, TrajDev nom,
                         TrajDev dinit) {
  int s = blockIdx.x;
  __shared__ int best_sh;
  if (threadIdx.x == 0) {
    int best = 0;
    if (mode == 1 && cost_cand) {
      double bc = cost_cand[(size_t)s * A];
      for (int a = 1; a < A; a++) {
        double c = cost_cand[(size_t)s * A + a];
        if (c < bc || (bc != bc && c == c)) { bc = c; best = a; }
      }
    }
    best_sh = best;
    if (sel) sel[s] = best;
    if (cost_sel && cost_cand) cost_sel[s] = cost_cand[(size_t)s * A + best];
  }
  __syncthreads();
  int best = best_sh;
  if (copy_cand) {
    size_t src0 = ((size_t)s * A + best) * P, dst0 = (size_t)s * P;
    for (int p = threadIdx.x; p < P; p += blockDim.x) {
      nom.time[dst0 + p] = cand.time[src0 + p];
      for (int i = 0; i < nq; i++) nom.qpos[(dst0 + p) * nq + i] = cand.qpos[(src0 + p) * nq + i];
      for (int i = 0; i < nv; i++) nom.qvel[(dst0 + p) * nv + i] = cand.qvel[(src0 + p) * nv + i];
      for (int i = 0; i < nv; i++) nom.warm[(dst0 + p) * nv + i] = cand.warm[(src0 + p) * nv + i];
      for (int i = 0; i < nu; i++) nom.ctrl[(dst0 + p) * nu + i] = cand.ctrl[(src0 + p) * nu + i];
    }
  }
  __syncthreads();
  // setDInit(dArray[N]), inc/ilqr.h:183
  if (threadIdx.x == 0) {
    size_t src = (size_t)s * P + (P - 1);
    const TrajDev& t = copy_cand ? cand : nom;
    size_t sp = copy_cand ? ((size_t)s * A + best) * P + (P - 1) : src;
    dinit.time[s] = t.time[sp];
    for (int i = 0; i < nq; i++) dinit.qpos[(size_t)s * nq + i] = t.qpos[sp * nq + i];
    for (int i = 0; i < nv; i++) dinit.qvel[(size_t)s * nv + i] = t.qvel[sp * nv + i];
    for (int i = 0; i < nv; i++) dinit.warm[(size_t)s * nv + i] = t.warm[sp * nv + i];
    for (int i = 0; i < nu; i++) dinit.ctrl[(size_t)s * nu + i] = t.ctrl[sp * nu + i];
  }
}

// ---- Riccati backward pass: same loops, same order as oracle/ilqr_ora.c ----
// temp: n doubles of LDS scratch (a private array would live in scratch memory)
__device__ void ldlt_factor(int n, double* mat, int* transp, double* temp) {
  for (int k = 0; k < n; k++) {
    int big = k;
    double bigv = fabs(mat[k + k * n]);
    int rs = n - k - 1;
    for (int i = k + 1; i < n; i++)
      if (fabs(mat[i + i * n]) > bigv) { bigv = fabs(mat[i + i * n]); big = i; }
    transp[k] = big;
    if (k != big) {
      int s = n - big - 1;
      double t;
      for (int j = 0; j < k; j++) { t = mat[k + j * n]; mat[k + j * n] = mat[big + j * n]; mat[big + j * n] = t; }
      for (int i = 0; i < s; i++) {
        t = mat[(big + 1 + i) + k * n];
        mat[(big + 1 + i) + k * n] = mat[(big + 1 + i) + big * n];
        mat[(big + 1 + i) + big * n] = t;
      }
      t = mat[k + k * n]; mat[k + k * n] = mat[big + big * n]; mat[big + big * n] = t;
      for (int i = k + 1; i < big; i++) { t = mat[i + k * n]; mat[i + k * n] = mat[big + i * n]; mat[big + i * n] = t; }
    }
    if (k > 0) {
      double s = 0;
      for (int j = 0; j < k; j++) temp[j] = mat[j + j * n] * mat[k + j * n];
      for (int j = 0; j < k; j++) s += mat[k + j * n] * temp[j];
      mat[k + k * n] -= s;
      for (int i = k + 1; i < n; i++) {
        double si = 0;
        for (int j = 0; j < k; j++) si += mat[i + j * n] * temp[j];
        mat[i + k * n] -= si;
      }
    }
    if (k == 0 && !(fabs(mat[0]) > 0)) {
      for (int j = 0; j < n; j++) transp[j] = j;
      return;
    }
    if (rs > 0 && fabs(mat[k + k * n]) > 0)
      for (int i = k + 1; i < n; i++) mat[i + k * n] /= mat[k + k * n];
  }
}
__device__ void ldlt_solve(int n, const double* Lm, const int* transp, double* x) {
  const double tol = 2.2250738585072014e-308;
  for (int k = 0; k < n; k++) { double t = x[k]; x[k] = x[transp[k]]; x[transp[k]] = t; }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < i; j++) x[i] -= Lm[i + j * n] * x[j];
  for (int i = 0; i < n; i++) {
    if (fabs(Lm[i + i * n]) > tol) x[i] /= Lm[i + i * n];
    else x[i] = 0;
  }
  for (int i = n - 1; i >= 0; i--)
    for (int j = i + 1; j < n; j++) x[i] -= Lm[j + i * n] * x[j];
  for (int k = n - 1; k >= 0; k--) { double t = x[k]; x[k] = x[transp[k]]; x[transp[k]] = t; }
}

#ifdef ILQG_STAMPS
__device__ unsigned long long g_bstamp_acc[16];
__device__ unsigned long long g_bstamp_cnt[16];
#define BSTAMP(id)                                                \
  do {                                                            \
    if (tid == 0 && blockIdx.x == 0) {                            \
      unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
      if ((id) >= 0) {                                            \
        g_bstamp_acc[(id) < 0 ? 0 : (id)] += t_ - bst_prev;       \
        g_bstamp_cnt[(id) < 0 ? 0 : (id)]++;                      \
      }                                                           \
      bst_prev = t_;                                              \
    }                                                             \
  } while (0)
#else
#define BSTAMP(id) \
  do {             \
  } while (0)
#endif
constexpr int BW_THREADS = 64;  // one wavefront: its barriers compile to nothing
constexpr int BW_PF = 8;        // prefetch registers per lane: D <= 512

// Three independent fixed-order dot products per lane (ILP 3): each output
// keeps the oracle's summation order, the three chains overlap in the pipe.
#define ILP3_BEGIN(n)                                                       \
  for (int e0 = tid; e0 < (n); e0 += 3 * nt) {                              \
    const int e1 = e0 + nt, e2 = e0 + 2 * nt;                               \
    const bool h1 = e1 < (n), h2 = e2 < (n);                                \
    const int f1 = h1 ? e1 : e0, f2 = h2 ? e2 : e0;

__global__ __launch_bounds__(BW_THREADS) void k_backward(int nq, int nv, int nu, int P, double dt, double mu,
                                                         const double* deriv, TrajDev tr, double* Kg, double* kg,
                                                         double* Vg, double* vg) {
  const int s = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const int nx = 2 * nv, D = nv * (2 * nv + nu) + 2 * nv + nu;
  extern __shared__ double sh[];
  double* V = sh;
  double* Vs = V + nx * nx;
  double* A = Vs + nx * nx;
  double* ABK = A + nx * nx;
  double* T4 = ABK + nx * nx;
  double* Vn = T4 + nx * nx;
  double* B = Vn + nx * nx;
  double* T1 = B + nx * nu;
  double* T3 = T1 + nu * nx;
  double* T6 = T3 + nu * nx;
  double* Kl = T6 + nx * nu;
  double* Mm = Kl + nu * nx;
  double* v = Mm + nu * nu;
  double* c = v + nx;
  double* w = c + nx;
  double* y = w + nx;
  double* z = y + nx;
  double* vn = z + nx;
  double* q = vn + nx;
  double* kl = q + nx;
  double* kR = kl + nu;
  double* col = kR + nu;
  double* r = col + nu;
  double* dl = r + nu;  // FD record of the current step (prefetched)
  int* trn = (int*)(dl + D);

  // initV at the terminal point dArray[0], inc/ilqr.h:100-107
  {
    const double* q0 = deriv + ((size_t)s * P + 0) * D + 2 * nv * nv + nv * nu;
    for (int i = tid; i < nx; i += nt) v[i] = q0[i];
    const double* d1 = deriv + ((size_t)s * P + (P > 1 ? 1 : 0)) * D;
    for (int i = tid; i < D; i += nt) dl[i] = d1[i];
    __syncthreads();
    for (int e = tid; e < nx * nx; e += nt) { int i = e % nx, j = e / nx; V[e] = v[i] * v[j]; }
    __syncthreads();
  }
#ifdef ILQG_STAMPS
  unsigned long long bst_prev = 0;
#endif
  BSTAMP(-1);
  for (int n = 1; n < P; n++) {
    const size_t pc = (size_t)s * P + n, pp = pc - 1;
    // prefetch the next step's FD record; consumed at the end of this step
    double pf[BW_PF];
    if (n + 1 < P) {
      const double* dn1 = deriv + (pc + 1) * D;
#pragma unroll
      for (int t = 0; t < BW_PF; t++) {
        int i = tid + t * nt;
        pf[t] = i < D ? dn1[i] : 0.0;
      }
    }
    const double* dn = dl;
    // stage 1: symmetrise V, assemble A/B (differentiator.h:66-71,89-92), q, r, c
    for (int e = tid; e < nx * nx; e += nt) {
      int i = e % nx, j = e / nx;
      Vs[e] = (V[i + j * nx] + V[j + i * nx]) / 2;
      double val;
      if (i < nv && j < nv) val = (i == j) ? 1 : 0;
      else if (i < nv) val = (i == j - nv) ? dt : 0;
      else if (j < nv) val = dn[(i - nv) + j * nv] * dt;
      else val = ((i - nv) == (j - nv) ? 1 : 0) + dn[nv * nv + (i - nv) + (j - nv) * nv] * dt;
      A[e] = val;
    }
    for (int e = tid; e < nx * nu; e += nt) {
      int i = e % nx, j = e / nx;
      B[e] = (i < nv) ? 0 : dn[2 * nv * nv + (i - nv) + j * nv] * dt;
    }
    for (int i = tid; i < nx; i += nt) {
      q[i] = dn[2 * nv * nv + nv * nu + i];
      double xp = i < nv ? tr.qpos[pp * nq + i] : tr.qvel[pp * nv + i - nv];
      double xc = i < nv ? tr.qpos[pc * nq + i] : tr.qvel[pc * nv + i - nv];
      c[i] = xp - xc;
    }
    for (int a = tid; a < nu; a += nt) r[a] = dn[2 * nv * nv + nv * nu + nx + a];
    __syncthreads();
    for (int i = tid; i < nx; i += nt) Vs[i + i * nx] += mu;
    __syncthreads();
    BSTAMP(0);
    // stage 2: T1 = B'V
    ILP3_BEGIN(nu * nx)
      double s0 = 0, s1 = 0, s2 = 0;
      const int a0 = e0 % nu, j0 = e0 / nu, a1 = f1 % nu, j1 = f1 / nu, a2 = f2 % nu, j2 = f2 / nu;
      for (int kk = 0; kk < nx; kk++) {
        s0 += B[kk + a0 * nx] * Vs[kk + j0 * nx];
        s1 += B[kk + a1 * nx] * Vs[kk + j1 * nx];
        s2 += B[kk + a2 * nx] * Vs[kk + j2 * nx];
      }
      T1[e0] = s0;
      if (h1) T1[e1] = s1;
      if (h2) T1[e2] = s2;
    }
    __syncthreads();
    BSTAMP(1);
    // stage 3: Mm = -2 T1 B - 2R ; T3 = T1 A ; w = v + 2 V c
    for (int e = tid; e < nu * nu; e += nt) {
      int a = e % nu, b = e / nu;
      double sm = 0;
      for (int kk = 0; kk < nx; kk++) sm += T1[a + kk * nu] * B[kk + b * nx];
      Mm[e] = -2 * sm - 2 * (r[a] * r[b]);
    }
    ILP3_BEGIN(nu * nx)
      double s0 = 0, s1 = 0, s2 = 0;
      const int a0 = e0 % nu, j0 = e0 / nu, a1 = f1 % nu, j1 = f1 / nu, a2 = f2 % nu, j2 = f2 / nu;
      for (int kk = 0; kk < nx; kk++) {
        s0 += T1[a0 + kk * nu] * A[kk + j0 * nx];
        s1 += T1[a1 + kk * nu] * A[kk + j1 * nx];
        s2 += T1[a2 + kk * nu] * A[kk + j2 * nx];
      }
      T3[e0] = s0;
      if (h1) T3[e1] = s1;
      if (h2) T3[e2] = s2;
    }
    for (int i = tid; i < nx; i += nt) {
      double sm = 0;
      for (int j = 0; j < nx; j++) sm += Vs[i + j * nx] * c[j];
      w[i] = v[i] + 2 * sm;
    }
    __syncthreads();
    if (tid == 0) ldlt_factor(nu, Mm, trn, y);  // y is free until stage 5
    for (int a = tid; a < nu; a += nt) {
      double sm = 0;
      for (int kk = 0; kk < nx; kk++) sm += B[kk + a * nx] * w[kk];
      col[a] = sm + r[a];
    }
    __syncthreads();
    BSTAMP(2);
    // stage 4: K = ldlt.solve(2 T3) column-parallel; k = ldlt.solve(B'w + r)
    for (int j = tid; j < nx + 1; j += nt) {
      // solved in place in LDS (a private array would live in scratch)
      double* x = j < nx ? Kl + j * nu : kl;
      if (j < nx)
        for (int a = 0; a < nu; a++) x[a] = 2 * T3[a + j * nu];
      else
        for (int a = 0; a < nu; a++) x[a] = col[a];
      ldlt_solve(nu, Mm, trn, x);
    }
    __syncthreads();
    BSTAMP(3);
    // stage 5: ABK = A + B K ; T6 = K'R ; y = Bk + c ; kR = k'R
    for (int e = tid; e < nx * nx; e += nt) {
      int i = e % nx, j = e / nx;
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += B[i + a * nx] * Kl[a + j * nu];
      ABK[e] = A[e] + sm;
    }
    for (int e = tid; e < nx * nu; e += nt) {
      int i = e % nx, b = e / nx;
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += Kl[a + i * nu] * (r[a] * r[b]);
      T6[e] = sm;
    }
    for (int i = tid; i < nx; i += nt) {
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += B[i + a * nx] * kl[a];
      y[i] = sm + c[i];
    }
    for (int b = tid; b < nu; b += nt) {
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += kl[a] * (r[a] * r[b]);
      kR[b] = sm;
    }
    __syncthreads();
    BSTAMP(4);
    // stage 6: T4 = ABK' V
    ILP3_BEGIN(nx * nx)
      double s0 = 0, s1 = 0, s2 = 0;
      const int i0 = e0 % nx, j0 = e0 / nx, i1 = f1 % nx, j1 = f1 / nx, i2 = f2 % nx, j2 = f2 / nx;
      for (int kk = 0; kk < nx; kk++) {
        s0 += ABK[kk + i0 * nx] * Vs[kk + j0 * nx];
        s1 += ABK[kk + i1 * nx] * Vs[kk + j1 * nx];
        s2 += ABK[kk + i2 * nx] * Vs[kk + j2 * nx];
      }
      T4[e0] = s0;
      if (h1) T4[e1] = s1;
      if (h2) T4[e2] = s2;
    }
    __syncthreads();
    BSTAMP(5);
    // stage 7: V_new = (T4 ABK + Q) + T6 K
    ILP3_BEGIN(nx * nx)
      double a0s = 0, a1s = 0, a2s = 0, b0s = 0, b1s = 0, b2s = 0;
      const int i0 = e0 % nx, j0 = e0 / nx, i1 = f1 % nx, j1 = f1 / nx, i2 = f2 % nx, j2 = f2 / nx;
      for (int kk = 0; kk < nx; kk++) {
        a0s += T4[i0 + kk * nx] * ABK[kk + j0 * nx];
        a1s += T4[i1 + kk * nx] * ABK[kk + j1 * nx];
        a2s += T4[i2 + kk * nx] * ABK[kk + j2 * nx];
      }
      for (int b = 0; b < nu; b++) {
        b0s += T6[i0 + b * nx] * Kl[b + j0 * nu];
        b1s += T6[i1 + b * nx] * Kl[b + j1 * nu];
        b2s += T6[i2 + b * nx] * Kl[b + j2 * nu];
      }
      Vn[e0] = (a0s + q[i0] * q[j0]) + b0s;
      if (h1) Vn[e1] = (a1s + q[i1] * q[j1]) + b1s;
      if (h2) Vn[e2] = (a2s + q[i2] * q[j2]) + b2s;
    }
    __syncthreads();
    BSTAMP(6);
    // stage 8: z = (2y)' V_new ; v_new (reads the NEW V, Q14)
    for (int j = tid; j < nx; j += nt) {
      double sm = 0;
      for (int i = 0; i < nx; i++) sm += (2 * y[i]) * Vn[i + j * nx];
      z[j] = sm;
    }
    __syncthreads();
    for (int j = tid; j < nx; j += nt) {
      double ta = 0, tb = 0, td = 0;
      for (int i = 0; i < nx; i++) {
        ta += z[i] * ABK[i + j * nx];
        tb += v[i] * ABK[i + j * nx];
      }
      for (int b = 0; b < nu; b++) td += (2 * kR[b]) * Kl[b + j * nu];
      vn[j] = ((ta + tb) + q[j]) + td;
    }
    BSTAMP(7);
    // gains out
    for (int e = tid; e < nu * nx; e += nt) Kg[pc * nu * nx + e] = Kl[e];
    for (int a = tid; a < nu; a += nt) kg[pc * nu + a] = kl[a];
    __syncthreads();
    for (int e = tid; e < nx * nx; e += nt) V[e] = Vn[e];
    for (int i = tid; i < nx; i += nt) v[i] = vn[i];
    if (n + 1 < P) {
#pragma unroll
      for (int t = 0; t < BW_PF; t++) {
        int i = tid + t * nt;
        if (i < D) dl[i] = pf[t];
      }
    }
    __syncthreads();
    BSTAMP(8);
  }
  if (Vg)
    for (int e = tid; e < nx * nx; e += nt) Vg[(size_t)s * nx * nx + e] = V[e];
  if (vg)
    for (int i = tid; i < nx; i += nt) vg[(size_t)s * nx + i] = v[i];
}

__global__ __launch_bounds__(LANE_BLOCK) void k_step(DevModel m, WsLayout L, WsDev ws, TrajDev stt, int n,
                                                     int nstep, const double* qfrc_applied,
                                                     const double* xfrc_applied) {
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  Lane ln{ws.d + lane, ws.i + lane, (size_t)ws.nlanes};
  load_state(m, L, ln, stt, lane, lane, qfrc_applied, xfrc_applied);
  for (int t = 0; t < nstep; t++) dev::step(m, L, ln);
  SPd qpos = ln.D(L.qpos), qvel = ln.D(L.qvel), warm = ln.D(L.warm);
  stt.time[lane] = ln.D(L.time)[0];
  for (int i = 0; i < m.nq; i++) stt.qpos[(size_t)lane * m.nq + i] = qpos[i];
  for (int i = 0; i < m.nv; i++) stt.qvel[(size_t)lane * m.nv + i] = qvel[i];
  for (int i = 0; i < m.nv; i++) stt.warm[(size_t)lane * m.nv + i] = warm[i];
}

__global__ __launch_bounds__(LANE_BLOCK) void k_fwd(DevModel m, WsLayout L, WsDev ws, TrajDev stt, int n,
                                                    const double* qfrc_applied, const double* xfrc_applied,
                                                    double* qacc_out) {
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= n) return;
  Lane ln{ws.d + lane, ws.i + lane, (size_t)ws.nlanes};
  load_state(m, L, ln, stt, lane, lane, qfrc_applied, xfrc_applied);
  dev::forward_skip(m, L, ln, dev::STAGE_NONE, m.opt_iterations, m.opt_tolerance);
  SPd qacc = ln.D(L.qacc), warm = ln.D(L.warm);
  for (int i = 0; i < m.nv; i++) qacc_out[(size_t)lane * m.nv + i] = qacc[i];
  for (int i = 0; i < m.nv; i++) stt.warm[(size_t)lane * m.nv + i] = warm[i];
}

inline int nblk(long n, int b) { return (int)((n + b - 1) / b); }

}  // namespace

size_t backward_lds_bytes(int nv, int nu) {
  const int nx = 2 * nv;
  const size_t D = (size_t)nv * (2 * nv + nu) + 2 * nv + nu;
  size_t nd = 6 * (size_t)nx * nx + 5 * (size_t)nx * nu + (size_t)nu * nu + 8 * (size_t)nx + 4 * (size_t)nu + D;
  return nd * sizeof(double) + (size_t)nu * sizeof(int) + 16;
}

hipError_t launch_fd_centre(const DevModel& m, const WsLayout& L, WsDev ws, TrajDev tr, int npts, int P,
                            const double* qfrc_applied, const double* xfrc_applied, CostDev cost, double* warm_c,
                            double* cost_c, hipStream_t st) {
  if (npts <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fd_centre, dim3(nblk(npts, LANE_BLOCK)), dim3(LANE_BLOCK), 0, st, m, L, ws, tr, npts, P,
                     qfrc_applied, xfrc_applied, cost, warm_c, cost_c);
  return hipGetLastError();
}

hipError_t launch_fd_cols(const DevModel& m, const WsLayout& L, WsDev ws, TrajDev tr, int npts, int P,
                          const double* qfrc_applied, const double* xfrc_applied, CostDev cost, const double* warm_c,
                          const double* cost_c, double* deriv, hipStream_t st) {
  int nctrl = m.nu < m.nv ? m.nu : m.nv;
  long lanes = (long)npts * (nctrl + 2 * m.nv);
  if (lanes <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fd_cols, dim3(nblk(lanes, LANE_BLOCK)), dim3(LANE_BLOCK), 0, st, m, L, ws, tr, npts, P,
                     qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv);
  return hipGetLastError();
}

hipError_t launch_rollout(const DevModel& m, const WsLayout& L, WsDev ws, int S, int A, int P, TrajDev nominal,
                          TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas,
                          TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive,
                          CostDev cost, double* cost_cand, hipStream_t st) {
  hipLaunchKernelGGL(k_rollout, dim3(nblk((long)S * A, LANE_BLOCK)), dim3(LANE_BLOCK), 0, st, m, L, ws, S, A, P,
                     nominal, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost,
                     cost_cand);
  return hipGetLastError();
}

hipError_t launch_select(const DevModel& m, int S, int A, int P, int mode, int copy_cand, const double* cost_cand,
                         int* sel, double* cost_sel, TrajDev cand, TrajDev nominal, TrajDev dinit, hipStream_t st) {
  hipLaunchKernelGGL(k_select, dim3(S), dim3(256), 0, st, m.nq, m.nv, m.nu, S, A, P, mode, copy_cand, cost_cand,
                     sel, cost_sel, cand, nominal, dinit);
  return hipGetLastError();
}

hipError_t launch_backward(const DevModel& m, int S, int P, double mu, const double* deriv, TrajDev tr, double* K,
                           double* k, double* V, double* v, hipStream_t st) {
  size_t lds = backward_lds_bytes(m.nv, m.nu);
  hipLaunchKernelGGL(k_backward, dim3(S), dim3(BW_THREADS), lds, st, m.nq, m.nv, m.nu, P, m.opt_timestep, mu, deriv,
                     tr, K, k, V, v);
  return hipGetLastError();
}

hipError_t launch_step(const DevModel& m, const WsLayout& L, WsDev ws, TrajDev stt, int n, int nstep,
                       const double* qfrc_applied, const double* xfrc_applied, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_step, dim3(nblk(n, LANE_BLOCK)), dim3(LANE_BLOCK), 0, st, m, L, ws, stt, n, nstep,
                     qfrc_applied, xfrc_applied);
  return hipGetLastError();
}

hipError_t launch_forward(const DevModel& m, const WsLayout& L, WsDev ws, TrajDev stt, int n,
                          const double* qfrc_applied, const double* xfrc_applied, double* qacc, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fwd, dim3(nblk(n, LANE_BLOCK)), dim3(LANE_BLOCK), 0, st, m, L, ws, stt, n, qfrc_applied,
                     xfrc_applied, qacc);
  return hipGetLastError();
}

}  // namespace ilqg

#ifdef ILQG_STAMPS
// diagnostic build only: per-stage cycles of the Riccati kernel (block 0)
extern "C" int ilqg_debug_bstamps(unsigned long long* acc, unsigned long long* cnt, int reset) {
  if (hipMemcpyFromSymbol(acc, HIP_SYMBOL(ilqg::g_bstamp_acc), sizeof(unsigned long long) * 16) != hipSuccess)
    return 3;
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(ilqg::g_bstamp_cnt), sizeof(unsigned long long) * 16) != hipSuccess)
    return 3;
  if (reset) {
    unsigned long long z[16] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_bstamp_acc), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_bstamp_cnt), z, sizeof(z));
  }
  return 0;
}
#endif
