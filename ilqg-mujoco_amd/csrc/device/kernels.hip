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
                                                        double* deriv, int Ds) {
  const int nv = m.nv, nu = m.nu;
  const int nctrl = nu < nv ? nu : nv;  // mjderivative.cpp:78-82 (assumes nv >= nu)
  const int ncol = nctrl + 2 * nv;
  int lane = blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= npts * ncol) return;
  int pt = lane / ncol, col = lane % ncol, seed = pt / P;
  Lane ln{ws.d + lane, ws.i + lane, (size_t)ws.nlanes};
  double* dr = deriv + (size_t)pt * Ds;  // record stride Ds >= D
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
      for (int j = 0; j < nv; j++) dx[j] = state_diff_dof(m, j, qpos, xs_q);
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
                          const double* cost_c, double* deriv, int Ds, hipStream_t st) {
  int nctrl = m.nu < m.nv ? m.nu : m.nv;
  long lanes = (long)npts * (nctrl + 2 * m.nv);
  if (lanes <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fd_cols, dim3(nblk(lanes, LANE_BLOCK)), dim3(LANE_BLOCK), 0, st, m, L, ws, tr, npts, P,
                     qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv, Ds);
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

