// fp32 FD sweep (BASELINE.json configs[4]: humanoid H = 200, "fp32 FD with
// fp64 Riccati"): the two-kernel sweep of kernels_fd.hip -- k_fd_centre32
// (src/mjderivative.cpp:61-75, one workgroup per point) and k_fd_cols32
// (:78-206, one workgroup per (point, column)) -- on the fp32 instance of the
// cooperative physics (dcoop_f32.h).  Workspace, state and arithmetic on them
// are fp32 (half the LDS per team: the humanoid's 147 KB fp64 workspace fits
// one team per CU, the fp32 one two); the model stays fp64 in global memory
// and is rounded where read.  The records are fp64 (the fp32 central
// differences, widened) for the fp64 Riccati recursion.  eps = 1e-3 (SURVEY.md
// §7(g): 1e-6 is below fp32 resolution); no bit-exactness claim -- parity is a
// stated tolerance against the fp64 oracle at the same eps.
#include "dcoop_f32.h"
#include "kernels.h"

namespace ilqg {
namespace {

using namespace coopf;

constexpr int TEAM32 = TEAM_SIZE;
constexpr int FD32_NITER = 30;   // mjderivative.cpp:37
constexpr int FD32_NWARMUP = 3;  // mjderivative.cpp:38
// The physics pipeline inlined at every call site of these kernels.  Left to
// the inliner's size heuristic, forward_skip stayed an outlined call, and a
// call takes the model (MT, a ~1 KB struct of sizes and pointers) and the
// layouts by reference: the kernel copied them into scratch memory (1,040 B a
// lane) and every model field the physics read was a load from it.  Inlined,
// the fields are kernel arguments again (0 scratch; VGPRs 248 -> 139 in
// k_fd_cols32<DevModelNV<27>>).  ILQG_FD32_INL=0 restores the call (A/B).
#ifndef ILQG_FD32_INL
#define ILQG_FD32_INL 1
#endif
#if ILQG_FD32_INL
#define FD32_INL [[clang::always_inline]]
#else
#define FD32_INL
#endif

// LDS: [workspace floats][coop floats][workspace ints][coop ints]; the model
// image is read from global memory
__device__ inline Team make_team32(const WsLayout& L, const coop::CoopLayout& C) {
  extern __shared__ float lds32[];
  Team T;
  T.w = lds32;
  T.c = lds32 + L.nd;
  T.iw = reinterpret_cast<int*>(lds32 + L.nd + C.nd);
  T.ci = T.iw + L.ni;
  T.tid = threadIdx.x & (TEAM32 - 1);
  T.nt = TEAM32;
  return T;
}

template <class X>
__device__ inline double cost_terms32(double c, const X* x, const double* w, const double* t, const double* l, int n) {
  for (int i = 0; i < n; i++) {
    const double xi = x[i];
    if (w[i] != 0) {
      const double dx = xi - t[i];
      c += w[i] * dx * dx;
    }
    if (l[i] != 0) c += l[i] * xi;
  }
  return c;
}
template <class X>
__device__ inline float step_cost32(const DevModel& m, const CostDev& c, const X* qpos, const X* qvel,
                                    const X* ctrl) {
  double s = 0;
  s = cost_terms32(s, qpos, c.wq, c.tq, c.lq, m.nq);
  s = cost_terms32(s, qvel, c.wv, c.tv, c.lv, m.nv);
  s = cost_terms32(s, ctrl, c.wu, c.tu, c.lu, m.nu);
  return (float)s;
}

// cpMjData(d, src) from a trajectory record (src/util.cpp:4-14), rounded to fp32
__device__ inline void load_state32(const DevModel& m, const WsLayout& L, const Team& T, const TrajDev& tr, int pt,
                                    int seed, const double* qfrc_applied, const double* xfrc_applied) {
  FOR_T(i, m.nq) T.w[L.qpos + i] = (float)tr.qpos[(size_t)pt * m.nq + i];
  FOR_T(i, m.nv) {
    T.w[L.qvel + i] = (float)tr.qvel[(size_t)pt * m.nv + i];
    T.w[L.warm + i] = (float)tr.warm[(size_t)pt * m.nv + i];
    T.w[L.qfrc_applied + i] = qfrc_applied ? (float)qfrc_applied[(size_t)seed * m.nv + i] : 0.f;
  }
  FOR_T(i, m.nu) T.w[L.ctrl + i] = (float)tr.ctrl[(size_t)pt * m.nu + i];
  FOR_T(i, 6 * m.nbody)
  T.w[L.xfrc_applied + i] = xfrc_applied ? (float)xfrc_applied[(size_t)seed * 6 * m.nbody + i] : 0.f;
  if (T.tid == 0) T.w[L.time] = (float)tr.time[pt];
  TSYNC();
}

// MT: DevModel, or DevModelNV<27> for 27-dof models (the humanoid: compile-time
// sizes in the Newton Cholesky and its substitution, as the rollout's instance)
template <class MT>
__global__ __launch_bounds__(TEAM32) void k_fd_centre32(DevModel mg, WsLayout L, coop::CoopLayout C, coop::CoopAux X,
                                                        TrajDev tr, int P, const double* qfrc_applied,
                                                        const double* xfrc_applied, CostDev cost, double* warm_c,
                                                        double* cost_c) {
  MT m;
  static_cast<DevModel&>(m) = mg;
  Team T = make_team32(L, C);
  const int pt = blockIdx.x;
  load_state32(m, L, T, tr, pt, pt / P, qfrc_applied, xfrc_applied);
  // every physics call inlined (FD32_INL): see k_fd_cols32
  FD32_INL forward_skip(m, L, C, X, T, STAGE_NONE, FD32_NITER, 0.0);
  for (int rep = 1; rep < FD32_NWARMUP; rep++) FD32_INL forward_skip(m, L, C, X, T, STAGE_VEL, FD32_NITER, 0.0);
  FOR_T(i, m.nv) warm_c[(size_t)pt * m.nv + i] = T.w[L.warm + i];
  // the centre cost on the fp32 state, as the perturbed costs below see it
  if (T.tid == 0) cost_c[pt] = step_cost32(m, cost, T.w + L.qpos, T.w + L.qvel, T.w + L.ctrl);
}

template <class MT>
__global__ __launch_bounds__(TEAM32) void k_fd_cols32(DevModel mg, WsLayout L, coop::CoopLayout C, coop::CoopAux X,
                                                      TrajDev tr, int P, const double* qfrc_applied,
                                                      const double* xfrc_applied, CostDev cost, const double* warm_c,
                                                      const double* cost_c, double* deriv, int Ds, float eps) {
  MT m;
  static_cast<DevModel&>(m) = mg;
  Team T = make_team32(L, C);
  const int nv = m.nv, nu = m.nu;
  const int nctrl = nu < nv ? nu : nv;  // mjderivative.cpp:78-82 (assumes nv >= nu)
  const int ncol = nctrl + 2 * nv;
  const int pt = blockIdx.x / ncol, col = blockIdx.x % ncol;
  double* dr = deriv + (size_t)pt * Ds;
  const double* wc = warm_c + (size_t)pt * nv;
  const float costCenter = (float)cost_c[pt];
  float* qpos = T.w + L.qpos;
  float* qvel = T.w + L.qvel;
  float* ctrl = T.w + L.ctrl;
  float* warm = T.w + L.warm;
  float* qacc = T.w + L.qacc;
  float* temp = T.w + L.s_fd;
  load_state32(m, L, T, tr, pt, pt / P, qfrc_applied, xfrc_applied);
  int kind, i, skip_minus;
  if (col < nctrl) { kind = 0; i = col; skip_minus = STAGE_VEL; }
  else if (col < nctrl + nv) { kind = 1; i = col - nctrl; skip_minus = STAGE_POS; }
  else { kind = 2; i = col - nctrl - nv; skip_minus = STAGE_NONE; }
  int quatadr = -1, dofpos = 0, jid = m.dof_jntid[i];
  if (kind == 2) {
    if (m.jnt_type[jid] == JNT_BALL) {
      quatadr = m.jnt_qposadr[jid];
      dofpos = i - m.jnt_dofadr[jid];
    } else if (m.jnt_type[jid] == JNT_FREE && i >= m.jnt_dofadr[jid] + 3) {
      quatadr = m.jnt_qposadr[jid] + 3;
      dofpos = i - m.jnt_dofadr[jid] - 3;
    }
  }
  // the unperturbed fp32 values, re-read from the trajectory point (any nq, nv, nu)
  const float ui = kind == 0 ? (float)tr.ctrl[(size_t)pt * nu + i] : 0.f;
  const float vi = kind == 1 ? (float)tr.qvel[(size_t)pt * nv + i] : 0.f;
  auto perturb = [&](float h) {
    if (kind == 0) ctrl[i] = ui + h;
    else if (kind == 1) qvel[i] = vi + h;
    else if (quatadr >= 0) {
      float angvel[3] = {0, 0, 0}, q[4];
      angvel[dofpos] = h;
      ldm<4>(q, qpos + quatadr);
      quat_integrate(q, angvel, 1.0f);
      for (int k = 0; k < 4; k++) qpos[quatadr + k] = q[k];
    } else {
      qpos[m.jnt_qposadr[jid] + i - m.jnt_dofadr[jid]] += h;
    }
  };
  // + side: perturb, forward-difference cost, dynamics from the centre warmstart
  if (T.tid == 0) {
    perturb(eps);
    const float cp = (step_cost32(m, cost, qpos, qvel, ctrl) - costCenter) / eps;
    const int at = kind == 0 ? 2 * nv * nv + nv * nu + 2 * nv + i
                             : (kind == 1 ? 2 * nv * nv + nv * nu + nv + i : 2 * nv * nv + nv * nu + i);
    dr[at] = cp;
  }
  FOR_T(j, nv) warm[j] = (float)wc[j];
  TSYNC();
  FD32_INL forward_skip(m, L, C, X, T, STAGE_NONE, FD32_NITER, 0.0);
  FOR_T(j, nv) temp[j] = qacc[j];
  // qpos undo before the minus side (mjderivative.cpp:184): the fp32 centre state
  if (kind == 2) FOR_T(k, m.nq) qpos[k] = (float)tr.qpos[(size_t)pt * m.nq + k];
  TSYNC();
  // - side
  if (T.tid == 0) {
    perturb(-eps);
  }
  FOR_T(j, nv) warm[j] = (float)wc[j];
  TSYNC();
  FD32_INL forward_skip(m, L, C, X, T, skip_minus, FD32_NITER, 0.0);
  FOR_T(j, nv) {
    const float v = (temp[j] - qacc[j]) / (2 * eps);
    if (kind == 0) dr[2 * nv * nv + i + j * nu] = v;
    else if (kind == 1) dr[nv * nv + i + j * nv] = v;
    else dr[i + j * nv] = v;
  }
}

}  // namespace

size_t coop_lds_bytes_f32(const WsLayout& L, const coop::CoopLayout& C) {
  return (size_t)(L.nd + C.nd) * sizeof(float) + (size_t)(L.ni + C.ni) * sizeof(int);
}

static hipError_t allow_lds32(const void* kern, size_t lds) {
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

template <class MT>
static hipError_t launch_fd32_t(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C, const coop::CoopAux& X,
                                TrajDev tr, int npts, int P, const double* qfrc_applied, const double* xfrc_applied,
                                CostDev cost, double* warm_c, double* cost_c, double* deriv, int Ds, double eps,
                                hipStream_t st) {
  const size_t lds = coop_lds_bytes_f32(L, C);
  hipError_t e = allow_lds32(reinterpret_cast<const void*>(k_fd_centre32<MT>), lds);
  if (e != hipSuccess) return e;
  e = allow_lds32(reinterpret_cast<const void*>(k_fd_cols32<MT>), lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fd_centre32<MT>, dim3(npts), dim3(TEAM32), lds, st, m, L, C, X, tr, P, qfrc_applied,
                     xfrc_applied, cost, warm_c, cost_c);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int nctrl = m.nu < m.nv ? m.nu : m.nv;
  const long blocks = (long)npts * (nctrl + 2 * m.nv);
  hipLaunchKernelGGL(k_fd_cols32<MT>, dim3((unsigned)blocks), dim3(TEAM32), lds, st, m, L, C, X, tr, P, qfrc_applied,
                     xfrc_applied, cost, warm_c, cost_c, deriv, Ds, (float)eps);
  return hipGetLastError();
}

hipError_t launch_fd_sweep_f32(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                               const coop::CoopAux& X, TrajDev tr, int npts, int P, const double* qfrc_applied,
                               const double* xfrc_applied, CostDev cost, double* warm_c, double* cost_c,
                               double* deriv, int Ds, double eps, hipStream_t st) {
  if (npts <= 0) return hipSuccess;
  static const int nvc_env = [] {
    const char* v = getenv("ILQG_NV_CONST");
    return (v && v[0] == '0') ? 0 : 1;
  }();
  if (nvc_env && m.nv == 27) return launch_fd32_t<DevModelNV<27>>(m, L, C, X, tr, npts, P, qfrc_applied, xfrc_applied,
                                                                 cost, warm_c, cost_c, deriv, Ds, eps, st);
  return launch_fd32_t<DevModel>(m, L, C, X, tr, npts, P, qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv, Ds,
                                 eps, st);
}

}  // namespace ilqg
