// Cooperative FD-sweep kernels: one 64-lane workgroup (one wavefront) per
// physics evaluation, workspace in LDS (dcoop.h).
//   k_fd_centre_coop  src/mjderivative.cpp:61-75   one workgroup per trajectory point
//   k_fd_cols_coop    src/mjderivative.cpp:78-206  one workgroup per (point, column)
//   k_fd_fused_*      the sweep with the Riccati recursion (inc/ilqr.h:133-176)
//                     streamed behind it, one ticketed launch
// diagnostic build: stamps from every 64th workgroup (a sample of every team role)
#define ILQG_STAMP_SAMPLE 6
#include "coop_common.h"
#include "riccati.h"

namespace ilqg {
namespace {

__device__ inline void fd_centre_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                TrajDev tr, int P, const double* qfrc_applied, const double* xfrc_applied, CostDev cost, double* warm_c, double* cost_c) {
  STAMP_INIT();
  const int pt = blockIdx.x;
  load_state(m, L, T, tr, pt, pt / P, qfrc_applied, xfrc_applied);
  forward_skip(m, L, C, X, T, STAGE_NONE, FD_NITER, 0.0);
  for (int rep = 1; rep < FD_NWARMUP; rep++) forward_skip(m, L, C, X, T, STAGE_VEL, FD_NITER, 0.0);
  FOR_T(i, m.nv) warm_c[(size_t)pt * m.nv + i] = T.w[L.warm + i];
  if (T.tid == 0)
    cost_c[pt] = step_cost(m, cost, tr.qpos + (size_t)pt * m.nq, tr.qvel + (size_t)pt * m.nv,
                           tr.ctrl + (size_t)pt * m.nu);
  STAMP_FLUSH();
}

__global__ __launch_bounds__(TEAM, FD_WAVES_PER_EU) void k_fd_centre_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, TrajDev tr, int P, const double* qfrc_applied, const double* xfrc_applied, CostDev cost, double* warm_c, double* cost_c) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  fd_centre_body(m, L, C, X, T, tr, P, qfrc_applied, xfrc_applied, cost, warm_c, cost_c);
}

// model-specific instance (static_models.h): compile-time sizes, tables and LDS layout
template <class SM, class SX>
__global__ __launch_bounds__(TEAM, FD_WAVES_PER_EU) void k_fd_centre_s(DevModel mg, TrajDev tr, int P, const double* qfrc_applied, const double* xfrc_applied, CostDev cost, double* warm_c, double* cost_c) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_s(mg, L, C, T, m);
  fd_centre_body(m, L, C, X, T, tr, P, qfrc_applied, xfrc_applied, cost, warm_c, cost_c);
}

__device__ inline void fd_cols_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                TrajDev tr, int P, const double* qfrc_applied, const double* xfrc_applied, CostDev cost, const double* warm_c, const double* cost_c, double* deriv, int Ds) {
  STAMP_INIT();
  const int nv = m.nv, nu = m.nu;
  const int nctrl = nu < nv ? nu : nv;  // mjderivative.cpp:78-82 (assumes nv >= nu)
  const int ncol = nctrl + 2 * nv;
  const int pt = blockIdx.x / ncol, col = blockIdx.x % ncol;
  double* dr = deriv + (size_t)pt * Ds;  // record stride Ds >= D
  const double* wc = warm_c + (size_t)pt * nv;
  const double costCenter = cost_c[pt];
  double* qpos = T.w + L.qpos;
  double* qvel = T.w + L.qvel;
  double* ctrl = T.w + L.ctrl;
  double* warm = T.w + L.warm;
  double* qacc = T.w + L.qacc;
  double* temp = T.w + L.s_fd;
  const double* dq = tr.qpos + (size_t)pt * m.nq;
  const double* dv = tr.qvel + (size_t)pt * nv;
  const double* du = tr.ctrl + (size_t)pt * nu;
  load_state(m, L, T, tr, pt, pt / P, qfrc_applied, xfrc_applied);
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
  // + side: perturb, forward-difference cost, dynamics from the centre warmstart
  if (T.tid == 0) {
    if (kind == 0) ctrl[i] = du[i] + FD_EPS;
    else if (kind == 1) qvel[i] = dv[i] + FD_EPS;
    else if (quatadr >= 0) {
      double angvel[3] = {0, 0, 0}, q[4];
      angvel[dofpos] = FD_EPS;
      ldm<4>(q, qpos + quatadr);
      quat_integrate(q, angvel, 1);
      for (int k = 0; k < 4; k++) qpos[quatadr + k] = q[k];
    } else {
      qpos[m.jnt_qposadr[jid] + i - m.jnt_dofadr[jid]] += FD_EPS;
    }
    double cp = (step_cost(m, cost, qpos, qvel, ctrl) - costCenter) / FD_EPS;
    int at = kind == 0 ? 2 * nv * nv + nv * nu + 2 * nv + i
                       : (kind == 1 ? 2 * nv * nv + nv * nu + nv + i : 2 * nv * nv + nv * nu + i);
    dr[at] = cp;
  }
  FOR_T(j, nv) warm[j] = wc[j];
  TSYNC();
  forward_skip(m, L, C, X, T, STAGE_NONE, FD_NITER, 0.0);
  FOR_T(j, nv) temp[j] = qacc[j];
  if (kind == 2) FOR_T(k, m.nq) qpos[k] = dq[k];
  TSYNC();
  // - side
  if (T.tid == 0) {
    if (kind == 0) ctrl[i] = du[i] - FD_EPS;
    else if (kind == 1) qvel[i] = dv[i] - FD_EPS;
    else if (quatadr >= 0) {
      double angvel[3] = {0, 0, 0}, q[4];
      angvel[dofpos] = -FD_EPS;
      ldm<4>(q, qpos + quatadr);
      quat_integrate(q, angvel, 1);
      for (int k = 0; k < 4; k++) qpos[quatadr + k] = q[k];
    } else {
      qpos[m.jnt_qposadr[jid] + i - m.jnt_dofadr[jid]] -= FD_EPS;
    }
  }
  FOR_T(j, nv) warm[j] = wc[j];
  TSYNC();
  forward_skip(m, L, C, X, T, skip_minus, FD_NITER, 0.0);
  FOR_T(j, nv) {
    double v = (temp[j] - qacc[j]) / (2 * FD_EPS);
    if (kind == 0) dr[2 * nv * nv + i + j * nu] = v;
    else if (kind == 1) dr[nv * nv + i + j * nv] = v;
    else dr[i + j * nv] = v;
  }
  STAMP_FLUSH();
}

__global__ __launch_bounds__(TEAM, FD_WAVES_PER_EU) void k_fd_cols_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, TrajDev tr, int P, const double* qfrc_applied, const double* xfrc_applied, CostDev cost, const double* warm_c, const double* cost_c, double* deriv, int Ds) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  fd_cols_body(m, L, C, X, T, tr, P, qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv, Ds);
}

// model-specific instance (static_models.h): compile-time sizes, tables and LDS layout
template <class SM, class SX>
__global__ __launch_bounds__(TEAM, FD_WAVES_PER_EU) void k_fd_cols_s(DevModel mg, TrajDev tr, int P, const double* qfrc_applied, const double* xfrc_applied, CostDev cost, const double* warm_c, const double* cost_c, double* deriv, int Ds) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_s(mg, L, C, T, m);
  fd_cols_body(m, L, C, X, T, tr, P, qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv, Ds);
}

// ---- fused FD sweep with the backward pass streamed behind it ------------
// One launch per sweep.  A workgroup takes a ticket (an atomic counter) when it
// starts; tickets < nB are backward-pass roles (one per seed), the rest are FD
// teams: first every centre team C(s,p), then per point p the column teams of
// every seed, points in the order the Riccati recursion consumes them
// (terminal point first, inc/ilqr.h:144):
//   C(s,p): cpMjData + mj_forward + 2 forwardSkip(VEL) (mjderivative.cpp:61-75),
//           publishes the centre warm start and cost;
//   U(s,p,i): ctrl column i (:78-111) on a position/velocity stage of its own
//           (ctrl enters only the acceleration stage);
//   V(s,p,i): qvel column i (:114-142);
//   Q(s,p,i): qpos column i (:145-206).
// Every team runs exactly one evaluation pair and no loop around the physics
// pipeline (a loop let the compiler hoist model reads out of it and keep them
// live across the whole pipeline: 51 VGPRs spilled).  U, V and Q teams run
// their first position/velocity stages before they wait for C's warm start
// (those stages never read it).  A team stores its deriv entries write-through
// and announces them on done[s,p] (handoff.h); the backward role reads record p
// once all 1 + nu + 2 nv teams have announced.  Every evaluation reads exactly
// the inputs the two-kernel sweep gives it, so the records are bit-identical.
// Deadlock-free: a team waits only on work holding a smaller ticket (already
// running, never waiting), the backward roles only on FD teams (which never
// wait on them).
__device__ inline unsigned take_ticket(unsigned* sync) {
  unsigned t = 0;
  if ((threadIdx.x & (TEAM - 1)) == 0)
    t = __hip_atomic_fetch_add((gu32*)sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane(t);
}

// FD item u -> role (0 = C, 1 = V, 2 = Q, 3 = U), seed, point, index; ntm = nu + 2 nv
// column teams per (seed, point)
// (a.halves: every column is two items, its + and - evaluations, adjacent;
// half = 0 / 1, else -1)
__device__ inline void fd_decode(const FdFused& a, unsigned ntm, unsigned u, int& role, int& s, int& p, int& idx,
                                 int& half) {
  const unsigned nt = a.halves ? 2 * ntm : ntm;
  const unsigned nC = a.S * a.P, nW = a.S * nt;
  idx = 0;
  half = -1;
  if (u < nC) {
    role = 0; p = u / a.S; s = u % a.S;
    return;
  }
  u -= nC;
  p = u / nW;
  const unsigned o = u % nW;
  s = o / nt;
  int w = o % nt;
  if (a.halves) {
    half = w & 1;
    w >>= 1;
  }
  if (w < a.nut) { role = 3; idx = w; }
  else if (w < a.nut + a.nv) { role = 1; idx = w - a.nut; }
  else { role = 2; idx = w - a.nut - a.nv; }
}

#ifdef ILQG_STAMPS
// diagnostic timeline of the fused sweep: per FD item u (ticket - nB) its
// start and end (s_memrealtime, 100 MHz) and its XCC / SE / CU; per backward
// role its start and end (tools/fused_timeline.py)
constexpr int TL_N = 131072;
static __device__ unsigned long long g_tl[3 * TL_N];
static __device__ unsigned long long g_tlb[2 * 64];
__device__ inline unsigned long long hw_where() {
  const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));       // HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));     // XCC_ID
  return ((unsigned long long)xcc << 32) | hw;
}
#endif
// The workspace doubles a qvel or ctrl FD team reads after taking the centre's
// state at the end of its velocity stage (the team then runs the velocity
// stage again, qvel teams, and the acceleration stage + constraint solve):
// the state block (qpos .. time), xipos, scom / cdof / cinert, qM / qLD /
// qLDinv / amom (the position stage's outputs the later stages read), the
// velocity stage's outputs (cvel .. qfrc_con), and the constraint rows
// [0, nefc) of efc_J / pos / margin / D / KBIP / vel / aref.  Everything else
// (the other frames, crb, the narrow phase's contacts and candidates, scratch)
// is dead by then.  tests/test_gpu_parity.py::test_fused_sweep_schedules runs
// with ILQG_SNAP_POISON=1 (every double not listed reads as NaN).
constexpr int SNAP_NR = 12;
__device__ __forceinline__ void snap_ranges(const auto& m, const auto& L, int nefc, int (&o)[SNAP_NR],
                                            int (&l)[SNAP_NR]) {
  const int nv = m.nv, nb = m.nbody, nu = m.nu;
  o[0] = L.qpos;       l[0] = L.time + 1 - L.qpos;
  o[1] = L.xipos;      l[1] = 3 * nb;
  o[2] = L.scom;       l[2] = L.cinert + 10 * nb - L.scom;
  o[3] = L.qM;         l[3] = L.amom + nu * nv - L.qM;
  o[4] = L.cvel;       l[4] = L.qfrc_con + nv - L.cvel;
  o[5] = L.efc_J;      l[5] = nefc * nv;
  o[6] = L.efc_pos;    l[6] = nefc;
  o[7] = L.efc_margin; l[7] = nefc;
  o[8] = L.efc_D;      l[8] = nefc;
  o[9] = L.efc_KBIP;   l[9] = L.kstr * nefc;
  o[10] = L.efc_vel;   l[10] = nefc;
  o[11] = L.efc_aref;  l[11] = nefc;
}
// LDS double of packed snapshot entry e
__device__ __forceinline__ int snap_dst(int e, const int (&o)[SNAP_NR], const int (&l)[SNAP_NR]) {
  int d = 0;
#pragma unroll
  for (int r = 0; r < SNAP_NR; r++) {
    if (e >= 0 && e < l[r]) d = o[r] + e;
    e -= l[r];
  }
  return d;
}

__device__ inline void fd_fused_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                     const FdFused& a, unsigned u) {
  // late tickets first in the SIMD's issue arbitration: they set the launch's tail
  if (u >= a.prio2) __builtin_amdgcn_s_setprio(2);
  else if (u >= a.prio1) __builtin_amdgcn_s_setprio(1);
  // the planned schedule (launch_fd_plan); readfirstlane: the item stays wave-uniform (SGPR)
  if (a.order) {
    u = __builtin_amdgcn_readfirstlane(a.order[u]);
    // launch_fd_order_check has validated the map; an id out of range is still
    // never decoded into addresses (a reported fault, not a memory fault)
    const unsigned nI = (unsigned)a.S * a.P * (1u + (a.halves ? 2u : 1u) * (unsigned)(a.nut + 2 * m.nv));
    if (u >= nI) {
      if ((threadIdx.x & (TEAM - 1)) == 0) raise_fault(a.fault);
      return;
    }
  }
  const unsigned long long tstart = __builtin_amdgcn_s_memrealtime();
  STAMP_INIT();
#ifdef ILQG_STAMPS
  const unsigned long long tteam_ = __builtin_amdgcn_s_memtime();
  if (T.tid == 0 && u < (unsigned)TL_N) {
    g_tl[3 * u] = __builtin_amdgcn_s_memrealtime();
    g_tl[3 * u + 2] = hw_where();
  }
#endif
  const int nv = m.nv, nu = m.nu, nq = m.nq;
  const int nctrl = nu < nv ? nu : nv;  // mjderivative.cpp:78-82 (assumes nv >= nu)
  int role, s, p, idx, half;
  const int ntm = a.nut + 2 * nv;
  fd_decode(a, ntm, u, role, s, p, idx, half);
  const int pt = s * a.P + p;
  double* dr = a.deriv + (size_t)pt * a.Dp;
  double* cwp = a.cw + (size_t)pt * a.WCp;
  unsigned* cflag = a.sync + 4 + pt;
  unsigned* done = a.sync + 4 + (size_t)a.S * a.P + pt;
  double* qpos = T.w + L.qpos;
  double* qvel = T.w + L.qvel;
  double* ctrl = T.w + L.ctrl;
  double* warm = T.w + L.warm;
  double* qacc = T.w + L.qacc;
  const int tid = T.tid;
  const int G = 2 * nv * nv + nv * nu;  // cost-gradient entries: qpos, qvel, ctrl
  const double* dq = a.tr.qpos + (size_t)pt * nq;
  // the centre's position/velocity workspace snapshot (a.snap): the team's LDS
  // ints [iw | ci] in full, then only the doubles a qvel or ctrl team reads
  // after the centre's velocity stage (snap_ranges), the constraint rows cut
  // to the point's nefc
  const int nwd = L.nd + C.nd, nid = L.ni + C.ni;
  const bool snap = a.snap && (nid + 1) / 2 + nwd <= a.snapd;
  double* sp = snap ? a.snap + (size_t)pt * a.snapd : nullptr;
  double* spd = sp + (nid + 1) / 2;
  unsigned* sflag = a.sync + 4 + 2 * (size_t)a.S * a.P + pt;
  int ro[SNAP_NR], rl[SNAP_NR];
  auto snap_store = [&]() {
    FOR_T(e, nid) st_sc1_i(reinterpret_cast<int*>(sp) + e, T.iw[e]);
    snap_ranges(m, L, T.iw[L.nefc], ro, rl);
    int base = 0;
#pragma unroll
    for (int r = 0; r < SNAP_NR; r++) {
      FOR_T(e, rl[r]) st_sc1(spd + base + e, T.w[ro[r] + e]);
      base += rl[r];
    }
    drain_stores();
    TSYNC();
    if (tid == 0) signal_set(sflag, 1u);
  };
  auto snap_load = [&]() {
    bw_wait_geq(sflag, 1u, a.fault);
    // sixteen loads in flight per lane before their LDS stores
    constexpr int CH = 16;
    for (int e0 = 0; e0 < nid; e0 += CH * TEAM) {
      int v[CH];
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const int e = e0 + q * TEAM + tid;
        v[q] = e < nid ? ld_sc1_i(reinterpret_cast<const int*>(sp) + e) : 0;
      }
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const int e = e0 + q * TEAM + tid;
        if (e < nid) T.iw[e] = v[q];
      }
    }
    // (a.poison, tests: every double the snapshot does not carry reads as NaN,
    // so a field missing from snap_ranges changes the records)
    if (a.poison) {
      FOR_T(e, nwd) T.w[e] = __builtin_nan("");
    }
    TSYNC();
    snap_ranges(m, L, T.iw[L.nefc], ro, rl);
    int n = 0;
#pragma unroll
    for (int r = 0; r < SNAP_NR; r++) n += rl[r];
    for (int e0 = 0; e0 < n; e0 += CH * TEAM) {
      double v[CH];
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const int e = e0 + q * TEAM + tid;
        v[q] = e < n ? ld_sc1(spd + e) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < CH; q++) {
        const int e = e0 + q * TEAM + tid;
        if (e < n) T.w[snap_dst(e, ro, rl)] = v[q];
      }
    }
    TSYNC();
  };
  // qvel / ctrl teams with a snapshot take their whole state from it
  if (!(snap && (role == 1 || role == 3))) load_state(m, L, T, a.tr, pt, s, a.qfrc_applied, a.xfrc_applied);
  bool announce = true;           // this team signals done[s,p] (a.halves: the column's second half)
  double wc = 0, costCenter = 0;  // centre warm start (lane j holds entry j) and cost
  auto set_warm = [&]() {
    if (tid < nv) warm[tid] = wc;
    TSYNC();
  };
  auto get_centre = [&]() {
    bw_wait_geq(cflag, 1u, a.fault);
    wc = tid < nv ? ld_sc1(cwp + tid) : 0.0;
    costCenter = ld_sc1(cwp + nv);
  };
  if (role == 0) {
    // centre: mj_forward + nwarmup - 1 = 2 forwardSkip(VEL) (written out: no loop)
    static_assert(FD_NWARMUP == 3, "centre warm-up");
    if (snap) {
      // forward_skip(STAGE_NONE) with the workspace published between its
      // velocity and acceleration stages
      forward_posvel(m, L, C, X, T, STAGE_NONE);
      snap_store();
      forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    } else {
      forward_skip(m, L, C, X, T, STAGE_NONE, FD_NITER, 0.0);
    }
    forward_skip(m, L, C, X, T, STAGE_VEL, FD_NITER, 0.0);
    forward_skip(m, L, C, X, T, STAGE_VEL, FD_NITER, 0.0);
    wc = tid < nv ? warm[tid] : 0.0;
    costCenter = step_cost(m, a.cost, qpos, qvel, ctrl);
    if (tid < nv) st_sc1(cwp + tid, wc);
    if (tid == 0) st_sc1(cwp + nv, costCenter);
    drain_stores();
    TSYNC();
    if (tid == 0) signal_set(cflag, 1u);
  } else if (half >= 0) {
    // one evaluation of a column (a.halves): the + half also writes the cost
    // entry; both publish their qacc, and the second to finish forms the
    // column (qp - qm) / 2 eps and announces it on done[s,p]
    const int i = idx;
    const int col = role == 3 ? i : (role == 1 ? a.nut + i : a.nut + nv + i);
    const double sg = half ? -FD_EPS : FD_EPS;
    if (role == 3) {
      if (snap) snap_load();
      else forward_posvel(m, L, C, X, T, STAGE_NONE);
      get_centre();
      const double u0 = ctrl[i];
      TSYNC();
      if (tid == 0) {
        ctrl[i] = u0 + sg;
        if (!half) st_sc1(dr + G + 2 * nv + i, (step_cost(m, a.cost, qpos, qvel, ctrl) - costCenter) / FD_EPS);
      }
      set_warm();
      forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    } else if (role == 1) {
      if (snap) snap_load();
      const double v0 = qvel[i];
      TSYNC();
      if (tid == 0) qvel[i] = v0 + sg;
      forward_posvel(m, L, C, X, T, snap ? STAGE_POS : STAGE_NONE);
      get_centre();
      if (tid == 0 && !half) st_sc1(dr + G + nv + i, (step_cost(m, a.cost, qpos, qvel, ctrl) - costCenter) / FD_EPS);
      set_warm();
      forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    } else {
      const int jid = m.dof_jntid[i];
      int quatadr = -1, dofpos = 0;
      if (m.jnt_type[jid] == JNT_BALL) {
        quatadr = m.jnt_qposadr[jid];
        dofpos = i - m.jnt_dofadr[jid];
      } else if (m.jnt_type[jid] == JNT_FREE && i >= m.jnt_dofadr[jid] + 3) {
        quatadr = m.jnt_qposadr[jid] + 3;
        dofpos = i - m.jnt_dofadr[jid] - 3;
      }
      if (tid == 0) {
        if (quatadr >= 0) {
          double angvel[3] = {0, 0, 0}, q[4];
          angvel[dofpos] = sg;
          ldm<4>(q, qpos + quatadr);
          quat_integrate(q, angvel, 1);
          for (int k = 0; k < 4; k++) qpos[quatadr + k] = q[k];
        } else {
          qpos[m.jnt_qposadr[jid] + i - m.jnt_dofadr[jid]] += sg;
        }
      }
      forward_posvel(m, L, C, X, T, STAGE_NONE);
      get_centre();
      if (tid == 0 && !half) st_sc1(dr + G + i, (step_cost(m, a.cost, qpos, qvel, ctrl) - costCenter) / FD_EPS);
      set_warm();
      forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    }
    const double mine = tid < nv ? qacc[tid] : 0.0;
    double* xs = a.xq + ((size_t)pt * ntm + col) * 2 * nv;
    if (tid < nv) st_sc1(xs + half * nv + tid, mine);
    drain_stores();
    TSYNC();
    unsigned prior = 0;
    if (tid == 0) prior = __hip_atomic_fetch_add((gu32*)(a.pairc + (size_t)pt * ntm + col), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    prior = __builtin_amdgcn_readfirstlane(prior);
    if (prior == 1u) {
      const double other = tid < nv ? ld_sc1(xs + (1 - half) * nv + tid) : 0.0;
      const double qp = half ? other : mine, qm = half ? mine : other;
      const double dv = (qp - qm) / (2 * FD_EPS);
      if (tid < nv) {
        if (role == 3) st_sc1(dr + 2 * nv * nv + i + tid * nu, dv);
        else if (role == 1) st_sc1(dr + nv * nv + i + tid * nv, dv);
        else st_sc1(dr + i + tid * nv, dv);
      }
    } else {
      announce = false;
    }
  } else if (role == 3) {
    // ctrl column idx on its own position/velocity stages (ctrl enters only the
    // acceleration stage, so they equal the centre's)
    const int i = idx;
    if (snap) snap_load();
    else forward_posvel(m, L, C, X, T, STAGE_NONE);
    get_centre();
    const double u0 = ctrl[i];
    TSYNC();
    if (tid == 0) {
      ctrl[i] = u0 + FD_EPS;
      st_sc1(dr + G + 2 * nv + i, (step_cost(m, a.cost, qpos, qvel, ctrl) - costCenter) / FD_EPS);
    }
    set_warm();
    forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    const double qp = tid < nv ? qacc[tid] : 0.0;
    if (tid == 0) ctrl[i] = u0 - FD_EPS;
    set_warm();
    forward_skip(m, L, C, X, T, STAGE_VEL, FD_NITER, 0.0);
    if (tid < nv) st_sc1(dr + 2 * nv * nv + i + tid * nu, (qp - qacc[tid]) / (2 * FD_EPS));
  } else if (role == 1) {
    // qvel column idx: + side from a position stage of its own, - side reusing it
    const int i = idx;
    if (snap) snap_load();
    const double v0 = qvel[i];
    TSYNC();
    if (tid == 0) qvel[i] = v0 + FD_EPS;
    // its position stage is the centre's (qpos unchanged): from the snapshot
    forward_posvel(m, L, C, X, T, snap ? STAGE_POS : STAGE_NONE);
    get_centre();
    if (tid == 0) st_sc1(dr + G + nv + i, (step_cost(m, a.cost, qpos, qvel, ctrl) - costCenter) / FD_EPS);
    set_warm();
    forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    const double qp = tid < nv ? qacc[tid] : 0.0;
    if (tid == 0) qvel[i] = v0 - FD_EPS;
    set_warm();
    forward_skip(m, L, C, X, T, STAGE_POS, FD_NITER, 0.0);
    if (tid < nv) st_sc1(dr + nv * nv + i + tid * nv, (qp - qacc[tid]) / (2 * FD_EPS));
  } else {
    const int i = idx;
    const int jid = m.dof_jntid[i];
    int quatadr = -1, dofpos = 0;
    if (m.jnt_type[jid] == JNT_BALL) {
      quatadr = m.jnt_qposadr[jid];
      dofpos = i - m.jnt_dofadr[jid];
    } else if (m.jnt_type[jid] == JNT_FREE && i >= m.jnt_dofadr[jid] + 3) {
      quatadr = m.jnt_qposadr[jid] + 3;
      dofpos = i - m.jnt_dofadr[jid] - 3;
    }
    // qpos (-)/(+) eps along dof i: quaternion dofs by mju_quatIntegrate (mjderivative.cpp:151-168,186-191)
    auto perturb = [&](double e) {
      if (tid == 0) {
        if (quatadr >= 0) {
          double angvel[3] = {0, 0, 0}, q[4];
          angvel[dofpos] = e;
          ldm<4>(q, qpos + quatadr);
          quat_integrate(q, angvel, 1);
          for (int k = 0; k < 4; k++) qpos[quatadr + k] = q[k];
        } else {
          qpos[m.jnt_qposadr[jid] + i - m.jnt_dofadr[jid]] += e;
        }
      }
    };
    perturb(FD_EPS);
    forward_posvel(m, L, C, X, T, STAGE_NONE);
    get_centre();
    if (tid == 0) st_sc1(dr + G + i, (step_cost(m, a.cost, qpos, qvel, ctrl) - costCenter) / FD_EPS);
    set_warm();
    forward_acc(m, L, C, X, T, FD_NITER, 0.0);
    const double qp = tid < nv ? qacc[tid] : 0.0;
    FOR_T(k, nq) qpos[k] = dq[k];
    TSYNC();
    perturb(-FD_EPS);
    set_warm();
    forward_skip(m, L, C, X, T, STAGE_NONE, FD_NITER, 0.0);
    if (tid < nv) st_sc1(dr + i + tid * nv, (qp - qacc[tid]) / (2 * FD_EPS));
  }
  drain_stores();
  TSYNC();
  if (tid == 0 && announce) signal_add(done);
  if (a.dur && tid == 0) a.dur[u] = (unsigned)(__builtin_amdgcn_s_memrealtime() - tstart);
#ifdef ILQG_STAMPS
  if (tid == 0 && u < (unsigned)TL_N) g_tl[3 * u + 1] = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) atomicMax(&g_fused_diag[4], __builtin_amdgcn_s_memtime());
  if (tid == 0) coop::s_cnt[7] += __builtin_amdgcn_s_memtime() - tteam_;
#endif
  STAMP_FLUSH();
}

template <int NV, int NU, class MD>
__device__ inline void fd_backward_role(const MD& mg, const FdFused& a, int s) {
  extern __shared__ double lds[];
  // the serial Riccati chain shares its CU with sweep teams: it takes the
  // SIMD's issue arbitration (MI355X_MICROARCH.md "VALU issue is arbitrated
  // ... by priority, then age")
  if (ILQG_BW_PRIO) __builtin_amdgcn_s_setprio(3);
#ifdef ILQG_STAMPS
  const unsigned long long t0_ = __builtin_amdgcn_s_memtime();
  if (s == 0 && threadIdx.x == 0) g_fused_diag[3] = t0_;
  if (s < 64 && threadIdx.x == 0) g_tlb[2 * s] = __builtin_amdgcn_s_memrealtime();
#endif
  backward_seed<NV, NU>(mg, mg.nq, mg.nv, mg.nu, a.P, mg.opt_timestep, a.mu, a.deriv, a.Dp, a.tr, a.K, a.k, a.V,
                        a.v, s, threadIdx.x, lds, a.sync + 4 + (size_t)a.S * a.P, (unsigned)(1 + a.nut + 2 * a.nv),
                        a.fault, a.fl);
#ifdef ILQG_STAMPS
  if (s < 64 && threadIdx.x == 0) g_tlb[2 * s + 1] = __builtin_amdgcn_s_memrealtime();
  if (s < 16 && threadIdx.x == 0) g_fused_diag[8 + s] = __builtin_amdgcn_s_memtime() - t0_;
  if (s == 0 && threadIdx.x == 0) {
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();
    g_fused_diag[0] += t1_ - t0_;
    g_fused_diag[5] = t1_;
  }
#endif
}

__global__ __launch_bounds__(TEAM, FD_WAVES_PER_EU) void k_fd_fused_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, FdFused a) {
  const unsigned t = take_ticket(a.sync);
  if (t < (unsigned)a.nB) {
    fd_backward_role<0, 0>(mg, a, (int)t);
    return;
  }
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  fd_fused_body(m, L, C, X, T, a, t - a.nB);
}

// compile-time models: the model read from its global image (L1/L2 cached)
// rather than an LDS copy, so the team's LDS holds only the workspace (8 teams
// per CU for the hopper instead of 7)
template <class SM, class SX>
__global__ __launch_bounds__(TEAM, FD_WAVES_PER_EU) void k_fd_fused_g(DevModel mg, FdFused a) {
  const unsigned t = take_ticket(a.sync);
  if (t < (unsigned)a.nB) {
    fd_backward_role<SM::nv, SM::nu>(mg, a, (int)t);
    return;
  }
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  extern __shared__ double lds[];
  Team T = make_team(L, C);
  T.iw = reinterpret_cast<int*>(lds + L.nd + C.nd);  // no image region
  T.ci = T.iw + L.ni;
  SM m;
  m.bind(mg.img, mg);
  fd_fused_body(m, L, C, X, T, a, t - a.nB);
}

// ---- the fused sweep's ticket schedule (launch_fd_plan) -----------------
// One 1024-thread workgroup.  Items: centre C(s,p) = p S + s (u < S P), column
// w of (s,p) = S P + (p S + s) ntm + w (fd_decode's identity order).  Groups g =
// p S + s with p >= p0 are dealt to threads in contiguous runs of G_RUN; three
// exclusive scans over the groups place section B (long groups: centre + long
// columns), section C1 (the other centres) and C2 (the other columns).
constexpr int PLAN_T = 1024;
__device__ inline unsigned block_excl_scan(unsigned v, unsigned* sh, unsigned& total) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
  for (int off = 1; off < PLAN_T; off <<= 1) {
    const unsigned x = t >= off ? sh[t - off] : 0u;
    __syncthreads();
    sh[t] += x;
    __syncthreads();
  }
  total = sh[PLAN_T - 1];
  const unsigned incl = sh[t];
  __syncthreads();
  return incl - v;
}

__global__ __launch_bounds__(PLAN_T) void k_fd_plan(int S, int P, int ntm, int p0, float kthr, const unsigned* dur,
                                                    unsigned* order) {
  __shared__ unsigned sh[PLAN_T];
  __shared__ unsigned long long sum_sh;
  const int t = threadIdx.x;
  const unsigned nC = (unsigned)S * P, nI = nC * (1 + ntm);
  if (p0 > P) p0 = P;
  if (t == 0) sum_sh = 0;
  __syncthreads();
  unsigned long long part = 0;
  for (unsigned u = t; u < nI; u += PLAN_T) part += dur[u];
  atomicAdd(&sum_sh, part);
  __syncthreads();
  const unsigned long long sum = sum_sh;
  if (sum == 0) {  // no history: identity
    for (unsigned u = t; u < nI; u += PLAN_T) order[u] = u;
    return;
  }
  const double thr = (double)kthr * (double)sum / (double)nI;
  // section A: the first p0 points keep their identity slots
  const unsigned nA_c = (unsigned)p0 * S, nA_w = nA_c * ntm;
  for (unsigned u = t; u < nA_c; u += PLAN_T) order[u] = u;
  for (unsigned j = t; j < nA_w; j += PLAN_T) order[nA_c + j] = nC + j;
  // groups g0 .. nC-1, G_RUN consecutive per thread
  const unsigned g0 = nA_c, ng = nC - g0, run = (ng + PLAN_T - 1) / PLAN_T;
  const unsigned ga = g0 + min(ng, t * run), gb = g0 + min(ng, (t + 1) * run);
  auto is_long = [&](unsigned u) { return (double)dur[u] > thr; };
  auto col = [&](unsigned g, int w) { return nC + g * ntm + (unsigned)w; };
  unsigned cB = 0, cC1 = 0, cC2 = 0;
  for (unsigned g = ga; g < gb; g++) {
    int nl = 0;
    for (int w = 0; w < ntm; w++) nl += is_long(col(g, w));
    const bool lg = nl > 0 || is_long(g);
    cB += lg ? 1 + nl : 0;
    cC1 += lg ? 0 : 1;
    cC2 += ntm - nl;
  }
  unsigned tB, tC1, tC2;
  unsigned oB = block_excl_scan(cB, sh, tB);
  unsigned oC1 = block_excl_scan(cC1, sh, tC1);
  unsigned oC2 = block_excl_scan(cC2, sh, tC2);
  const unsigned baseB = nA_c + nA_w, baseC1 = baseB + tB, baseC2 = baseC1 + tC1;
  for (unsigned g = ga; g < gb; g++) {
    int nl = 0;
    for (int w = 0; w < ntm; w++) nl += is_long(col(g, w));
    const bool lg = nl > 0 || is_long(g);
    if (lg) {
      order[baseB + oB++] = g;
      for (int w = 0; w < ntm; w++)
        if (is_long(col(g, w))) order[baseB + oB++] = col(g, w);
    } else {
      order[baseC1 + oC1++] = g;
    }
    for (int w = 0; w < ntm; w++)
      if (!is_long(col(g, w))) order[baseC2 + oC2++] = col(g, w);
  }
}

// ---- schedule validation (launch_fd_order_check) -------------------------
// The fused sweep trusts its ticket -> item map twice: an item id out of range
// would address records and hand-off words past their buffers, and a map that
// is not a permutation with every column behind its centre could let a team
// wait on work holding a larger ticket, or announce a record before a missing
// column is written.  One 1024-thread workgroup checks, before the sweep reads
// it: every entry < nI, no item twice (so, by counting, a permutation), and
// slot(centre(s,p)) < slot(column) for every column item.  On failure it sets
// bit 1 of the fault report word (ilqg_synchronize reports it once) and
// rewrites the map as the identity, which satisfies all three, so the sweep
// still runs and its records are the same bits.  pos: nI words of scratch,
// preset to ~0 on the stream.
__global__ __launch_bounds__(PLAN_T) void k_fd_order_check(unsigned nC, unsigned nt, unsigned* order, unsigned* pos,
                                                           unsigned* fault) {
  __shared__ int bad_sh;
  const int t = threadIdx.x;
  const unsigned nI = nC * (1 + nt);
  if (t == 0) bad_sh = 0;
  __syncthreads();
  int bad = 0;
  for (unsigned u = t; u < nI; u += PLAN_T) {
    const unsigned v = order[u];
    if (v >= nI) bad = 1;
    else if (atomicExch(&pos[v], u) != ~0u) bad = 1;
  }
  if (bad) atomicOr(&bad_sh, 1);
  __threadfence_block();
  __syncthreads();
  if (!bad_sh) {
    for (unsigned v = nC + t; v < nI; v += PLAN_T)
      if (pos[(v - nC) / nt] >= pos[v]) bad = 1;
    if (bad) atomicOr(&bad_sh, 1);
    __syncthreads();
  }
  if (bad_sh) {
    for (unsigned u = t; u < nI; u += PLAN_T) order[u] = u;
    if (t == 0) atomicOr(fault, 2u);
  }
}

}  // namespace

hipError_t launch_fd_plan(int S, int P, int ntm, int p0, float kthr, const unsigned* dur, unsigned* order,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_fd_plan, dim3(1), dim3(PLAN_T), 0, st, S, P, ntm, p0, kthr, dur, order);
  return hipGetLastError();
}
hipError_t launch_fd_order_check(int S, int P, int nt, unsigned* order, unsigned* pos, unsigned* fault,
                                 hipStream_t st) {
  const unsigned nC = (unsigned)S * (unsigned)P;
  hipError_t e = hipMemsetAsync(pos, 0xff, (size_t)nC * (1 + nt) * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fd_order_check, dim3(1), dim3(PLAN_T), 0, st, nC, (unsigned)nt, order, pos, fault);
  return hipGetLastError();
}

size_t coop_lds_bytes(const WsLayout& L, const CoopLayout& C) {
  return (size_t)(L.nd + C.nd + C.imgd) * sizeof(double) + (size_t)(L.ni + C.ni) * sizeof(int);
}
hipError_t launch_fd_centre_coop(const DevModel& m, const WsLayout& L, const CoopLayout& C, const CoopAux& X,
                                 TrajDev tr, int npts, int P, const double* qfrc_applied, const double* xfrc_applied,
                                 CostDev cost, double* warm_c, double* cost_c, hipStream_t st) {
  if (npts <= 0) return hipSuccess;
  const size_t lds = coop_lds_bytes(L, C);
  hipError_t e;
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id:                                                                                                      \
    e = allow_lds(k_fd_centre_s<stat::SMT, stat::SXT>, lds);                                                    \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_fd_centre_s<stat::SMT, stat::SXT>), dim3(npts), dim3(TEAM), lds, st, m, tr, P,         \
                       qfrc_applied, xfrc_applied, cost, warm_c, cost_c);                                       \
    return hipGetLastError();
  switch (m.static_id) {
    ILQG_STATIC_MODELS(ILQG_CASE)
    default:
      break;
  }
#undef ILQG_CASE
  e = allow_lds(k_fd_centre_coop, coop_lds_bytes(L, C));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fd_centre_coop, dim3(npts), dim3(TEAM), coop_lds_bytes(L, C), st, m, L, C, X, tr, P,
                     qfrc_applied, xfrc_applied, cost, warm_c, cost_c);
  return hipGetLastError();
}

hipError_t launch_fd_cols_coop(const DevModel& m, const WsLayout& L, const CoopLayout& C, const CoopAux& X,
                               TrajDev tr, int npts, int P, const double* qfrc_applied, const double* xfrc_applied,
                               CostDev cost, const double* warm_c, const double* cost_c, double* deriv, int Ds,
                               hipStream_t st) {
  const int nctrl = m.nu < m.nv ? m.nu : m.nv;
  const long blocks = (long)npts * (nctrl + 2 * m.nv);
  if (blocks <= 0) return hipSuccess;
  const size_t lds = coop_lds_bytes(L, C);
  hipError_t e;
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id:                                                                                                      \
    e = allow_lds(k_fd_cols_s<stat::SMT, stat::SXT>, lds);                                                      \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_fd_cols_s<stat::SMT, stat::SXT>), dim3((unsigned)blocks), dim3(TEAM), lds, st, m, tr,  \
                       P, qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv, Ds);                         \
    return hipGetLastError();
  switch (m.static_id) {
    ILQG_STATIC_MODELS(ILQG_CASE)
    default:
      break;
  }
#undef ILQG_CASE
  e = allow_lds(k_fd_cols_coop, coop_lds_bytes(L, C));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fd_cols_coop, dim3((unsigned)blocks), dim3(TEAM), coop_lds_bytes(L, C), st, m, L, C, X, tr, P,
                     qfrc_applied, xfrc_applied, cost, warm_c, cost_c, deriv, Ds);
  return hipGetLastError();
}

hipError_t launch_fd_fused_coop(const DevModel& m, const WsLayout& L, const CoopLayout& C, const CoopAux& X,
                                const FdFused& a, hipStream_t st) {
  const long items = (long)a.S * a.P * (1 + (a.halves ? 2 : 1) * (a.nut + 2 * m.nv));
  const long blocks = items + a.nB;
  if (items <= 0) return hipSuccess;
  size_t lds = coop_lds_bytes(L, C);
  if (a.nB > 0) lds = std::max(lds, backward_lds_bytes(m.nv, m.nu));
  hipError_t e;
  const size_t lds_g = std::max((size_t)(L.nd + C.nd) * sizeof(double) + (size_t)(L.ni + C.ni) * sizeof(int),
                                a.nB > 0 ? backward_lds_bytes(m.nv, m.nu) : (size_t)0);
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id:                                                                                                      \
    e = allow_lds(k_fd_fused_g<stat::SMT, stat::SXT>, lds_g);                                                   \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_fd_fused_g<stat::SMT, stat::SXT>), dim3((unsigned)blocks), dim3(TEAM), lds_g, st, m, a); \
    return hipGetLastError();
  switch (m.static_id) {
    ILQG_STATIC_MODELS(ILQG_CASE)
    default:
      break;
  }
#undef ILQG_CASE
  e = allow_lds(k_fd_fused_coop, lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fd_fused_coop, dim3((unsigned)blocks), dim3(TEAM), lds, st, m, L, C, X, a);
  return hipGetLastError();
}

}  // namespace ilqg

#ifdef ILQG_STAMPS
// the fused sweep's timeline (g_tl: 3 words per FD item, then g_tlb: 2 per role)
extern "C" int ilqg_debug_timeline(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ilqg::g_tl), sizeof(unsigned long long) * 3 * ilqg::TL_N) != hipSuccess)
    return 3;
  if (hipMemcpyFromSymbol(out + 3 * ilqg::TL_N, HIP_SYMBOL(ilqg::g_tlb), sizeof(unsigned long long) * 128) !=
      hipSuccess)
    return 3;
  // then the backward roles' per-step completion times (handoff.h g_bstep)
  if (hipMemcpyFromSymbol(out + 3 * ilqg::TL_N + 128, HIP_SYMBOL(ilqg::g_bstep), sizeof(unsigned long long) * 8 * 512) !=
      hipSuccess)
    return 3;
  if (reset) {
    static unsigned long long z[3 * ilqg::TL_N];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_tl), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_tlb), z, sizeof(unsigned long long) * 128);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_bstep), z, sizeof(unsigned long long) * 8 * 512);
  }
  return 0;
}
extern "C" int ilqg_debug_fused(unsigned long long* d, int reset) {
  if (hipMemcpyFromSymbol(d, HIP_SYMBOL(ilqg::g_fused_diag), sizeof(unsigned long long) * 24) != hipSuccess) return 3;
  if (reset) {
    unsigned long long z[24] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::g_fused_diag), z, sizeof(z));
  }
  return 0;
}
#endif

#ifdef ILQG_STAMPS
// the FD kernels' line-search counters (dcoop_impl.h g_ls)
extern "C" int ilqg_debug_ls_fd(unsigned long long* out5, int reset) {
  if (hipMemcpyFromSymbol(out5, HIP_SYMBOL(ilqg::coop::g_ls), sizeof(unsigned long long) * 8) != hipSuccess) return 3;
  if (reset) {
    unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_ls), z, sizeof(z));
  }
  return 0;
}
// the FD kernels' copy of the stamp counters (tools/stamps.py)
extern "C" int ilqg_debug_stamps_fd(unsigned long long* acc, unsigned long long* cnt, int reset) {
  if (hipMemcpyFromSymbol(acc, HIP_SYMBOL(ilqg::coop::g_stamp_acc), sizeof(unsigned long long) * STAMP_NG) != hipSuccess)
    return 3;
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(ilqg::coop::g_stamp_cnt), sizeof(unsigned long long) * STAMP_NG) != hipSuccess)
    return 3;
  unsigned long long nw[2];
  (void)hipMemcpyFromSymbol(&nw[0], HIP_SYMBOL(ilqg::coop::g_newton_iters), 8);
  (void)hipMemcpyFromSymbol(&nw[1], HIP_SYMBOL(ilqg::coop::g_newton_calls), 8);
  acc[44] = nw[0];
  acc[45] = nw[1];
  if (reset) {
    unsigned long long z[STAMP_NG] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_newton_iters), z, 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_newton_calls), z, 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_stamp_acc), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_stamp_cnt), z, sizeof(z));
  }
  return 0;
}
#endif
