// Launch interface of the hot-path kernels (kernels_rollout.hip, kernels_fd.hip, riccati.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "dmodel.h"

namespace ilqg {

// trajectory / state arrays on the device, [point][field]
struct TrajDev {
  double* time;
  double* qpos;
  double* qvel;
  double* warm;
  double* ctrl;
};

// a rollout launch over points n_hi .. n_lo (descending) of the horizon: the
// whole trajectory (n_hi < 0, the default), or one chunk of a chunked rollout
// whose FD sweep runs behind it (ilqg_iterate's pipelined path).  A chunk that
// does not start at point P-1 takes its state from carry[candidate] and adds
// to the candidate's cost already in cost_cand; one that does not end at
// point 0 leaves its state in carry[candidate].
struct RollChunk {
  TrajDev carry{};
  int n_hi = -1, n_lo = 0;
  // set by launch_rollout_coop (two-wave generic kernel): the nominal record
  // double-buffered in LDS past the team's workspace, the next point's copied
  // by the helper wave while the primary runs the constraint solve
  int dbuf = 0;
};

// device cost descriptor (all 9 arrays present, zero where unused)
struct CostDev {
  const double *wq, *tq, *lq, *wv, *tv, *lv, *wu, *tu, *lu;
};

// How the Riccati recursion reads an FD record (ilqg_solver_set_layout).
// The record is always the reference's (row-major by output, mjderivative.cpp:
// 107,138,202).  REFERENCE: A's lower blocks and B are Eigen column-major maps
// of those row-major blocks (differentiator.h:57-59,89-92, quirk Q1: dt J^T,
// and a permuted dt J_u for nu > 1).  CORRECTED: the true Jacobians, dt J and
// dt J_u.  The recursion stages entry e of a record from record index
// rec_src(e): identity in the reference layout, the three Jacobian blocks
// transposed in the corrected one.
struct RicFlags {
  int layout;  // 0 reference, 1 corrected
  int vinit;   // 1: V0 / v0 are read from V / v instead of initV's (inc/ilqr.h:100-107)
  int ldlt_lds = 0;  // k_backward_mfma<27, 21>: 1 the LDS-resident LDLT instead of ldlt_factor_reg_t, 2 its pivot replay forced (ILQG_LDLT_REG)
};
__host__ __device__ inline int rec_src(int e, int nv, int nu, int layout) {
  if (!layout) return e;
  const int nn = nv * nv;
  if (e < 2 * nn) {  // A block b (0 qpos, 1 qvel): staged (r + c nv) <- record (c + r nv)
    const int b = e >= nn, f = e - b * nn, r = f % nv, c = f / nv;
    return b * nn + c + r * nv;
  }
  if (e < 2 * nn + nv * nu) {  // B: staged (r + a nv) <- record (a + r nu)
    const int f = e - 2 * nn, r = f % nv, a = f / nv;
    return 2 * nn + a + r * nu;
  }
  return e;  // cost gradients
}

// candidate selection + setDInit(dArray[N])
hipError_t launch_selftest_div(const double* a, const double* b, double* q, double* q2, int n, hipStream_t st);
hipError_t launch_select(const DevModel& m, int S, int A, int P, int mode, int copy_cand, const double* cost_cand,
                         int* sel, double* cost_sel, TrajDev cand, TrajDev nominal, TrajDev dinit, hipStream_t st);
// Riccati backward pass, one workgroup per seed
// deriv records at stride Ds (>= D) doubles
hipError_t launch_backward(const DevModel& m, int S, int P, double mu, const double* deriv, int Ds, TrajDev tr,
                           double* K, double* k, double* V, double* v, RicFlags fl, hipStream_t st);
size_t backward_lds_bytes(int nv, int nu);
// the same recursion with the matrix products on the fp64 matrix cores
// (riccati_mfma.h): one 8-wave workgroup per seed; agrees with the oracle to
// rounding (the product sums run in the matrix core's order)
hipError_t launch_backward_mfma(const DevModel& m, int S, int P, double mu, const double* deriv, int Ds, TrajDev tr,
                                double* K, double* k, double* V, double* v, RicFlags fl, hipStream_t st);
size_t backward_mfma_lds_bytes(int nv, int nu);
bool backward_mfma_supported(int nv, int nu);

// fused FD sweep + streamed backward pass (kernels_fd.hip)
struct FdFused {
  TrajDev tr;
  int S, P;
  int nB;        // backward roles (S, or 0 for the sweep alone)
  int nv;        // qvel and qpos teams per point (one column each)
  int nut;       // ctrl teams per point, min(nu, nv) (mjderivative.cpp:78-82)
  int Dp, WCp;   // padded record strides (doubles, multiples of 16 = 128 B)
  const double* qfrc_applied;
  const double* xfrc_applied;
  CostDev cost;
  double* cw;      // [S*P][WCp]: centre warm start (nv) + centre cost
  double* deriv;   // [S*P][Dp]
  unsigned* sync;  // [4 + 2 S P]: ticket, pad, cflag[S*P], done[S*P]; zeroed before each launch
  unsigned* fault; // set by a timed-out wait
  double mu;
  double *K, *k, *V, *v;
  RicFlags fl;
  // ticket schedule (launch_fd_plan): slot -> FD item, null = identity; each
  // FD item's duration in this launch (s_memrealtime ticks), null = not kept
  const unsigned* order;
  unsigned* dur;
  // issue priority of the FD teams by ticket slot: slots >= prio1 run at
  // s_setprio 1, >= prio2 at 2 (the backward roles run at 3); ~0u = never
  unsigned prio1 = ~0u, prio2 = ~0u;
  // the centre team's workspace after its position and velocity stages, per
  // point ([S*P][snapd] doubles: the team's LDS ints, then the doubles the
  // column teams read, kernels_fd.hip snap_ranges), which the qvel and ctrl
  // teams load instead of recomputing those stages; null = every team
  // computes its own
  double* snap = nullptr;
  int snapd = 0;
  int poison = 0;  // tests (ILQG_SNAP_POISON): every double a snapshot does not carry reads as NaN
  // every column as two items, its + and - evaluations ([S*P][ntm][2][nv]
  // qacc exchange, [S*P][ntm] pair counters zeroed with sync); 0 = one item
  int halves = 0;
  double* xq = nullptr;
  unsigned* pairc = nullptr;
};
// Plan the fused sweep's ticket order from the previous launch's per-item
// durations (dur, all zero = no history: identity order).  Items of the first
// p0 points keep their slots; then, point-major, every (seed, point) with an
// item longer than kthr x the mean duration: its centre team and its long
// column teams; then the rest in identity order.  Every column team still
// follows its centre team, so the deadlock argument is unchanged.
hipError_t launch_fd_plan(int S, int P, int ntm, int p0, float kthr, const unsigned* dur, unsigned* order,
                          hipStream_t st);
// validates a ticket -> item map (nt items per (seed, point) besides its
// centre); replaces an invalid one by the identity and sets fault bit 1
hipError_t launch_fd_order_check(int S, int P, int nt, unsigned* order, unsigned* pos, unsigned* fault,
                                 hipStream_t st);

}  // namespace ilqg

// ---- cooperative (one wavefront per evaluation, LDS workspace) variants ----
namespace ilqg {
size_t coop_lds_bytes(const WsLayout& L, const coop::CoopLayout& C);
hipError_t launch_fd_centre_coop(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                                 const coop::CoopAux& X, TrajDev tr, int npts, int P, const double* qfrc_applied,
                                 const double* xfrc_applied, CostDev cost, double* warm_c, double* cost_c,
                                 hipStream_t st);
hipError_t launch_fd_cols_coop(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                               const coop::CoopAux& X, TrajDev tr, int npts, int P, const double* qfrc_applied,
                               const double* xfrc_applied, CostDev cost, const double* warm_c, const double* cost_c,
                               double* deriv, int Ds, hipStream_t st);
// fp32 FD sweep (kernels_fd32.hip; BASELINE.json configs[4]): centre + column
// kernels on the fp32 physics, fp64 records; eps is the FD step (1e-3)
size_t coop_lds_bytes_f32(const WsLayout& L, const coop::CoopLayout& C);
hipError_t launch_fd_sweep_f32(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                               const coop::CoopAux& X, TrajDev tr, int npts, int P, const double* qfrc_applied,
                               const double* xfrc_applied, CostDev cost, double* warm_c, double* cost_c,
                               double* deriv, int Ds, double eps, hipStream_t st);
hipError_t launch_fd_fused_coop(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                                const coop::CoopAux& X, const FdFused& a, hipStream_t st);
hipError_t launch_rollout_coop(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                               const coop::CoopAux& X, int S, int A, int P, TrajDev nominal, TrajDev out,
                               int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit,
                               const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost,
                               double* cost_cand, hipStream_t st, RollChunk ch = RollChunk{});
// n independent states, one wavefront each: nstep mj_step (in place)
hipError_t launch_step_coop(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C, const coop::CoopAux& X,
                            TrajDev stt, int n, int nstep, const double* qfrc_applied, const double* xfrc_applied,
                            hipStream_t st);
// n independent states, one wavefront each: mj_forward -> qacc, warm start updated
hipError_t launch_forward_coop(const DevModel& m, const WsLayout& L, const coop::CoopLayout& C,
                               const coop::CoopAux& X, TrajDev stt, int n, const double* qfrc_applied,
                               const double* xfrc_applied, double* qacc, hipStream_t st);
}  // namespace ilqg
