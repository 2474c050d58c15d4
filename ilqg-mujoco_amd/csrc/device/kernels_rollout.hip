// Cooperative rollout kernels (inc/ilqr.h:116-130): one workgroup per
// (seed, alpha) candidate; two-wave teams (step_dual) by default.
//
// The rollout's Newton solves use the model's tolerance, and their line
// searches take ~1.4 iterations: the uniform-row line search (dcoop_impl.h
// ls_iterate_rows, for the FD sweep's tolerance-0 solves) does not pay here,
// and its code grew the hopper rollout kernel from 240 to 299 KB, slowing
// every stage (instruction cache): this translation unit keeps the lane form
// for the iterations of the generic solver, and runs the compile-time models'
// line searches (eval(0) included) on rows padded to 4 or 8 (linesearch_u).
#ifndef ILQG_LS_NE
#define ILQG_LS_NE 0
#endif
#ifndef ILQG_LS_U
#define ILQG_LS_U 1
#endif
// (~1.4 iterations per line search: the speculative bisection tree does not pay)
#ifndef ILQG_LS_TREE
#define ILQG_LS_TREE 0
#endif
#include "coop_common.h"

namespace ilqg {
namespace {

__device__ inline void rollout_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand, RollChunk ch, int wave, auto split, auto lowreg) {
  // wave < 0: one-wave team; 0/1: primary/helper wave of a two-wave team (step_dual)
  const bool prim = wave <= 0;
  STAMP_INIT();
#ifdef ILQG_STAMPS
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
#endif
  const int lane = blockIdx.x;
  const int s = lane / A, a = lane % A;
  const int nq = m.nq, nv = m.nv, nu = m.nu, nx = 2 * nv;
  // the points this launch rolls over (RollChunk): n_hi .. n_lo, descending
  const int nhi = ch.n_hi >= 0 ? ch.n_hi : P - 1, nlo = ch.n_hi >= 0 ? ch.n_lo : 0;
  const bool resume = nhi < P - 1;
  if (resume) load_state(m, L, T, ch.carry, lane, s, qfrc_applied, xfrc_applied);
  else load_state(m, L, T, dinit, s, s, qfrc_applied, xfrc_applied);
  const CostDev cl = stage_cost(m, C, T, cost);
  double* qpos = T.w + L.qpos;
  double* qvel = T.w + L.qvel;
  double* ctrl = T.w + L.ctrl;
  double* warm = T.w + L.warm;
  double* dx = T.w + L.s_fd;
  // per-point record of the nominal trajectory and gains, [x*_q | x*_v | u* | K | k],
  // prefetched one point ahead into registers and parked in LDS (C.rec)
  double* rec = T.c + C.rec;
  const int R = nq + nv + nu + nu * nx + nu;
  // ch.dbuf (generic two-wave kernel): point n's record in buffer (nhi - n) & 1,
  // the second one past the team's LDS (launch_rollout_coop sized the launch)
  double* rec2 = rec;
  if (ch.dbuf) {
    extern __shared__ double lds[];
    const size_t off = ((size_t)(L.nd + C.nd + C.imgd) * 8 + (size_t)(L.ni + C.ni) * 4 + 15) / 16 * 16;
    rec2 = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + off);
  }
  auto recp = [&](int n) -> double* { return ((nhi - n) & 1) ? rec2 : rec; };
  auto fetch = [&](size_t pn, int t) -> double {
    if (t < nq) return nom.qpos[pn * nq + t];
    t -= nq;
    if (t < nv) return nom.qvel[pn * nv + t];
    t -= nv;
    if (t < nu) return nom.ctrl[pn * nu + t];
    t -= nu;
    if (t < nu * nx) return K[pn * nu * nx + t];
    return k[pn * nu + t - nu * nx];
  };
  // registers per lane: R <= PFR * 64.  The run-time (generic) models take
  // records up to 20 * 64 doubles (the humanoid's is 1231: K alone is
  // nu x 2nv = 1134) in flight a step ahead as well
  using MT = std::remove_cvref_t<decltype(m)>;
  // (lowreg: the two-wave generic kernel, whose record is double-buffered in LDS
  // instead -- 20 prefetch registers spilled to scratch there, a 512-register kernel)
  constexpr int PFR = StaticModel<MT> ? 4 : (decltype(lowreg)::value ? 1 : 20);
  double pf[PFR];
  // larger records are not prefetched: park() copies them from global memory directly
  const bool pfok = R <= PFR * TEAM_SIZE;
  if (!passive) {
    FOR_T(t, R) rec[t] = fetch((size_t)s * P + nhi, t);
    TSYNC();
  }
  const double alpha = alphas ? alphas[a] : 1.0;
  const int ob = out_is_cand ? lane : s;
  // the wave that runs the control law and writes the record: the helper wave
  // of a two-wave team (beside the primary's kinematics), else the only wave
  const bool ctl = wave < 0 || wave == 1;
  double c = 0;
  if (resume && ctl && T.tid == 0 && cost_cand) c = cost_cand[lane];
  // control law u = u* + alpha k + K (x - x*) for point n, its record and cost
  // (ilqr.h:116-133); the next point's nominal record is prefetched first
  auto pre_step = [&](int n) {
    const double* rq = recp(n);
    const double* rv = rq + nq;
    const double* ru = rq + nq + nv;
    const double* rK = ru + nu;
    const double* rk = rK + nu * nx;
    const bool pre = !passive && n > 0 && pfok && !ch.dbuf;
    if (pre) {
      const size_t pn1 = (size_t)s * P + (n - 1);
#pragma unroll
      for (int q = 0; q < PFR; q++) {
        const int t = T.tid + q * TEAM_SIZE;
        pf[q] = t < R ? fetch(pn1, t) : 0.0;
      }
    }
    if (!passive) {
      FOR_T(j, nx) dx[j] = j < nv ? state_diff_dof(m, j, qpos, rq) : qvel[j - nv] - rv[j - nv];
      TSYNC();
      FOR_T(i, nu) {
        double t = 0;
        int j = 0;
        if constexpr (!StaticModel<MT>) {
          // run-time nx: eight terms' loads in flight at once, additions in order
          for (; j + 8 <= nx; j += 8) {
            double kk[8], xx[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
              kk[q] = rK[i + (j + q) * nu];
              xx[q] = dx[j + q];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) t += kk[q] * xx[q];
          }
        }
        for (; j < nx; j++) t += rK[i + j * nu] * dx[j];
        ctrl[i] = (t + alpha * rk[i]) + ru[i];
      }
      TSYNC();
    }
    const size_t po = (size_t)ob * P + n;
    FOR_T(i, nq) out.qpos[po * nq + i] = qpos[i];
    FOR_T(i, nv) {
      out.qvel[po * nv + i] = qvel[i];
      out.warm[po * nv + i] = warm[i];
    }
    FOR_T(i, nu) out.ctrl[po * nu + i] = ctrl[i];
    if (T.tid == 0) {
      out.time[po] = T.w[L.time];
      c += step_cost(m, cl, qpos, qvel, ctrl);
    }
    TSYNC();
  };
  // the prefetched record replaces the current one once the step no longer reads it
  auto park = [&](int n) {
    if (!passive && n > 0 && !ch.dbuf) {
      if (pfok) {
#pragma unroll
        for (int q = 0; q < PFR; q++) {
          const int t = T.tid + q * TEAM_SIZE;
          if (t < R) rec[t] = pf[q];
        }
      } else {
        FOR_T(t, R) rec[t] = fetch((size_t)s * P + (n - 1), t);
      }
      TSYNC();
    }
  };
  if (wave >= 0) {
    // the step ids of the two-wave hand-off flags (step_dual_split) start above 0
    if (threadIdx.x == 0)
      T.ci[C.ibc + 1] = T.ci[C.ibc + 2] = T.ci[C.ibc + 3] = T.ci[C.ibc + 4] = T.ci[C.ibc + 6] = T.ci[C.ibc + 7] = 0;
    __syncthreads();
  }
  for (int n = nhi; n >= nlo; n--) {
    if (wave < 0) {
      pre_step(n);
      step(m, L, C, X, T);
      park(n);
    } else {
      // split layout (compile-time models): the rebalanced three-wave
      // schedule, which parks the record in a later phase
      if constexpr (decltype(split)::value) {
        step_dual_split(m, L, C, X, T, wave, P - n, [&]() { pre_step(n); }, [&]() { park(n); });
      } else {
        step_dual(
            m, L, C, X, T, wave,
            [&]() {
              pre_step(n);
              park(n);
            },
            [&]() {
              // the next point's record into the other buffer (ch.dbuf)
              if (ch.dbuf && !passive && n > 0) {
                double* dst = recp(n - 1);
                const size_t pn1 = (size_t)s * P + (n - 1);
                for (int t0 = T.tid; t0 < R; t0 += 4 * TEAM_SIZE) {
                  double v[4];
#pragma unroll
                  for (int q = 0; q < 4; q++) {
                    const int t = t0 + q * TEAM_SIZE;
                    v[q] = t < R ? fetch(pn1, t) : 0.0;
                  }
#pragma unroll
                  for (int q = 0; q < 4; q++)
                    if (t0 + q * TEAM_SIZE < R) dst[t0 + q * TEAM_SIZE] = v[q];
                }
              }
            });
      }
    }
  }
  if (ctl && T.tid == 0 && cost_cand) cost_cand[lane] = c;
  if (nlo > 0) {
    // the state the next chunk starts from (point nlo - 1, before its control)
    if (wave >= 0) __syncthreads();
    if (prim) {
      FOR_T(i, nq) ch.carry.qpos[(size_t)lane * nq + i] = qpos[i];
      FOR_T(i, nv) {
        ch.carry.qvel[(size_t)lane * nv + i] = qvel[i];
        ch.carry.warm[(size_t)lane * nv + i] = warm[i];
      }
      FOR_T(i, nu) ch.carry.ctrl[(size_t)lane * nu + i] = ctrl[i];
      if (T.tid == 0) ch.carry.time[lane] = T.w[L.time];
    }
  }
#ifdef ILQG_STAMPS
  if (prim && T.tid == 0 && blockIdx.x == 0) {
    g_stamp_acc[46] += __builtin_amdgcn_s_memrealtime() - rt0;
    g_stamp_acc[47] += __builtin_amdgcn_s_memtime() - mt0;
  }
#endif
  STAMP_FLUSH();
}

__global__ __launch_bounds__(TEAM) void k_rollout_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand, RollChunk ch) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand, ch, -1, std::false_type{}, std::false_type{});
}

// model-specific instance (static_models.h): compile-time sizes, tables and LDS layout
template <class SM, class SX>
__global__ __launch_bounds__(TEAM) void k_rollout_s(DevModel mg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand, RollChunk ch) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_sep(mg, T, m);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand, ch, -1, std::false_type{}, std::false_type{});
}

// two-wave teams (step_dual): 128 threads per (seed, candidate).  MT: DevModel,
// or DevModelNV<27> for 27-dof models (the humanoid: compile-time sizes in the
// Newton Cholesky and its substitution)
template <class MT>
__global__ __launch_bounds__(2 * TEAM) void k_rollout2_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand, RollChunk ch) {
  Team T = make_team(L, C);
  MT m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied,
               passive, cost, cost_cand, ch, (int)(threadIdx.x / TEAM), std::false_type{}, std::true_type{});
}
// three-wave teams for the compile-time register-row models (step_dual_split),
// two-wave otherwise
template <class SM>
constexpr int rollout_waves() { return SM::nv <= RMAX ? 3 : 2; }
template <class SM, class SX>
__global__ __launch_bounds__(3 * TEAM) void k_rollout2_s(DevModel mg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand, RollChunk ch) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair, true);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_sep(mg, T, m);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied,
               passive, cost, cost_cand, ch, (int)(threadIdx.x / TEAM), std::bool_constant<SM::nv <= RMAX>{},
               std::false_type{});
}

// ---- batch physics (ilqg_step_batch / ilqg_forward_batch): one wavefront per state
// mj_step x nstep from each state (cpMjData in, the state out)
__device__ inline void step_batch_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                       TrajDev stt, int nstep, const double* qfrc_applied, const double* xfrc_applied) {
  const int i = blockIdx.x;
  load_state(m, L, T, stt, i, i, qfrc_applied, xfrc_applied);
  for (int t = 0; t < nstep; t++) step(m, L, C, X, T);
  if (T.tid == 0) stt.time[i] = T.w[L.time];
  FOR_T(k, m.nq) stt.qpos[(size_t)i * m.nq + k] = T.w[L.qpos + k];
  FOR_T(k, m.nv) {
    stt.qvel[(size_t)i * m.nv + k] = T.w[L.qvel + k];
    stt.warm[(size_t)i * m.nv + k] = T.w[L.warm + k];
  }
}
// mj_forward at each state: qacc out, qacc_warmstart updated in place
__device__ inline void fwd_batch_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                      TrajDev stt, const double* qfrc_applied, const double* xfrc_applied,
                                      double* qacc) {
  const int i = blockIdx.x;
  load_state(m, L, T, stt, i, i, qfrc_applied, xfrc_applied);
  forward_skip(m, L, C, X, T, STAGE_NONE, m.opt_iterations, m.opt_tolerance);
  FOR_T(k, m.nv) {
    qacc[(size_t)i * m.nv + k] = T.w[L.qacc + k];
    stt.warm[(size_t)i * m.nv + k] = T.w[L.warm + k];
  }
}
__global__ __launch_bounds__(TEAM) void k_step_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, TrajDev stt,
                                                    int nstep, const double* qfrc_applied, const double* xfrc_applied) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  step_batch_body(m, L, C, X, T, stt, nstep, qfrc_applied, xfrc_applied);
}
template <class SM, class SX>
__global__ __launch_bounds__(TEAM) void k_step_s(DevModel mg, TrajDev stt, int nstep, const double* qfrc_applied,
                                                 const double* xfrc_applied) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_sep(mg, T, m);
  step_batch_body(m, L, C, X, T, stt, nstep, qfrc_applied, xfrc_applied);
}
__global__ __launch_bounds__(TEAM) void k_fwd_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, TrajDev stt,
                                                   const double* qfrc_applied, const double* xfrc_applied,
                                                   double* qacc) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  fwd_batch_body(m, L, C, X, T, stt, qfrc_applied, xfrc_applied, qacc);
}
template <class SM, class SX>
__global__ __launch_bounds__(TEAM) void k_fwd_s(DevModel mg, TrajDev stt, const double* qfrc_applied,
                                                const double* xfrc_applied, double* qacc) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_sep(mg, T, m);
  fwd_batch_body(m, L, C, X, T, stt, qfrc_applied, xfrc_applied, qacc);
}

// line-search selection + setDInit (inc/ilqr.h:110-113): per seed, the
// candidate with the smallest trajectory cost (mode 1; a NaN cost never wins
// over a number) or alpha = 1 (mode 0), copied to the nominal trajectory
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

}  // namespace

static bool use_dual() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ILQG_DUAL");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}
// LDS a rollout workgroup reserves: its workspace, or (ILQG_ROLLOUT_LDS) more,
// so that no FD team can share its CU
static size_t rollout_lds(size_t need) {
  static long pad = -1;
  if (pad < 0) {
    const char* e = getenv("ILQG_ROLLOUT_LDS");
    pad = e ? atol(e) : 0;
  }
  return (size_t)pad > need ? (size_t)pad : need;
}

hipError_t launch_rollout_coop(const DevModel& m, const WsLayout& L, const CoopLayout& C, const CoopAux& X, int S,
                               int A, int P, TrajDev nominal, TrajDev out, int out_is_cand, const double* K,
                               const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied,
                               const double* xfrc_applied, int passive, CostDev cost, double* cost_cand,
                               hipStream_t st, RollChunk ch) {
  const size_t lds = rollout_lds(coop_lds_bytes(L, C));
  hipError_t e;
  if (use_dual()) {
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id: {                                                                                                    \
    const size_t lds2 = rollout_lds(coop_lds_bytes(make_layout(stat::SMT{}, stat::SXT::npair, true), C));       \
    e = allow_lds(k_rollout2_s<stat::SMT, stat::SXT>, lds2);                                                    \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_rollout2_s<stat::SMT, stat::SXT>), dim3(S * A),                                       \
                       dim3(rollout_waves<stat::SMT>() * TEAM), lds2, st, m, S, A, P,                            \
                       nominal, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, \
                       cost_cand, ch);                                                                              \
    return hipGetLastError();                                                                                   \
  }
    switch (m.static_id) {
      ILQG_STATIC_MODELS(ILQG_CASE)
      default:
        break;
    }
#undef ILQG_CASE
    // the record's second buffer past the workspace when it fits (RollChunk.dbuf;
    // ILQG_ROLL_DBUF=0 keeps the register prefetch, A/B)
    size_t lds_d = lds;
    {
      static const int dbuf_env = [] {
        const char* v = getenv("ILQG_ROLL_DBUF");
        return (v && v[0] == '0') ? 0 : 1;
      }();
      const size_t R = (size_t)m.nq + m.nv + m.nu + (size_t)m.nu * 2 * m.nv + m.nu;
      const size_t need = (coop_lds_bytes(L, C) + 15) / 16 * 16 + R * sizeof(double);
      if (dbuf_env && need <= 160 * 1024) {
        ch.dbuf = 1;
        lds_d = need > lds ? need : lds;
      }
    }
    static const int nvc_env = [] {
      const char* v = getenv("ILQG_NV_CONST");
      return (v && v[0] == '0') ? 0 : 1;
    }();
    const bool nv27 = nvc_env && m.nv == 27;
    const void* kf = nv27 ? reinterpret_cast<const void*>(k_rollout2_coop<DevModelNV<27>>)
                          : reinterpret_cast<const void*>(k_rollout2_coop<DevModel>);
    e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_d);
    if (e != hipSuccess) return e;
    if (nv27)
      hipLaunchKernelGGL(k_rollout2_coop<DevModelNV<27>>, dim3(S * A), dim3(2 * TEAM), lds_d, st, m, L, C, X, S, A,
                         P, nominal, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost,
                         cost_cand, ch);
    else
    hipLaunchKernelGGL(k_rollout2_coop<DevModel>, dim3(S * A), dim3(2 * TEAM), lds_d, st, m, L, C, X, S, A, P, nominal, out,
                       out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand, ch);
    return hipGetLastError();
  }
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id:                                                                                                      \
    e = allow_lds(k_rollout_s<stat::SMT, stat::SXT>, lds);                                                      \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_rollout_s<stat::SMT, stat::SXT>), dim3(S * A), dim3(TEAM), lds, st, m, S, A, P,        \
                       nominal, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, \
                       cost_cand, ch);                                                                              \
    return hipGetLastError();
  switch (m.static_id) {
    ILQG_STATIC_MODELS(ILQG_CASE)
    default:
      break;
  }
#undef ILQG_CASE
  e = allow_lds(k_rollout_coop, coop_lds_bytes(L, C));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_rollout_coop, dim3(S * A), dim3(TEAM), coop_lds_bytes(L, C), st, m, L, C, X, S, A, P, nominal,
                     out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand, ch);
  return hipGetLastError();
}

hipError_t launch_select(const DevModel& m, int S, int A, int P, int mode, int copy_cand, const double* cost_cand,
                         int* sel, double* cost_sel, TrajDev cand, TrajDev nominal, TrajDev dinit, hipStream_t st) {
  hipLaunchKernelGGL(k_select, dim3(S), dim3(256), 0, st, m.nq, m.nv, m.nu, S, A, P, mode, copy_cand, cost_cand,
                     sel, cost_sel, cand, nominal, dinit);
  return hipGetLastError();
}

hipError_t launch_step_coop(const DevModel& m, const WsLayout& L, const CoopLayout& C, const CoopAux& X,
                            TrajDev stt, int n, int nstep, const double* qfrc_applied, const double* xfrc_applied,
                            hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipError_t e;
#define ILQG_CASE(id, SMT, SXT)                                                                                  \
  case id: {                                                                                                     \
    const size_t lds = coop_lds_bytes(make_layout(stat::SMT{}, stat::SXT::npair), C);                           \
    e = allow_lds(k_step_s<stat::SMT, stat::SXT>, lds);                                                          \
    if (e != hipSuccess) return e;                                                                               \
    hipLaunchKernelGGL((k_step_s<stat::SMT, stat::SXT>), dim3(n), dim3(TEAM), lds, st, m, stt, nstep,           \
                       qfrc_applied, xfrc_applied);                                                              \
    return hipGetLastError();                                                                                    \
  }
  switch (m.static_id) {
    ILQG_STATIC_MODELS(ILQG_CASE)
    default:
      break;
  }
#undef ILQG_CASE
  e = allow_lds(k_step_coop, coop_lds_bytes(L, C));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_step_coop, dim3(n), dim3(TEAM), coop_lds_bytes(L, C), st, m, L, C, X, stt, nstep,
                     qfrc_applied, xfrc_applied);
  return hipGetLastError();
}

hipError_t launch_forward_coop(const DevModel& m, const WsLayout& L, const CoopLayout& C, const CoopAux& X,
                               TrajDev stt, int n, const double* qfrc_applied, const double* xfrc_applied,
                               double* qacc, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipError_t e;
#define ILQG_CASE(id, SMT, SXT)                                                                                  \
  case id: {                                                                                                     \
    const size_t lds = coop_lds_bytes(make_layout(stat::SMT{}, stat::SXT::npair), C);                           \
    e = allow_lds(k_fwd_s<stat::SMT, stat::SXT>, lds);                                                           \
    if (e != hipSuccess) return e;                                                                               \
    hipLaunchKernelGGL((k_fwd_s<stat::SMT, stat::SXT>), dim3(n), dim3(TEAM), lds, st, m, stt, qfrc_applied,     \
                       xfrc_applied, qacc);                                                                      \
    return hipGetLastError();                                                                                    \
  }
  switch (m.static_id) {
    ILQG_STATIC_MODELS(ILQG_CASE)
    default:
      break;
  }
#undef ILQG_CASE
  e = allow_lds(k_fwd_coop, coop_lds_bytes(L, C));
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_fwd_coop, dim3(n), dim3(TEAM), coop_lds_bytes(L, C), st, m, L, C, X, stt, qfrc_applied,
                     xfrc_applied, qacc);
  return hipGetLastError();
}

}  // namespace ilqg

#ifdef ILQG_STAMPS
// the rollout kernels' line-search counters (dcoop_impl.h g_ls)
extern "C" int ilqg_debug_ls_rollout(unsigned long long* out5, int reset) {
  if (hipMemcpyFromSymbol(out5, HIP_SYMBOL(ilqg::coop::g_ls), sizeof(unsigned long long) * 8) != hipSuccess) return 3;
  if (reset) {
    unsigned long long z[8] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_ls), z, sizeof(z));
  }
  return 0;
}
extern "C" int ilqg_debug_stamps(unsigned long long* acc, unsigned long long* cnt, int reset) {
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
