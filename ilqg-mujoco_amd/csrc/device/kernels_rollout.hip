// Cooperative rollout kernels (inc/ilqr.h:116-130): one workgroup per
// (seed, alpha) candidate; two-wave teams (step_dual) by default.
#include "coop_common.h"

namespace ilqg {
namespace {

__device__ inline void rollout_body(const auto& m, const auto& L, const auto& C, const auto& X, const Team& T,
                                int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand, int wave, auto split) {
  // wave < 0: one-wave team; 0/1: primary/helper wave of a two-wave team (step_dual)
  const bool prim = wave <= 0;
  STAMP_INIT();
#ifdef ILQG_STAMPS
  unsigned long long rt0 = __builtin_amdgcn_s_memrealtime(), mt0 = __builtin_amdgcn_s_memtime();
#endif
  const int lane = blockIdx.x;
  const int s = lane / A, a = lane % A;
  const int nq = m.nq, nv = m.nv, nu = m.nu, nx = 2 * nv;
  load_state(m, L, T, dinit, s, s, qfrc_applied, xfrc_applied);
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
  const double* rq = rec;
  const double* rv = rec + nq;
  const double* ru = rec + nq + nv;
  const double* rK = ru + nu;
  const double* rk = rK + nu * nx;
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
  constexpr int PFR = 4;  // registers per lane: R <= 4 * 64
  double pf[PFR];
  if (!passive) {
    FOR_T(t, R) rec[t] = fetch((size_t)s * P + (P - 1), t);
    TSYNC();
  }
  const double alpha = alphas ? alphas[a] : 1.0;
  const int ob = out_is_cand ? lane : s;
  // the wave that runs the control law and writes the record: the helper wave
  // of a two-wave team (beside the primary's kinematics), else the only wave
  const bool ctl = wave != 0;
  double c = 0;
  // control law u = u* + alpha k + K (x - x*) for point n, its record and cost
  // (ilqr.h:116-133); the next point's nominal record is prefetched first
  auto pre_step = [&](int n) {
    const bool pre = !passive && n > 0;
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
        for (int j = 0; j < nx; j++) t += rK[i + j * nu] * dx[j];
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
    if (!passive && n > 0) {
#pragma unroll
      for (int q = 0; q < PFR; q++) {
        const int t = T.tid + q * TEAM_SIZE;
        if (t < R) rec[t] = pf[q];
      }
      TSYNC();
    }
  };
  if (wave >= 0) __syncthreads();
  for (int n = P - 1; n >= 0; n--) {
    if (wave < 0) {
      pre_step(n);
      step(m, L, C, X, T);
      park(n);
    } else {
      auto pre = [&]() {
        pre_step(n);
        park(n);
      };
      // split layout (compile-time models): the rebalanced two-wave schedule
      if constexpr (decltype(split)::value) step_dual_split(m, L, C, X, T, wave, pre);
      else step_dual(m, L, C, X, T, wave, pre);
    }
  }
  if (ctl && T.tid == 0 && cost_cand) cost_cand[lane] = c;
#ifdef ILQG_STAMPS
  if (prim && T.tid == 0 && blockIdx.x == 0) {
    g_stamp_acc[46] += __builtin_amdgcn_s_memrealtime() - rt0;
    g_stamp_acc[47] += __builtin_amdgcn_s_memtime() - mt0;
  }
#endif
  STAMP_FLUSH();
}

__global__ __launch_bounds__(TEAM) void k_rollout_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand, -1, std::false_type{});
}

// model-specific instance (static_models.h): compile-time sizes, tables and LDS layout
template <class SM, class SX>
__global__ __launch_bounds__(TEAM) void k_rollout_s(DevModel mg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_sep(mg, T, m);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand, -1, std::false_type{});
}

// two-wave teams (step_dual): 128 threads per (seed, candidate)
__global__ __launch_bounds__(2 * TEAM) void k_rollout2_coop(DevModel mg, WsLayout L, CoopLayout C, CoopAux Xg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand) {
  Team T = make_team(L, C);
  DevModel m;
  CoopAux X;
  stage_model(mg, Xg, L, C, T, m, X);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied,
               passive, cost, cost_cand, (int)(threadIdx.x / TEAM), std::false_type{});
}
template <class SM, class SX>
__global__ __launch_bounds__(2 * TEAM) void k_rollout2_s(DevModel mg, int S, int A, int P, TrajDev nom, TrajDev out, int out_is_cand, const double* K, const double* k, const double* alphas, TrajDev dinit, const double* qfrc_applied, const double* xfrc_applied, int passive, CostDev cost, double* cost_cand) {
  static constexpr WsLayout L = make_layout(SM{}, SX::npair, true);
  static constexpr CoopLayout C = make_coop_layout(SM{}, SX::npair);
  static constexpr SX X{};
  Team T = make_team(L, C);
  SM m;
  stage_model_sep(mg, T, m);
  rollout_body(m, L, C, X, T, S, A, P, nom, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied,
               passive, cost, cost_cand, (int)(threadIdx.x / TEAM), std::bool_constant<SM::nv <= RMAX>{});
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
                               hipStream_t st) {
  const size_t lds = rollout_lds(coop_lds_bytes(L, C));
  hipError_t e;
  if (use_dual()) {
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id: {                                                                                                    \
    const size_t lds2 = rollout_lds(coop_lds_bytes(make_layout(stat::SMT{}, stat::SXT::npair, true), C));       \
    e = allow_lds(k_rollout2_s<stat::SMT, stat::SXT>, lds2);                                                    \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_rollout2_s<stat::SMT, stat::SXT>), dim3(S * A), dim3(2 * TEAM), lds2, st, m, S, A, P,  \
                       nominal, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, \
                       cost_cand);                                                                              \
    return hipGetLastError();                                                                                   \
  }
    switch (m.static_id) {
      ILQG_STATIC_MODELS(ILQG_CASE)
      default:
        break;
    }
#undef ILQG_CASE
    e = allow_lds(k_rollout2_coop, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_rollout2_coop, dim3(S * A), dim3(2 * TEAM), lds, st, m, L, C, X, S, A, P, nominal, out,
                       out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand);
    return hipGetLastError();
  }
#define ILQG_CASE(id, SMT, SXT)                                                                                 \
  case id:                                                                                                      \
    e = allow_lds(k_rollout_s<stat::SMT, stat::SXT>, lds);                                                      \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((k_rollout_s<stat::SMT, stat::SXT>), dim3(S * A), dim3(TEAM), lds, st, m, S, A, P,        \
                       nominal, out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, \
                       cost_cand);                                                                              \
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
                     out, out_is_cand, K, k, alphas, dinit, qfrc_applied, xfrc_applied, passive, cost, cost_cand);
  return hipGetLastError();
}

}  // namespace ilqg

#ifdef ILQG_STAMPS
extern "C" int ilqg_debug_stamps(unsigned long long* acc, unsigned long long* cnt, int reset) {
  if (hipMemcpyFromSymbol(acc, HIP_SYMBOL(ilqg::coop::g_stamp_acc), sizeof(unsigned long long) * 48) != hipSuccess)
    return 3;
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(ilqg::coop::g_stamp_cnt), sizeof(unsigned long long) * 48) != hipSuccess)
    return 3;
  unsigned long long nw[2];
  (void)hipMemcpyFromSymbol(&nw[0], HIP_SYMBOL(ilqg::coop::g_newton_iters), 8);
  (void)hipMemcpyFromSymbol(&nw[1], HIP_SYMBOL(ilqg::coop::g_newton_calls), 8);
  acc[44] = nw[0];
  acc[45] = nw[1];
  if (reset) {
    unsigned long long z[48] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_newton_iters), z, 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_newton_calls), z, 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_stamp_acc), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(ilqg::coop::g_stamp_cnt), z, sizeof(z));
  }
  return 0;
}
#endif
