// Shared pieces of the cooperative hot-path kernels (kernels_fd.hip,
// kernels_rollout.hip): one 64-lane workgroup (one wavefront) per physics
// evaluation, workspace in LDS (dcoop.h).  Each translation unit includes this
// once (everything here is internal to it).
#pragma once
#include <algorithm>

#include "dcoop.h"
#include "handoff.h"
#include "kernels.h"
#include "static_models.h"

namespace ilqg {
namespace {

using namespace coop;

using namespace coop;

constexpr double FD_EPS = 1e-6;  // mjderivative.cpp:39
constexpr int FD_NITER = 30;     // mjderivative.cpp:37
constexpr int FD_NWARMUP = 3;    // mjderivative.cpp:38
constexpr int TEAM = TEAM_SIZE;
// FD teams: at least 2 waves per SIMD (<= 256 VGPRs), so LDS (6 teams per CU
// for the hopper) and not registers bounds the sweep's occupancy
constexpr int FD_WAVES_PER_EU = 2;
#ifndef ILQG_BW_PRIO
#define ILQG_BW_PRIO 1
#endif

// LDS: [workspace doubles][coop doubles][model image][workspace ints][coop ints]
__device__ inline Team make_team(const auto& L, const auto& C) {
  extern __shared__ double lds[];
  Team T;
  T.w = lds;
  T.c = lds + L.nd;
  T.iw = reinterpret_cast<int*>(lds + L.nd + C.nd + C.imgd);
  T.ci = T.iw + L.ni;
  T.tid = threadIdx.x & (TEAM - 1);  // lane within this wave (two-wave teams: one Team per wave)
  T.nt = TEAM;  // every cooperative kernel is launched with one 64-lane wavefront
  return T;
}

// Stage the read-only model image into LDS (one coalesced copy) and return a
// DevModel / CoopAux whose array pointers address the LDS copy: every model
// read on the serial paths then costs an LDS round trip instead of an L2 one.
__device__ inline void stage_model(const DevModel& g, const CoopAux& Xg, const WsLayout& L, const CoopLayout& C,
                                   const Team& T, DevModel& m, CoopAux& X) {
  if (C.imgd == 0) {
    // layouts without an image region (models whose workspace leaves no LDS
    // for it, e.g. the humanoid): every model read goes to the global image
    m = g;
    X = Xg;
    return;
  }
  extern __shared__ double lds[];
  double* dst = lds + L.nd + C.nd;
  const double* src = reinterpret_cast<const double*>(g.img);
  FOR_T(w, C.imgd) dst[w] = src[w];
  const unsigned char* base = reinterpret_cast<const unsigned char*>(dst);
  m = g;
#define ILQG_RB(nm, cnt) \
  m.nm = reinterpret_cast<decltype(m.nm)>(base + (reinterpret_cast<const unsigned char*>(g.nm) - g.img));
  ILQG_MODEL_F64_ARRAYS(ILQG_RB)
  ILQG_MODEL_I32_ARRAYS(ILQG_RB)
#undef ILQG_RB
  X.isanc = reinterpret_cast<const int*>(base + (reinterpret_cast<const unsigned char*>(Xg.isanc) - g.img));
  X.pair = reinterpret_cast<const int*>(base + (reinterpret_cast<const unsigned char*>(Xg.pair) - g.img));
  X.npair = Xg.npair;
  X.haspm = Xg.haspm;
  // (an offset select, not a pointer one: a null LDS pointer cast to flat is
  // what ROCm's backend miscompiles in the stamps build; unread when !haspm)
  X.pmask = reinterpret_cast<const unsigned long long*>(
      base + (Xg.haspm ? reinterpret_cast<const unsigned char*>(Xg.pmask) - g.img : 0));
  TSYNC();
}

// model-specific variant: same image copy; sizes/tables are compile-time
// (static_models.h), float arrays bound at compile-time LDS offsets
template <class SM>
__device__ inline void stage_model_s(const DevModel& g, const auto& L, const auto& C, const Team& T, SM& m) {
  extern __shared__ double lds[];
  double* dst = lds + L.nd + C.nd;
  const double* src = reinterpret_cast<const double*>(g.img);
  FOR_T(w, C.imgd) dst[w] = src[w];
  m.bind(reinterpret_cast<const unsigned char*>(dst), g);
  TSYNC();
}

// model-specific variant with the image in a __shared__ object of its own
// (not the workspace array): loads of model data provably do not alias the
// workspace stores, so the compiler may hoist and overlap them
template <class SM>
__device__ inline void stage_model_sep(const DevModel& g, const Team& T, SM& m) {
  constexpr int ND = (SM::img_bytes + 7) / 8;
  __shared__ double img[ND];
  const double* src = reinterpret_cast<const double*>(g.img);
  FOR_T(w, ND) img[w] = src[w];
  m.bind(reinterpret_cast<const unsigned char*>(img), g);
  TSYNC();
}

__device__ inline double cost_terms(double c, const double* x, const double* w, const double* t, const double* l,
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
__device__ inline double step_cost(const auto& m, const CostDev& c, const double* qpos, const double* qvel,
                                   const double* ctrl) {
  double s = 0;
  s = cost_terms(s, qpos, c.wq, c.tq, c.lq, m.nq);
  s = cost_terms(s, qvel, c.wv, c.tv, c.lv, m.nv);
  s = cost_terms(s, ctrl, c.wu, c.tu, c.lu, m.nu);
  return s;
}

// copy the cost descriptor into LDS (C.cdesc): the per-step cost loop on lane 0
// then reads LDS instead of global memory
__device__ inline CostDev stage_cost(const auto& m, const auto& C, const Team& T, const CostDev& g) {
  double* d = T.c + C.cdesc;
  const int nq = m.nq, nv = m.nv, nu = m.nu;
  const double* src[9] = {g.wq, g.tq, g.lq, g.wv, g.tv, g.lv, g.wu, g.tu, g.lu};
  const int off[9] = {0, nq, 2 * nq, 3 * nq, 3 * nq + nv, 3 * nq + 2 * nv, 3 * (nq + nv), 3 * (nq + nv) + nu,
                      3 * (nq + nv) + 2 * nu};
  const int len[9] = {nq, nq, nq, nv, nv, nv, nu, nu, nu};
  for (int a = 0; a < 9; a++) FOR_T(i, len[a]) d[off[a] + i] = src[a][i];
  TSYNC();
  CostDev l;
  l.wq = d + off[0]; l.tq = d + off[1]; l.lq = d + off[2];
  l.wv = d + off[3]; l.tv = d + off[4]; l.lv = d + off[5];
  l.wu = d + off[6]; l.tu = d + off[7]; l.lu = d + off[8];
  return l;
}

// cpMjData(d, src) from a trajectory record (src/util.cpp:4-14).  Every global
// load is issued before the first LDS store (one memory round trip, not one
// per field: the FD teams start with this, ~64k of them per sweep)
__device__ inline void load_state(const auto& m, const auto& L, const Team& T, const TrajDev& tr, int pt,
                                  int seed, const double* qfrc_applied, const double* xfrc_applied) {
  const int nq = m.nq, nv = m.nv, nu = m.nu, nx6 = 6 * m.nbody;
  const int t = T.tid;
  if (nq <= TEAM && nv <= TEAM && nu <= TEAM && nx6 <= 2 * TEAM && T.nt == TEAM) {
    const double q = t < nq ? tr.qpos[(size_t)pt * nq + t] : 0.0;
    const double v = t < nv ? tr.qvel[(size_t)pt * nv + t] : 0.0;
    const double w = t < nv ? tr.warm[(size_t)pt * nv + t] : 0.0;
    const double fa = (t < nv && qfrc_applied) ? qfrc_applied[(size_t)seed * nv + t] : 0.0;
    const double c = t < nu ? tr.ctrl[(size_t)pt * nu + t] : 0.0;
    const double x0 = (t < nx6 && xfrc_applied) ? xfrc_applied[(size_t)seed * nx6 + t] : 0.0;
    const double x1 = (t + TEAM < nx6 && xfrc_applied) ? xfrc_applied[(size_t)seed * nx6 + t + TEAM] : 0.0;
    const double tm = tr.time[pt];
    if (t < nq) T.w[L.qpos + t] = q;
    if (t < nv) {
      T.w[L.qvel + t] = v;
      T.w[L.warm + t] = w;
      T.w[L.qfrc_applied + t] = fa;
    }
    if (t < nu) T.w[L.ctrl + t] = c;
    if (t < nx6) T.w[L.xfrc_applied + t] = x0;
    if (t + TEAM < nx6) T.w[L.xfrc_applied + t + TEAM] = x1;
    if (t == 0) T.w[L.time] = tm;
    TSYNC();
    return;
  }
  FOR_T(i, nq) T.w[L.qpos + i] = tr.qpos[(size_t)pt * nq + i];
  FOR_T(i, nv) {
    T.w[L.qvel + i] = tr.qvel[(size_t)pt * nv + i];
    T.w[L.warm + i] = tr.warm[(size_t)pt * nv + i];
    T.w[L.qfrc_applied + i] = qfrc_applied ? qfrc_applied[(size_t)seed * nv + i] : 0.0;
  }
  FOR_T(i, nu) T.w[L.ctrl + i] = tr.ctrl[(size_t)pt * nu + i];
  FOR_T(i, nx6) T.w[L.xfrc_applied + i] = xfrc_applied ? xfrc_applied[(size_t)seed * nx6 + i] : 0.0;
  if (T.tid == 0) T.w[L.time] = tr.time[pt];
  TSYNC();
}

template <typename K>
hipError_t allow_lds(K kern, size_t lds) {
  if (lds <= 65536) return hipSuccess;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds);
}


}  // namespace
}  // namespace ilqg
