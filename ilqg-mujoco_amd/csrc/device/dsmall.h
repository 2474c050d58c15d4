// Register-resident small-matrix kernels for one wavefront (nv <= RMAX).
//
// The serial recursions of the physics pipeline -- MuJoCo's tree L'DL of the
// mass matrix, its solve, the dense Cholesky of the Newton Hessian and the
// search-direction solve -- ran on lane 0 out of LDS, paying an LDS round trip
// (~64-140 cycles on gfx950) per dependent access.  Here lane t holds row t
// (and, for the solves, column t) of the matrix in VGPRs; the row needed by
// step k is broadcast with v_readlane (k is wave-uniform), so the divisions
// and row updates of one step run on all lanes at once.
//
// Bit-exactness: every matrix entry still receives exactly the same sequence
// of IEEE operations as in the oracle's serial loops (oracle/mjsub.c
// factor_ld / solve_ld / the Newton Cholesky): updates to entry (i,j) happen
// in the same k order, dot products keep ascending index order, and every
// division is the same operand pair.  Only independent work is overlapped.
#pragma once

#include <type_traits>

#include "dphys.h"

namespace ilqg {
namespace coop {

// Team synchronisation.  A team is exactly one wavefront (every cooperative
// kernel launches 64 lanes), whose LDS accesses the hardware executes in
// instruction order, so the only thing needed between phases is a compiler
// barrier that keeps LDS accesses from moving across it: wavefront-scope
// fences emit no s_waitcnt.  __syncthreads() would also wait for every
// outstanding global load/store (vmcnt(0)) at each phase boundary, exposing
// HBM latency in the per-step output stores and prefetches.
__device__ __forceinline__ void team_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

using dev::MINVAL;
constexpr int TEAM_SIZE = 64;  // lanes of a team: exactly one wavefront
constexpr int RMAX = 8;  // register rows up to this many dofs

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1, so
// every register-array index is a constant (no scratch, no select chains)
template <int B, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}
#define SK(v) decltype(v)::value
#define SLAM(v) [&](auto v) __attribute__((always_inline))

// v_readlane of a double from a wave-uniform lane
__device__ __forceinline__ double bcast(double x, int lane) {
  long long b = __double_as_longlong(x);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ unsigned long long bcast_u64(unsigned long long x, int lane) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffull), lane);
  const unsigned hi = __builtin_amdgcn_readlane((int)(x >> 32), lane);
  return ((unsigned long long)hi << 32) | lo;
}

// ---- fp64 division with the divisor's refined reciprocal computed early ----
// The compiler's f64 division is ten dependent operations: v_div_scale of the
// divisor, v_rcp, four fma refining that reciprocal, v_div_scale of the
// dividend, mul, fma, v_div_fmas, v_div_fixup.  The reciprocal part reads only
// the (scaled) divisor.  When the divisor is known before the dividend (a
// Cholesky diagonal, the line search's curvature), rcp_ref() runs that part
// once, off the critical path, and div_ref() runs the rest of the same
// sequence on the same operands: the same IEEE quotient, bit for bit.
// v_div_scale leaves the divisor unscaled except at extreme exponents
// (|a| >= 2^768 |b|, denormal b or 1/b) and for a == 0, NaN or Inf; there the
// precomputed reciprocal is not the sequence's, and the ordinary division runs.
__device__ __forceinline__ double rcp_ref(double b) {
  double r = __builtin_amdgcn_rcp(b);
  double t = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, t, r);
  t = __builtin_fma(-b, r, 1.0);
  return __builtin_fma(r, t, r);
}
// the quotient's tail; `den_ok` is false where the divisor would be scaled
__device__ __forceinline__ double div_tail(double a, double b, double r, bool& den_ok) {
  bool fd, fn;
  const double ds = __builtin_amdgcn_div_scale(a, b, false, &fd);
  const double ns = __builtin_amdgcn_div_scale(a, b, true, &fn);
  den_ok = __builtin_bit_cast(long long, ds) == __builtin_bit_cast(long long, b);
  const double q = ns * r;
  const double e = __builtin_fma(-b, q, ns);
  return __builtin_amdgcn_div_fixup(__builtin_amdgcn_div_fmas(e, r, q, fn), b, a);
}
// the ordinary division, kept behind its branch: the empty volatile asm stops
// the compiler from speculating it (and its ten-operation chain) beside the tail
__device__ __forceinline__ double div_slow(double a, double b) {
  asm volatile("" : "+v"(a));
  return a / b;
}
// a / b on every lane (r = rcp_ref(b))
__device__ __forceinline__ double div_ref(double a, double b, double r) {
  bool ok;
  double q = div_tail(a, b, r, ok);
  if (__builtin_expect(!ok, 0)) q = div_slow(a, b);
  return q;
}
// a / b where only lane k's quotient is used (the other lanes' operands may
// be anything): the fallback is taken only when lane k needs it (uniform)
template <int K>
__device__ __forceinline__ double div_ref_lane(double a, double b, double r) {
  bool ok;
  double q = div_tail(a, b, r, ok);
  if (__builtin_expect((__ballot(!ok) >> K) & 1, 0)) q = div_slow(a, b);
  return q;
}

// fp32 physics (coopf, the fp32 FD sweep): plain IEEE division
__device__ __forceinline__ float rcp_ref(float) { return 0.f; }
template <int K>
__device__ __forceinline__ float div_ref_lane(float a, float b, float) {
  return a / b;
}
// v_readlane of a float
__device__ __forceinline__ float bcast(float x, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}

// r[idx] for a per-lane index: select chain over constant indices (written
// with sfor so SROA sees constant subscripts and keeps r in registers)
template <class R>
__device__ __forceinline__ R rsel(const R (&r)[RMAX], int idx) {
  R v = r[0];
  sfor<1, RMAX>(SLAM(jj) { v = (idx == SK(jj)) ? r[SK(jj)] : v; });
  return v;
}

// Tree L'DL factorization of the lower triangle of `mat` (nv x nv, row-major)
// into LD (full nv x nv, zero upper) and diaginv.  pmask[i]: proper ancestors
// of dof i.  Mirrors coop::factor_ld's serial loop entry by entry.
template <class R>
__device__ inline void factor_ld_rows(int nv, const auto& pmask, int tid, const R* mat, R* LD, R* diaginv) {
  R r[RMAX];
  unsigned long long pm[RMAX];  // wave-uniform ancestor masks, loaded up front
  const bool own = tid < nv;
  sfor<0, RMAX>(SLAM(jj) {
    constexpr int j = SK(jj);
    r[j] = (own && j < nv && j <= tid) ? mat[tid * nv + j] : 0.0;
    pm[j] = j < nv ? pmask[j] : 0ull;
  });
  const unsigned long long self = own ? (pmask[tid] | (1ull << tid)) : 0ull;  // {t} u anc(t)
  team_sync();  // all rows read before LD (may alias mat) is written
  sfor<0, RMAX>(SLAM(kk) {
    constexpr int k = RMAX - 1 - SK(kk);
    if (k >= nv) return;
    const unsigned long long ak = pm[k];
    R dk = bcast(r[k], k);
    if (dk < MINVAL) dk = MINVAL;
    R rk[RMAX];
    sfor<0, RMAX>(SLAM(jj) {
      constexpr int j = SK(jj);
      rk[j] = (j <= k) ? bcast(r[j], k) : 0.0;
    });
    // lanes i in anc(k): tmp_i = LD[k][i] / LD[k][k]; row i -= tmp_i * row k
    R tmp = 0;
    if (own && ((ak >> tid) & 1)) {
      tmp = rsel(rk, tid) / dk;
      sfor<0, k>(SLAM(jj) {
        constexpr int j = SK(jj);
        if ((self >> j) & 1) r[j] -= tmp * rk[j];
      });
    }
    // lane k: LD[k][i] = tmp_i (the same quotient, gathered) and the clamp
    sfor<0, k>(SLAM(ii) {
      constexpr int i = SK(ii);
      if ((ak >> i) & 1) {
        const R ti = bcast(tmp, i);
        if (tid == k) r[i] = ti;
      }
    });
    if (tid == k) r[k] = dk;
  });
  if (own) {
    sfor<0, RMAX>(SLAM(jj) {
      if (SK(jj) < nv) LD[tid * nv + SK(jj)] = r[SK(jj)];
    });
    diaginv[tid] = 1 / rsel(r, tid);
  }
  team_sync();
}

// Two tree L'DL factorizations with the same sparsity at once: lanes 0..31
// factor mat0 (row t on lane t), lanes 32..63 factor mat1 (row t on lane
// 32 + t); every broadcast reads the lane of the caller's own half.  Each
// factor receives exactly the operations of factor_ld_rows.  The matrices and
// factors are addressed as offsets from mat0 / LD0 / dinv0 (no pointer
// selects).  nv <= RMAX <= 32.
template <class R>
__device__ inline void factor_ld_rows2(int nv, const auto& pmask, int tid, const R* mat0, R* LD0, R* diaginv0,
                                       const R* mat1, R* LD1, R* diaginv1) {
  const bool hi = tid >= 32;
  const int t = tid & 31;
  const int om = hi ? (int)(mat1 - mat0) : 0, ol = hi ? (int)(LD1 - LD0) : 0,
            od = hi ? (int)(diaginv1 - diaginv0) : 0;
  const R* mat = mat0 + om;
  R* LD = LD0 + ol;
  R* diaginv = diaginv0 + od;
  auto bc = [&](R x, int k) __attribute__((always_inline)) {
    const R a = bcast(x, k), b = bcast(x, 32 + k);
    return hi ? b : a;
  };
  R r[RMAX];
  unsigned long long pm[RMAX];
  const bool own = t < nv;
  sfor<0, RMAX>(SLAM(jj) {
    constexpr int j = SK(jj);
    r[j] = (own && j < nv && j <= t) ? mat[t * nv + j] : 0.0;
    pm[j] = j < nv ? pmask[j] : 0ull;
  });
  const unsigned long long self = own ? (pmask[t] | (1ull << t)) : 0ull;
  team_sync();
  sfor<0, RMAX>(SLAM(kk) {
    constexpr int k = RMAX - 1 - SK(kk);
    if (k >= nv) return;
    const unsigned long long ak = pm[k];
    R dk = bc(r[k], k);
    if (dk < MINVAL) dk = MINVAL;
    R rk[RMAX];
    sfor<0, RMAX>(SLAM(jj) {
      constexpr int j = SK(jj);
      rk[j] = (j <= k) ? bc(r[j], k) : 0.0;
    });
    R tmp = 0;
    if (own && ((ak >> t) & 1)) {
      tmp = rsel(rk, t) / dk;
      sfor<0, k>(SLAM(jj) {
        constexpr int j = SK(jj);
        if ((self >> j) & 1) r[j] -= tmp * rk[j];
      });
    }
    sfor<0, k>(SLAM(ii) {
      constexpr int i = SK(ii);
      if ((ak >> i) & 1) {
        const R ti = bc(tmp, i);
        if (t == k) r[i] = ti;
      }
    });
    if (t == k) r[k] = dk;
  });
  if (own) {
    sfor<0, RMAX>(SLAM(jj) {
      if (SK(jj) < nv) LD[t * nv + SK(jj)] = r[SK(jj)];
    });
    diaginv[t] = 1 / rsel(r, t);
  }
  team_sync();
}

// Tree L'DL factorization with compile-time sparsity (XT::pmask[k]: proper
// ancestors of dof k), one matrix per lane, wholly in that lane's registers:
// lane 0 factors mat into (LD0, diaginv0); with `two`, lane 1 factors
// mat + diag(add) into (LD0 + o1, diaginv0 + od1) -- the Euler matrix M + h D,
// whose diagonal sum is formed here exactly as euler_prefactor forms it.
// This is the oracle's serial loop (coop::factor_ld, oracle/mjsub.c factor_ld)
// with every index a constant: no broadcasts, no lane-dependent branches, no
// SGPR masks (factor_ld_rows2's two-half broadcasts and selects cost ~800
// wave instructions for the hopper, three quarters of them v_readlane / v_mov /
// v_cndmask; this is ~300, all arithmetic).  Same operations on the same
// operands per entry; LD is written in full with a zero upper triangle.
template <class XT, int NV, class R>
__device__ inline void factor_ld_lanes(int tid, const R* mat, const R (&add)[NV], bool two, R* LD0, R* diaginv0,
                                       int o1, int od1) {
  const bool l1 = two && tid == 1;
  R a[NV][NV];
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    sfor<0, i + 1>(SLAM(jj) { a[i][SK(jj)] = mat[i * NV + SK(jj)]; });
  });
  sfor<0, NV>(SLAM(ii) {
    constexpr int i = SK(ii);
    const R s = a[i][i] + add[i];
    a[i][i] = l1 ? s : a[i][i];
  });
  team_sync();  // every lane has read mat before LD (may alias it) is written
  sfor<0, NV>(SLAM(kk) {
    constexpr int k = NV - 1 - SK(kk);
    R dk = a[k][k];
    if (dk < MINVAL) dk = MINVAL;
    a[k][k] = dk;
    sfor<0, k>(SLAM(ii) {
      constexpr int i = k - 1 - SK(ii);
      if constexpr ((XT::pmask[k] >> i) & 1) {
        const R tmp = a[k][i] / dk;
        sfor<0, i + 1>(SLAM(jj) {
          constexpr int j = i - SK(jj);
          if constexpr (j == i || ((XT::pmask[i] >> j) & 1)) a[i][j] -= tmp * a[k][j];
        });
        a[k][i] = tmp;
      }
    });
  });
  if (tid == 0 || l1) {
    const int o = l1 ? o1 : 0, od = l1 ? od1 : 0;
    sfor<0, NV>(SLAM(ii) {
      constexpr int i = SK(ii);
      sfor<0, NV>(SLAM(jj) {
        constexpr int j = SK(jj);
        if constexpr (j <= i) LD0[o + i * NV + j] = a[i][j];
        else LD0[o + i * NV + j] = (R)0;
      });
      diaginv0[od + i] = 1 / a[i][i];
    });
  }
  team_sync();
}

// x <- (L'DL)^-1 x for the factor above; mirrors coop::solve_ld.
template <class R>
__device__ inline void solve_ld_rows(int nv, const auto& pmask, int tid, const R* LD, const R* diaginv, R* x) {
  const bool own = tid < nv;
  R row[RMAX], col[RMAX], xt = 0, dinv = 0;
  unsigned long long anc = 0;
  sfor<0, RMAX>(SLAM(jj) {
    constexpr int j = SK(jj);
    row[j] = (own && j < nv) ? LD[tid * nv + j] : 0.0;
    col[j] = (own && j < nv) ? LD[j * nv + tid] : 0.0;
  });
  if (own) {
    xt = x[tid];
    dinv = diaginv[tid];
    anc = pmask[tid];
  }
  // x[j] -= LD[i][j] * x[i] for j in anc(i), i descending (skipped when x[i] == 0)
  sfor<0, RMAX>(SLAM(ii) {
    constexpr int i = RMAX - 1 - SK(ii);
    if (i >= nv) return;
    const R xi = bcast(xt, i);
    if (xi != 0 && own && ((pmask[i] >> tid) & 1)) xt -= col[i] * xi;
  });
  xt *= dinv;
  // x[i] -= LD[i][j] * x[j] for j in anc(i) descending, i ascending
  R xf[RMAX];
  sfor<0, RMAX>(SLAM(ii) {
    constexpr int i = SK(ii);
    if (i >= nv) {
      xf[i] = 0;
      return;
    }
    if (tid == i) {
      sfor<0, i>(SLAM(jj) {
        constexpr int j = i - 1 - SK(jj);
        if ((anc >> j) & 1) xt -= row[j] * xf[j];
      });
    }
    xf[i] = bcast(xt, i);
  });
  team_sync();  // every lane has read x before it is overwritten
  if (own) x[tid] = xt;
  team_sync();
}

// In-place dense Cholesky of the lower triangle of H (row-major nv x nv);
// mirrors coop::hessian_factor's serial loop.
template <class R>
__device__ inline void cholesky_rows(int nv, int tid, R* H) {
  const bool own = tid < nv;
  R r[RMAX];
  sfor<0, RMAX>(SLAM(jj) {
    constexpr int j = SK(jj);
    r[j] = (own && j < nv && j <= tid) ? H[tid * nv + j] : 0.0;
  });
  sfor<0, RMAX>(SLAM(jc) {
    constexpr int j = SK(jc);
    if (j >= nv) return;
    R rj[RMAX];  // row j, entries 0..j-1 final
    sfor<0, j>(SLAM(qq) { rj[SK(qq)] = bcast(r[SK(qq)], j); });
    R t = bcast(r[j], j);
    if (j) {
      R s = 0;
      sfor<0, j>(SLAM(qq) { s += rj[SK(qq)] * rj[SK(qq)]; });
      t -= s;
    }
    if (t < MINVAL) t = MINVAL;
    const R d = sqrt(t);
    const R tinv = 1 / d;
    if (tid == j) r[j] = d;
    if (own && tid > j) {
      R s = 0;
      sfor<0, j>(SLAM(qq) { s += r[SK(qq)] * rj[SK(qq)]; });
      r[j] = (r[j] - s) * tinv;
    }
  });
  team_sync();
  if (own) {
    sfor<0, RMAX>(SLAM(jj) {
      if (SK(jj) < nv && SK(jj) <= tid) H[tid * nv + SK(jj)] = r[SK(jj)];
    });
  }
  team_sync();
}

// The same Cholesky for RMAX < nv <= 32 (the humanoid, nv = 27) with run-time
// nv: lane t keeps row t in registers for the whole factorization, row j is
// broadcast entry by entry (v_readlane) as column j needs it, and the
// diagonal's dot product is lane j's own row dot product -- the oracle's
// tdot(H_j, H_j, j) and tdot(H_i, H_j, j), ascending from +0.  No LDS round
// trip or barrier per column (the LDS form: one of each).
template <int NC = 0, class R>
__device__ inline void cholesky_rows32(int nv_rt, int tid, R* H) {
  // NC > 0: the dof count known at compile time (DevModelNV): no size guards
  constexpr int NM = NC > 0 ? NC : 32;
  const int nv = NC > 0 ? NC : nv_rt;
  const bool own = tid < nv;
  R r[NM];
  sfor<0, NM>(SLAM(jj) {
    constexpr int j = SK(jj);
    r[j] = (own && j < nv && j <= tid) ? H[tid * nv + j] : (R)0.0;
  });
  sfor<0, NM>(SLAM(jc) {
    constexpr int j = SK(jc);
    if (j >= nv) return;
    R s = 0;
    sfor<0, j>(SLAM(qq) { s += r[SK(qq)] * bcast(r[SK(qq)], j); });
    R t = r[j];
    if (j) t -= s;
    t = bcast(t, j);
    if (t < MINVAL) t = MINVAL;
    const R d = sqrt(t);
    const R tinv = 1 / d;
    if (tid == j) r[j] = d;
    if (own && tid > j) r[j] = (r[j] - s) * tinv;
  });
  team_sync();
  if (own) {
    sfor<0, NM>(SLAM(jj) {
      if (SK(jj) < nv && SK(jj) <= tid) H[tid * nv + SK(jj)] = r[SK(jj)];
    });
  }
  team_sync();
}

// search = -(H H')^-1 grad with the Cholesky factor in H's lower triangle;
// mirrors the lane-0 substitution in coop::solver_newton.
template <class R>
__device__ inline void chol_solve_rows(int nv, int tid, const R* H, const R* grad, R* search) {
  const bool own = tid < nv;
  R row[RMAX], col[RMAX], g = 0;
  sfor<0, RMAX>(SLAM(jj) {
    constexpr int j = SK(jj);
    row[j] = (own && j < nv) ? H[tid * nv + j] : 0.0;
    col[j] = (own && j < nv) ? H[j * nv + tid] : 0.0;
  });
  if (own) g = grad[tid];
  const R dg = own ? rsel(row, tid) : (R)1.0;
  const R rg = rcp_ref(dg);
  // forward: s[i] = (s[i] - sum_{j<i} H[i][j] s[j]) / H[i][i].  Every lane
  // accumulates its dot product as the s[j] arrive (ascending j, from +0: the
  // oracle's dotn), so step i is one subtraction and the division's tail; no
  // lane-divergent branches
  R sf[RMAX], acc = 0, gf = 0;
  sfor<0, RMAX>(SLAM(ii) {
    constexpr int i = SK(ii);
    if (i >= nv) {
      sf[i] = 0;
      return;
    }
    const R q = div_ref_lane<i>(i ? g - acc : g, dg, rg);
    sf[i] = bcast(q, i);
    acc += row[i] * sf[i];
    gf = tid == i ? sf[i] : gf;
  });
  g = gf;
  // backward: s[i] -= H[j][i] s[j] for j = i+1.. ascending, then / H[i][i];
  // the products are formed as the s[j] arrive
  R sb[RMAX], pr[RMAX];
  sfor<0, RMAX>(SLAM(ii) {
    constexpr int i = RMAX - 1 - SK(ii);
    if (i >= nv) {
      sb[i] = 0;
      pr[i] = 0;
      return;
    }
    R t = g;
    sfor<i + 1, RMAX>(SLAM(jj) {
      constexpr int j = SK(jj);
      if (j < nv) t -= pr[j];
    });
    sb[i] = bcast(div_ref_lane<i>(t, dg, rg), i);
    pr[i] = col[i] * sb[i];
    gf = tid == i ? sb[i] : gf;
  });
  if (own) search[tid] = -gf;
  team_sync();
}

// a / b where only lane k's quotient is used, k wave-uniform at run time
__device__ __forceinline__ double div_ref_lane_rt(double a, double b, double r, int k) {
  bool ok;
  double q = div_tail(a, b, r, ok);
  if (__builtin_expect((__ballot(!ok) >> k) & 1, 0)) q = div_slow(a, b);
  return q;
}
__device__ __forceinline__ float div_ref_lane_rt(float a, float b, float, int) { return a / b; }
// a / b on every lane, b's reciprocal refined ahead (fp64) / plain (fp32)
__device__ __forceinline__ double div_u(double a, double b, double r) { return div_ref(a, b, r); }
__device__ __forceinline__ float div_u(float a, float b, float) { return a / b; }

// The same substitution for RMAX < nv <= TEAM_SIZE (the humanoid, nv = 27),
// with run-time loops: lane t holds row t's running dot product (forward) and
// its final entry; nothing but the matrix entries goes through LDS.  Mirrors the
// lane-0 loops of coop::solver_newton entry by entry:
//   forward  s[i] = (g[i] - sum_{j<i} H[i][j] s[j]) / H[i][i], the sum ascending
//            from +0 (tdot) -- lane t adds H[t][i] s[i] as s[i] is broadcast;
//   backward s[i] -= H[j][i] s[j] for j = i+1 .. nv-1 ascending, then / H[i][i]
//            -- lane j forms its product H[j][i] s[j] (the oracle's product),
//            and the subtractions run in the oracle's order on broadcasts.
template <class R>
__device__ inline void chol_solve_wave(int nv, int tid, const R* H, const R* grad, R* search) {
  const bool own = tid < nv;
  const R dg = own ? H[tid * nv + tid] : (R)1.0;
  const R rg = rcp_ref(dg);
  const R g = own ? grad[tid] : (R)0.0;
  R acc = 0, sv = 0;
  R h = own ? H[tid * nv] : (R)0.0;  // column 0 of lane tid's row
  for (int i = 0; i < nv; i++) {
    const R hn = (own && i + 1 < nv) ? H[tid * nv + i + 1] : (R)0.0;  // next column, off the chain
    const R q = div_ref_lane_rt(i ? g - acc : g, dg, rg, i);
    const R si = bcast(q, i);
    sv = tid == i ? si : sv;
    acc += h * si;
    h = hn;
  }
  R sb = 0;
  R hc = own ? H[tid * nv + nv - 1] : (R)0.0;  // H[tid][i] for i = nv-1
  for (int i = nv - 1; i >= 0; i--) {
    const R hcn = (own && i > 0) ? H[tid * nv + i - 1] : (R)0.0;
    R t = bcast(sv, i);
    const R pr = (own && tid > i) ? hc * sb : (R)0.0;
#pragma unroll 4
    for (int j = i + 1; j < nv; j++) t -= bcast(pr, j);
    const R q = div_ref_lane_rt(t, bcast(dg, i), bcast(rg, i), 0);
    sb = tid == i ? q : sb;
    hc = hcn;
  }
  team_sync();
  if (own) search[tid] = -sb;
  team_sync();
}

// chol_solve_wave for RMAX < nv <= 32 with compile-time step indices: the same
// lanes and operations (lane t: row t's running dot product, column t's
// product in the backward pass), but every broadcast reads an immediate lane,
// the next step's matrix entries are loaded a step ahead, and the divisor of
// each backward step is broadcast from its lane with its reciprocal ready.
// A handful of VGPRs: no per-row register arrays (register-light for the
// large generic kernels).
template <int NC = 0, class R>
__device__ inline void chol_solve_u2(int nv_rt, int tid, const R* H, const R* grad, R* search) {
  constexpr int NM = NC > 0 ? NC : 32;
  const int nv = NC > 0 ? NC : nv_rt;
  const bool own = tid < nv;
  const R dg = own ? H[tid * nv + tid] : (R)1.0;
  const R rg = rcp_ref(dg);
  const R g = own ? grad[tid] : (R)0.0;
  R acc = 0, sv = 0;
  R h = own ? H[tid * nv] : (R)0.0;
  sfor<0, NM>(SLAM(ii) {
    constexpr int i = SK(ii);
    if (i >= nv) return;
    const R hn = (own && i + 1 < nv) ? H[tid * nv + i + 1] : (R)0.0;
    const R a = bcast(i ? g - acc : g, i);
    const R si = div_u(a, bcast(dg, i), bcast(rg, i));
    sv = tid == i ? si : sv;
    acc += h * si;
    h = hn;
  });
  R sb = 0;
  R hc = own ? H[tid * nv + nv - 1] : (R)0.0;
  sfor<0, NM>(SLAM(kk) {
    constexpr int i = NM - 1 - SK(kk);
    if (i >= nv) return;
    const R hcn = (own && i > 0) ? H[tid * nv + i - 1] : (R)0.0;
    const R pr = (own && tid > i) ? hc * sb : (R)0.0;
    R t = bcast(sv, i);
    sfor<i + 1, NM>(SLAM(jj) {
      constexpr int j = SK(jj);
      if (j < nv) t -= bcast(pr, j);
    });
    const R q = div_u(t, bcast(dg, i), bcast(rg, i));
    sb = tid == i ? q : sb;
    hc = hcn;
  });
  team_sync();
  if (own) search[tid] = -sb;
  team_sync();
}


// The substitution of chol_solve_wave for RMAX < nv <= 32 with the solution
// wave-uniform in registers.  Forward as there (lane t accumulates row t's dot
// product as each s[i] is formed; s[i] itself is computed on every lane from
// the broadcast numerator, so it needs no broadcast of its own).  Backward,
// the oracle's chain s[i] -= H[j][i] s[j] (j ascending) runs on every lane on
// uniform operands: H[j][i] by broadcast LDS reads, which depend on nothing
// on the chain and are issued ahead, so the chain is one subtraction per term
// and the division's tail per row -- no v_readlane on it.
template <class R>
__device__ inline void chol_solve_rows32(int nv, int tid, const R* H, const R* grad, R* search) {
  constexpr int NM = 32;
  const bool own = tid < nv;
  R row[NM];
  sfor<0, NM>(SLAM(jj) {
    constexpr int j = SK(jj);
    row[j] = (own && j < nv && j < tid) ? H[tid * nv + j] : (R)0.0;
  });
  const R g = own ? grad[tid] : (R)0.0;
  R acc = 0, out = 0;
  R s[NM];
  sfor<0, NM>(SLAM(ii) {
    constexpr int i = SK(ii);
    if (i >= nv) {
      s[i] = 0;
      return;
    }
    const R d = H[i * nv + i];
    const R a = bcast(i ? g - acc : g, i);
    s[i] = div_u(a, d, rcp_ref(d));
    acc += row[i] * s[i];
  });
  sfor<0, NM>(SLAM(kk) {
    constexpr int i = NM - 1 - SK(kk);
    if (i >= nv) return;
    R t = s[i];
    sfor<i + 1, NM>(SLAM(jj) {
      constexpr int j = SK(jj);
      if (j < nv) t -= H[j * nv + i] * s[j];
    });
    const R d = H[i * nv + i];
    s[i] = div_u(t, d, rcp_ref(d));
    out = tid == i ? s[i] : out;
  });
  team_sync();
  if (own) search[tid] = -out;
  team_sync();
}

}  // namespace coop
}  // namespace ilqg
