// initV + Riccati backward pass (inc/ilqr.h:100-107,133-176) for one seed on
// one 64-lane wavefront, every matrix LDS-resident: the body of k_backward
// (riccati.hip) and the backward role of the fused FD sweep (kernels_coop.hip),
// which streams the FD records in as the sweep publishes them.
//
// Same loops, same summation order as oracle/ilqr_ora.c ora_riccati_step, so
// K, k, V, v are bit-identical to the oracle.  Templated on (NV, NU): the
// bundled models' sizes get compile-time loop bounds and index arithmetic;
// <0,0> is the generic instance.  Square matrices use a padded leading
// dimension nx+1 so the strided column walks spread over the LDS banks.
#pragma once
#include <hip/hip_runtime.h>

#include "dphys.h"
#include "handoff.h"
#include "kernels.h"

#ifndef BSTAMP
#define BSTAMP(id) \
  do {             \
  } while (0)
#endif

#include "riccati_reg.h"

namespace ilqg {

constexpr int BW_THREADS = 64;  // one wavefront: its barriers compile to nothing
constexpr int BW_PF = 8;        // prefetch registers per lane: D <= 512


// Eigen-style LDLT with symmetric pivoting (oracle ora_ldlt_factor); lane 0.
// temp: n doubles of LDS scratch (a private array would live in scratch memory)
__device__ inline void ldlt_factor(int n, double* mat, int* transp, double* temp) {
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
// The same factorization by one wavefront (lane = the calling thread's lane,
// every lane of the wave calls it; n <= 32): each matrix entry receives
// exactly ldlt_factor's operations in ldlt_factor's order -- the pivot scan,
// the four swap groups (disjoint entries: one lane each), temp, the dot
// products of row k and of every row below it (one lane per row, ascending j)
// and the column scaling -- so the factor is bit-identical; the phases of
// column k are separated by wavefront-scope barriers.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ inline void ldlt_factor_wave(int n, double* mat, int* transp, double* temp, int lane) {
  for (int k = 0; k < n; k++) {
    // pivot: the first row of largest |diagonal| among k..n-1 (strict >, as the oracle)
    const double dg = (lane >= k && lane < n) ? fabs(mat[lane + lane * n]) : 0.0;
    int big = k;
    double bigv = __shfl(dg, k);
    for (int i = k + 1; i < n; i++) {
      const double a = __shfl(dg, i);
      if (a > bigv) {
        bigv = a;
        big = i;
      }
    }
    if (lane == 0) transp[k] = big;
    if (k != big) {
      const int s = n - big - 1;
      double t;
      if (lane < k) {  // row k <-> row big, columns j < k
        const int j = lane;
        t = mat[k + j * n]; mat[k + j * n] = mat[big + j * n]; mat[big + j * n] = t;
      }
      if (lane < s) {  // rows below big: column k <-> column big
        const int i = lane;
        t = mat[(big + 1 + i) + k * n];
        mat[(big + 1 + i) + k * n] = mat[(big + 1 + i) + big * n];
        mat[(big + 1 + i) + big * n] = t;
      }
      if (lane == 32) {
        t = mat[k + k * n]; mat[k + k * n] = mat[big + big * n]; mat[big + big * n] = t;
      }
      if (lane > 32 + k && lane < 32 + big) {  // between: column k <-> row big
        const int i = lane - 32;
        t = mat[i + k * n]; mat[i + k * n] = mat[big + i * n]; mat[big + i * n] = t;
      }
    }
    wave_sync();
    if (k > 0) {
      if (lane < k) temp[lane] = mat[lane + lane * n] * mat[k + lane * n];
      wave_sync();
      // lane i >= k: row i's dot with temp (row k: the diagonal update)
      if (lane >= k && lane < n) {
        double si = 0;
        for (int j = 0; j < k; j++) si += mat[lane + j * n] * temp[j];
        mat[lane + k * n] -= si;
      }
      wave_sync();
    }
    if (k == 0 && !(fabs(mat[0]) > 0)) {
      for (int j = lane; j < n; j += 64) transp[j] = j;
      wave_sync();
      return;
    }
    const double d = mat[k + k * n];
    if (n - k - 1 > 0 && fabs(d) > 0 && lane > k && lane < n) mat[lane + k * n] /= d;
    wave_sync();
  }
}

__device__ inline void ldlt_solve(int n, const double* Lm, const int* transp, double* x) {
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

// ldlt_solve with the vector in registers (n <= 32, every index a compile-time
// constant): the pivot swaps before and after the substitutions are one
// gather and one scatter through perm (ldlt_perm), and every entry receives
// ldlt_solve's operations in ldlt_solve's order.  Lm reads are uniform LDS
// loads independent of x, so they issue ahead of the dependent chain.
// Each calling lane solves its own vector x (active lanes only).
// perm[i] = the source position of entry i after ldlt_solve's forward swaps:
// lane i applies the transpositions to its index, last one first
__device__ inline void ldlt_perm(int n, const int* transp, int* perm, int lane) {
  if (lane < n) {
    int p = lane;
    for (int k = n - 1; k >= 0; k--) {
      const int t = transp[k];
      p = p == k ? t : (p == t ? k : p);
    }
    perm[lane] = p;
  }
}
__device__ inline void ldlt_solve_reg(int n, const double* Lm, const int* perm, double* x, bool active) {
  constexpr int NM = 32;
  const double tol = 2.2250738585072014e-308;
  double r[NM];
  rreg::sf<0, NM>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    r[i] = (active && i < n) ? x[perm[i]] : 0.0;
  });
  rreg::sf<0, NM>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    if (i < n)
      rreg::sf<0, i>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        r[i] -= Lm[i + j * n] * r[j];
      });
  });
  rreg::sf<0, NM>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    if (i < n) {
      const double d = Lm[i + i * n];
      r[i] = fabs(d) > tol ? r[i] / d : 0.0;
    }
  });
  rreg::sf<0, NM>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = NM - 1 - decltype(ii)::value;
    if (i < n)
      rreg::sf<i + 1, NM>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        if (j < n) r[i] -= Lm[j + i * n] * r[j];
      });
  });
  rreg::sf<0, NM>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    if (active && i < n) x[perm[i]] = r[i];
  });
}

// ldlt_factor_wave and ldlt_solve_reg for a compile-time size N (the MFMA
// engine's humanoid instance, nu = 21): every loop unrolled, no size guards.
// The pivot scan is a wave max-reduction instead of the serial shuffle chain:
// |diagonal| >= 0, so its IEEE bits order like the values; rows whose
// |diagonal| is NaN take key 0 (the strict > of the scan never picks them), a
// NaN at row k keeps k (the scan never moves), and the first row attaining the
// maximum is the scan's choice (a tie at key 0 includes row k itself).
// max(x, x rotated right by S lanes within its 16-lane row) (DPP row_ror)
template <int S>
__device__ __forceinline__ unsigned long long umax_ror(unsigned long long x) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)x, 0x120 + S, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(x >> 32), 0x120 + S, 0xf, 0xf, false);
  const unsigned long long y = ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
  return y > x ? y : x;
}
__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long x, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
template <int N>
__device__ inline void ldlt_factor_wave_t(double* mat, int* transp, double* temp, int lane) {
  static_assert(N >= 1 && N <= 32, "one wavefront, n <= 32");
  bool stop = false;
  rreg::sf<0, N>([&](auto kk) __attribute__((always_inline)) {
    constexpr int k = decltype(kk)::value;
    if (stop) return;
    const bool in = lane >= k && lane < N;
    const int li = lane < N ? lane : N - 1;
    const double dg = fabs(mat[li + li * N]);
    unsigned long long key = (in && dg == dg) ? (unsigned long long)__double_as_longlong(dg) : 0ull;
    // max over each 16-lane row by DPP row rotations, then rows 0 and 1 (n <= 32)
    key = umax_ror<8>(key);
    key = umax_ror<4>(key);
    key = umax_ror<2>(key);
    key = umax_ror<1>(key);
    const unsigned long long m0 = readlane_u64(key, 0), m1 = readlane_u64(key, 16);
    const unsigned long long kmax = m1 > m0 ? m1 : m0;
    const double dk = fabs(mat[k + k * N]);
    int big = k;
    if (dk == dk) {
      const unsigned long long hit = __ballot(in && dg == dg && (unsigned long long)__double_as_longlong(dg) == kmax);
      // kmax == 0: every candidate is 0 or NaN, row k (0) the first of them
      if (kmax != 0ull) big = (int)__builtin_ctzll(hit);
    }
    if (lane == 0) transp[k] = big;
    if (k != big) {
      const int s = N - big - 1;
      double t;
      if (lane < k) {  // row k <-> row big, columns j < k
        const int j = lane;
        t = mat[k + j * N]; mat[k + j * N] = mat[big + j * N]; mat[big + j * N] = t;
      }
      if (lane < s) {  // rows below big: column k <-> column big
        const int i = lane;
        t = mat[(big + 1 + i) + k * N];
        mat[(big + 1 + i) + k * N] = mat[(big + 1 + i) + big * N];
        mat[(big + 1 + i) + big * N] = t;
      }
      if (lane == 32) {
        t = mat[k + k * N]; mat[k + k * N] = mat[big + big * N]; mat[big + big * N] = t;
      }
      if (lane > 32 + k && lane < 32 + big) {  // between: column k <-> row big
        const int i = lane - 32;
        t = mat[i + k * N]; mat[i + k * N] = mat[big + i * N]; mat[big + i * N] = t;
      }
    }
    wave_sync();
    if constexpr (k > 0) {
      if (lane < k) temp[lane] = mat[lane + lane * N] * mat[k + lane * N];
      wave_sync();
      // lane i >= k: row i's dot with temp (row k: the diagonal update), ascending j
      double a[k], b[k];
      rreg::sf<0, k>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        a[j] = mat[li + j * N];
        b[j] = temp[j];
      });
      double si = 0;
      rreg::sf<0, k>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        si += a[j] * b[j];
      });
      if (in) mat[lane + k * N] -= si;
      wave_sync();
    }
    if constexpr (k == 0) {
      if (!(fabs(mat[0]) > 0)) {
        for (int j = lane; j < N; j += 64) transp[j] = j;
        wave_sync();
        stop = true;
        return;
      }
    }
    if constexpr (N - k - 1 > 0) {
      const double d = mat[k + k * N];
      if (fabs(d) > 0 && lane > k && lane < N) mat[lane + k * N] /= d;
    }
    wave_sync();
  });
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
  return __longlong_as_double((long long)readlane_u64((unsigned long long)__double_as_longlong(x), l));
}
// ldlt_factor_wave_t's factor with the matrix in registers, one row per lane.
// ldlt_factor's pivot scan reads the diagonal entries of rows k..n-1, which no
// earlier column has updated (entry (k, k) is updated at step k), so the pivot
// sequence is a function of the input's diagonal alone: it is replayed first
// (lane q holds the key of the row at position q; ldlt_factor_wave_t's scan and
// row swaps on the keys), which also yields the rows' final order -- perm,
// what ldlt_perm derives from transp.  Lane i then holds row perm[i] of the
// (lower-triangle) symmetric input in that order and forms column k with
// ldlt_factor's operations in ldlt_factor's order: temp[j] = D[j] L(k, j)
// (lane k's products, read across the wave with v_readlane), the row's dot
// product with temp ascending from +0, its subtraction from the input entry,
// the division by the updated diagonal.  The factor is the same bit for bit
// (tests/test_gpu_parity.py::test_ldlt_reg_matches_lds); a NaN or an all-zero
// diagonal (ldlt_factor's early exit) takes ldlt_factor_wave_t + ldlt_perm.
// Writes the lower triangle and diagonal of mat, transp and perm.
// (replay: the replay even without equal keys, for the test)
template <int N>
__device__ inline void ldlt_factor_reg_t(double* mat, int* transp, int* perm, double* temp, int lane,
                                         bool replay = false) {
  static_assert(N >= 1 && N <= 32, "one wavefront, n <= 32");
  const int li = lane < N ? lane : N - 1;
  const double dg = fabs(mat[li + li * N]);
  const unsigned long long key0 = lane < N ? (unsigned long long)__double_as_longlong(dg) : 0ull;
  if (__ballot(lane < N && dg != dg) != 0ull || __ballot(lane < N && dg > 0) == 0ull) {
    ldlt_factor_wave_t<N>(mat, transp, temp, lane);
    ldlt_perm(N, transp, perm, lane);
    return;
  }
  // the pivot sequence.  Distinct keys: the scan picks the largest remaining
  // key whatever the rows' positions, so the order is the rows by |diagonal|
  // descending -- each lane counts the keys above its own.  Equal keys (the
  // first in the current order wins, and the swaps reorder the rest): the scan
  // and its swaps replayed on the keys, lane q holding position q's row and key.
  int rank = 0;
  bool tie = false;
  rreg::sf<0, N>([&](auto jj) __attribute__((always_inline)) {
    constexpr int j = decltype(jj)::value;
    const double dj = fabs(mat[j + j * N]);
    rank += dj > dg ? 1 : 0;
    tie = tie || (lane < N && lane != j && dj == dg);
  });
  int pos;
  if (__ballot(tie) == 0ull && !replay) {
    if (lane < N) perm[rank] = lane;
    wave_sync();
    pos = lane < N ? perm[lane] : 0;
  } else {
    pos = lane < N ? lane : 0;
    unsigned long long ky = key0;
    rreg::sf<0, N>([&](auto kk) __attribute__((always_inline)) {
      constexpr int k = decltype(kk)::value;
      const bool in = lane >= k && lane < N;
      unsigned long long key = in ? ky : 0ull;
      key = umax_ror<8>(key);
      key = umax_ror<4>(key);
      key = umax_ror<2>(key);
      key = umax_ror<1>(key);
      const unsigned long long m0 = readlane_u64(key, 0), m1 = readlane_u64(key, 16);
      const unsigned long long kmax = m1 > m0 ? m1 : m0;
      const unsigned long long hit = __ballot(in && ky == kmax);
      const int big = kmax != 0ull ? (int)__builtin_ctzll(hit) : k;
      if (big != k) {
        const unsigned long long kb = readlane_u64(ky, big), kk0 = readlane_u64(ky, k);
        const int pb = __builtin_amdgcn_readlane(pos, big), pk = __builtin_amdgcn_readlane(pos, k);
        if (lane == k) {
          ky = kb;
          pos = pb;
        } else if (lane == big) {
          ky = kk0;
          pos = pk;
        }
      }
    });
    if (lane < N) perm[lane] = pos;
  }
  // row pos of the symmetric input, columns in the final order (all reads issue
  // before the first write below)
  double a[N];
  rreg::sf<0, N>([&](auto cc) __attribute__((always_inline)) {
    constexpr int c = decltype(cc)::value;
    const int pc = __builtin_amdgcn_readlane(pos, c);
    const int hi = pos > pc ? pos : pc, lo = pos > pc ? pc : pos;
    a[c] = mat[hi + lo * N];
  });
  // the column loop is one basic block (no stores, no branches), so the
  // scheduler can start column k's dot products beside column k-1's division
  double l[N], dl[N];  // L(i, j); D[j] L(i, j)
  double dd = 0;       // lane i: D[i]
  rreg::sf<0, N>([&](auto kk) __attribute__((always_inline)) {
    constexpr int k = decltype(kk)::value;
    double v = a[k];
    if constexpr (k > 0) {
      double si = 0;
      rreg::sf<0, k>([&](auto jj) __attribute__((always_inline)) {
        constexpr int j = decltype(jj)::value;
        si += l[j] * readlane_f64(dl[j], k);
      });
      v -= si;
    }
    const double d = readlane_f64(v, k);
    dd = lane == k ? d : dd;
    if constexpr (N - k - 1 > 0) {
      const double lk = fabs(d) > 0 ? v / d : v;
      l[k] = lk;
      dl[k] = d * lk;
    }
  });
  // column j of lane i: L(i, j) below the diagonal; the lanes above it write
  // their (unused) values into the upper triangle, which nothing reads; the
  // diagonal last
  if (lane < N) {
    rreg::sf<0, N - 1>([&](auto jj) __attribute__((always_inline)) {
      constexpr int j = decltype(jj)::value;
      mat[lane + j * N] = l[j];
    });
    mat[lane + lane * N] = dd;
  }
}
// a zero the compiler cannot see through, produced after v: L reads addressed
// with it cannot be hoisted above v's computation (left free, the scheduler
// issues all N^2 reads of an unrolled solve at once and the kernel spills)
__device__ __forceinline__ int zero_after(double v) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z) : "v"(v));
  return z;
}
template <int N>
__device__ inline void ldlt_solve_reg_t(const double* Lm, const int* perm, const double* src, double* x, bool dbl,
                                        bool active) {
  const double tol = 2.2250738585072014e-308;
  double r[N];
  // the right-hand side src (2 src when dbl: the caller's doubling, exact),
  // solved into x
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    const double b = active ? src[perm[i]] : 0.0;
    r[i] = dbl ? 2 * b : b;
  });
  // forward substitution column by column: r[i] -= L(i, j) r[j] for i > j --
  // each r[i] still receives its subtractions in ascending j, ldlt_solve's
  // order.  Column j's L reads wait for r[j - 1] (final one column earlier):
  // they overlap the previous column's updates, no further ahead.
  rreg::sf<0, N>([&](auto jj) __attribute__((always_inline)) {
    constexpr int j = decltype(jj)::value;
    const double* Lc = Lm + (j > 0 ? zero_after(r[j > 0 ? j - 1 : 0]) : 0);
    rreg::sf<j + 1, N>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      r[i] -= Lc[i + j * N] * r[j];
    });
  });
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    const double d = Lm[i + i * N];
    r[i] = fabs(d) > tol ? r[i] / d : 0.0;
  });
  // backward rows, i descending: row i's reads wait for r[i + 2]
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = N - 1 - decltype(ii)::value;
    const double* Lc = Lm + (i + 2 < N ? zero_after(r[i + 2 < N ? i + 2 : 0]) : 0);
    rreg::sf<i + 1, N>([&](auto jj) __attribute__((always_inline)) {
      constexpr int j = decltype(jj)::value;
      r[i] -= Lc[j + i * N] * r[j];
    });
  });
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    if (active) x[perm[i]] = r[i];
  });
}

// x, copied once dep is computed (the copy cannot move above dep)
__device__ __forceinline__ double copy_after(double x, double dep) {
  double y;
  asm volatile("v_mov_b64 %0, %1" : "=v"(y) : "v"(x), "v"(dep));
  return y;
}
// ldlt_solve_reg_t with the factor read across the wave instead of from LDS:
// lane i holds row i of the factor (L(i, j), j < i, and D(i)) in registers,
// loaded once, and every use of L(i, j) is a v_readlane of lane i's register j
// into scalar registers -- no LDS load, so no LDS latency, on the
// substitutions' dependent chain.  The same operations in the same order.
template <int N>
__device__ inline void ldlt_solve_bcast_t(const double* Lm, const int* perm, const double* src, double* x, bool dbl,
                                          bool active, int lane) {
  const double tol = 2.2250738585072014e-308;
  const int li = lane < N ? lane : 0;
  double Lr[N];  // row li of the factor (its upper part unused)
  rreg::sf<0, N>([&](auto jj) __attribute__((always_inline)) {
    constexpr int j = decltype(jj)::value;
    Lr[j] = Lm[li + j * N];
  });
  double r[N];
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    const double b = active ? src[perm[i]] : 0.0;
    r[i] = dbl ? 2 * b : b;
  });
  // (column j's reads are issued once r[j - 1] is final, row i's once r[i + 2]
  // is: left free, the scheduler hoists every read into scalar registers and
  // spills them -- as zero_after does for ldlt_solve_reg_t's LDS reads)
  rreg::sf<0, N>([&](auto jj) __attribute__((always_inline)) {
    constexpr int j = decltype(jj)::value;
    const double Lc = j > 0 ? copy_after(Lr[j], r[j > 0 ? j - 1 : 0]) : Lr[j];
    rreg::sf<j + 1, N>([&](auto ii) __attribute__((always_inline)) {
      constexpr int i = decltype(ii)::value;
      r[i] -= readlane_f64(Lc, i) * r[j];
    });
  });
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    const double d = readlane_f64(Lr[i], i);
    r[i] = fabs(d) > tol ? r[i] / d : 0.0;
  });
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = N - 1 - decltype(ii)::value;
    const double Lc = i + 2 < N ? copy_after(Lr[i], r[i + 2 < N ? i + 2 : 0]) : Lr[i];
    rreg::sf<i + 1, N>([&](auto jj) __attribute__((always_inline)) {
      constexpr int j = decltype(jj)::value;
      r[i] -= readlane_f64(Lc, j) * r[j];
    });
  });
  rreg::sf<0, N>([&](auto ii) __attribute__((always_inline)) {
    constexpr int i = decltype(ii)::value;
    if (active) x[perm[i]] = r[i];
  });
}

// Three independent fixed-order dot products per lane (ILP 3): each output
// keeps the oracle's summation order, the three chains overlap in the pipe.
#define ILP3_BEGIN(n)                                    \
  for (int e0 = tid; e0 < (n); e0 += 3 * BW_THREADS) {   \
    const int e1 = e0 + BW_THREADS, e2 = e0 + 2 * BW_THREADS; \
    const bool h1 = e1 < (n), h2 = e2 < (n);             \
    const int f1 = h1 ? e1 : e0, f2 = h2 ? e2 : e0;

template <int NV_, int NU_, class MD>
__device__ inline void backward_seed(const MD& m, int nq, int nv_rt, int nu_rt, int P, double dt, double mu,
                                     const double* deriv, int Ds, TrajDev tr, double* Kg, double* kg, double* Vg,
                                     double* vg, int s, int tid, double* sh, const unsigned* done, unsigned target,
                                     unsigned* fault, RicFlags fl) {
#ifndef ILQG_RIC_LDS
  // bundled small models: the register/exchange formulation (riccati_reg.h)
  if constexpr (RicReg<NV_, NU_>::ok) {
    if (nq == NV_) {
      backward_seed_reg<NV_, NU_>(m, P, dt, mu, deriv, Ds, tr, Kg, kg, Vg, vg, s, tid, sh, done, target, fault, fl);
      return;
    }
  }
#endif
  const int nv = NV_ > 0 ? NV_ : nv_rt;
  const int nu = NU_ > 0 ? NU_ : nu_rt;
  const int nx = 2 * nv, D = nv * (2 * nv + nu) + 2 * nv + nu;
  // padded leading dimension of the nx-row matrices (unpadded for large nx,
  // where LDS capacity binds)
  const int LX = nx <= 32 ? nx + 1 : nx;
  // FD record prefetched into LDS (always, when streaming from the FD sweep)
  const bool pref = D <= BW_PF * BW_THREADS;
  // streaming (done != nullptr): record p is read only once its FD teams have
  // all published it (done[s P + p] >= target), with sc1 loads
  // (the flags of records up to ready_upto were seen published by an earlier poll)
  int ready_upto = -1;
  auto ready = [&](int p) {
    if (!done || p <= ready_upto) return;
#ifdef ILQG_STAMPS
    const unsigned long long t0_ = __builtin_amdgcn_s_memtime();
#endif
    ready_upto = bw_wait_window(done + (size_t)s * P, p, P, target, fault);
#ifdef ILQG_STAMPS
    if (s == 0 && tid == 0) {
      g_fused_diag[1] += __builtin_amdgcn_s_memtime() - t0_;
      g_fused_diag[2]++;
    }
    if (s < 8 && tid == 0) g_fused_diag[16 + s] += __builtin_amdgcn_s_memtime() - t0_;
#endif
  };
  auto ld = [&](const double* a) -> double { return done ? ld_sc1(a) : *a; };
  // buffers are reused once dead: V holds V_new (V is read only by stage 1),
  // A holds T4 (A is last read in stage 5)
  double* V = sh;                 // nx x nx, ld LX; V_new from stage 7
  double* Vs = V + nx * LX;
  double* A = Vs + nx * LX;       // T4 from stage 6
  double* ABK = A + nx * LX;
  double* B = ABK + nx * LX;      // nx x nu, ld LX
  double* T6 = B + nu * LX;       // nx x nu, ld LX
  double* T1 = T6 + nu * LX;      // nu x nx, ld nu
  double* T3 = T1 + nu * nx;
  double* Kl = T3 + nu * nx;
  double* Mm = Kl + nu * nx;      // nu x nu
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
  double* dl = r + nu;  // FD record of the current step (prefetched), D doubles when pref
  int* trn = (int*)(dl + (pref ? D : 0));
  double* T4 = A;
  double* Vn = V;
#ifdef ILQG_STAMPS
  unsigned long long bst_prev = 0;
#endif

  // initV at the terminal point dArray[0], inc/ilqr.h:100-107
  {
    ready(0);
    const double* q0 = deriv + ((size_t)s * P + 0) * Ds + 2 * nv * nv + nv * nu;
    // v0 = dgdx at the terminal point, or the caller's (an initV override)
    for (int i = tid; i < nx; i += BW_THREADS) v[i] = fl.vinit ? vg[(size_t)s * nx + i] : ld(q0 + i);
    ready(P > 1 ? 1 : 0);
    const double* d1 = deriv + ((size_t)s * P + (P > 1 ? 1 : 0)) * Ds;
    if (pref)
      for (int i = tid; i < D; i += BW_THREADS) dl[i] = ld(d1 + rec_src(i, nv, nu, fl.layout));
    __syncthreads();
    for (int e = tid; e < nx * nx; e += BW_THREADS) {
      int i = e % nx, j = e / nx;
      V[i + j * LX] = fl.vinit ? Vg[(size_t)s * nx * nx + e] : v[i] * v[j];
    }
    __syncthreads();
  }
  BSTAMP(-1);
  // the nominal states for c = x*_{n-1} - x*_n: one lane per component, in
  // registers, each point loaded one step ahead (nq == nv; quaternion models
  // take the tangent-space difference from memory below)
  const bool xreg = nq == nv && nx <= BW_THREADS;
  auto xload = [&](size_t pt) -> double {
    return tid < nv ? tr.qpos[pt * nq + tid] : (tid < nx ? tr.qvel[pt * nv + tid - nv] : 0.0);
  };
  double xa = 0, xb = 0;
  if (xreg) {
    xa = xload((size_t)s * P);
    if (P > 1) xb = xload((size_t)s * P + 1);
  }
  for (int n = 1; n < P; n++) {
    const size_t pc = (size_t)s * P + n, pp = pc - 1;
    double xn = 0;
    if (xreg && n + 1 < P) xn = xload(pc + 1);
    // prefetch the next step's FD record; consumed at the end of this step
    double pf[BW_PF];
    if (pref && n + 1 < P) {
      ready(n + 1);
      const double* dn1 = deriv + (pc + 1) * Ds;
#pragma unroll
      for (int t = 0; t < BW_PF; t++) {
        int i = tid + t * BW_THREADS;
        pf[t] = i < D ? ld(dn1 + rec_src(i, nv, nu, fl.layout)) : 0.0;
      }
    }
    const double* dn0 = pref ? dl : deriv + pc * Ds;
    // record entry e as the recursion reads it (staged records are already in the layout)
    const int lay = pref ? 0 : fl.layout;
    auto dn = [&](int e) -> double { return dn0[rec_src(e, nv, nu, lay)]; };
    // stage 1: symmetrise V, assemble A/B (differentiator.h:66-71,89-92), q, r, c
    for (int e = tid; e < nx * nx; e += BW_THREADS) {
      int i = e % nx, j = e / nx;
      Vs[i + j * LX] = (V[i + j * LX] + V[j + i * LX]) / 2;
      double val;
      if (i < nv && j < nv) val = (i == j) ? 1 : 0;
      else if (i < nv) val = (i == j - nv) ? dt : 0;
      else if (j < nv) val = dn((i - nv) + j * nv) * dt;
      else val = ((i - nv) == (j - nv) ? 1 : 0) + dn(nv * nv + (i - nv) + (j - nv) * nv) * dt;
      A[i + j * LX] = val;
    }
    for (int e = tid; e < nx * nu; e += BW_THREADS) {
      int i = e % nx, j = e / nx;
      B[i + j * LX] = (i < nv) ? 0 : dn(2 * nv * nv + (i - nv) + j * nv) * dt;
    }
    for (int i = tid; i < nx; i += BW_THREADS) {
      q[i] = dn(2 * nv * nv + nv * nu + i);
      // c = x*_{n-1} (-) x*_n (inc/ilqr.h:154-157; tangent space for quaternion joints)
      if (xreg) {
        c[i] = xa - xb;  // i == tid
      } else if (i < nv && nq != nv) {
        c[i] = dev::state_diff_dof(m, i, tr.qpos + pp * nq, tr.qpos + pc * nq);
      } else {
        double xp = i < nv ? tr.qpos[pp * nq + i] : tr.qvel[pp * nv + i - nv];
        double xc = i < nv ? tr.qpos[pc * nq + i] : tr.qvel[pc * nv + i - nv];
        c[i] = xp - xc;
      }
    }
    for (int a = tid; a < nu; a += BW_THREADS) r[a] = dn(2 * nv * nv + nv * nu + nx + a);
    __syncthreads();
    for (int i = tid; i < nx; i += BW_THREADS) Vs[i + i * LX] += mu;
    __syncthreads();
    BSTAMP(0);
    // stage 2: T1 = B'V
    ILP3_BEGIN(nu * nx)
      double s0 = 0, s1 = 0, s2 = 0;
      const int a0 = e0 % nu, j0 = e0 / nu, a1 = f1 % nu, j1 = f1 / nu, a2 = f2 % nu, j2 = f2 / nu;
      for (int kk = 0; kk < nx; kk++) {
        s0 += B[kk + a0 * LX] * Vs[kk + j0 * LX];
        s1 += B[kk + a1 * LX] * Vs[kk + j1 * LX];
        s2 += B[kk + a2 * LX] * Vs[kk + j2 * LX];
      }
      T1[e0] = s0;
      if (h1) T1[e1] = s1;
      if (h2) T1[e2] = s2;
    }
    __syncthreads();
    BSTAMP(1);
    // stage 3: Mm = -2 T1 B - 2R ; T3 = T1 A ; w = v + 2 V c
    for (int e = tid; e < nu * nu; e += BW_THREADS) {
      int a = e % nu, b = e / nu;
      double sm = 0;
      for (int kk = 0; kk < nx; kk++) sm += T1[a + kk * nu] * B[kk + b * LX];
      Mm[e] = -2 * sm - 2 * (r[a] * r[b]);
    }
    ILP3_BEGIN(nu * nx)
      double s0 = 0, s1 = 0, s2 = 0;
      const int a0 = e0 % nu, j0 = e0 / nu, a1 = f1 % nu, j1 = f1 / nu, a2 = f2 % nu, j2 = f2 / nu;
      for (int kk = 0; kk < nx; kk++) {
        s0 += T1[a0 + kk * nu] * A[kk + j0 * LX];
        s1 += T1[a1 + kk * nu] * A[kk + j1 * LX];
        s2 += T1[a2 + kk * nu] * A[kk + j2 * LX];
      }
      T3[e0] = s0;
      if (h1) T3[e1] = s1;
      if (h2) T3[e2] = s2;
    }
    for (int i = tid; i < nx; i += BW_THREADS) {
      double sm = 0;
      for (int j = 0; j < nx; j++) sm += Vs[i + j * LX] * c[j];
      w[i] = v[i] + 2 * sm;
    }
    __syncthreads();
    ldlt_factor_wave(nu, Mm, trn, y, tid);  // y is free until stage 5
    for (int a = tid; a < nu; a += BW_THREADS) {
      double sm = 0;
      for (int kk = 0; kk < nx; kk++) sm += B[kk + a * LX] * w[kk];
      col[a] = sm + r[a];
    }
    __syncthreads();
    BSTAMP(2);
    // stage 4: K = ldlt.solve(2 T3) column-parallel; k = ldlt.solve(B'w + r), in place in LDS
    int* perm = trn + nu;
    ldlt_perm(nu, trn, perm, tid);
    for (int j = tid; j < nx + 1; j += BW_THREADS) {
      double* x = j < nx ? Kl + j * nu : kl;
      if (j < nx)
        for (int a = 0; a < nu; a++) x[a] = 2 * T3[a + j * nu];
      else
        for (int a = 0; a < nu; a++) x[a] = col[a];
    }
    __syncthreads();
    if (nu <= 32 && nx + 1 <= BW_THREADS) {
      const int j = tid;
      ldlt_solve_reg(nu, Mm, perm, j < nx ? Kl + j * nu : kl, j < nx + 1);
    } else {
      for (int j = tid; j < nx + 1; j += BW_THREADS) ldlt_solve(nu, Mm, trn, j < nx ? Kl + j * nu : kl);
    }
    __syncthreads();
    BSTAMP(3);
    // stage 5: ABK = A + B K ; T6 = K'R ; y = Bk + c ; kR = k'R
    for (int e = tid; e < nx * nx; e += BW_THREADS) {
      int i = e % nx, j = e / nx;
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += B[i + a * LX] * Kl[a + j * nu];
      ABK[i + j * LX] = A[i + j * LX] + sm;
    }
    for (int e = tid; e < nx * nu; e += BW_THREADS) {
      int i = e % nx, b = e / nx;
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += Kl[a + i * nu] * (r[a] * r[b]);
      T6[i + b * LX] = sm;
    }
    for (int i = tid; i < nx; i += BW_THREADS) {
      double sm = 0;
      for (int a = 0; a < nu; a++) sm += B[i + a * LX] * kl[a];
      y[i] = sm + c[i];
    }
    for (int b = tid; b < nu; b += BW_THREADS) {
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
        s0 += ABK[kk + i0 * LX] * Vs[kk + j0 * LX];
        s1 += ABK[kk + i1 * LX] * Vs[kk + j1 * LX];
        s2 += ABK[kk + i2 * LX] * Vs[kk + j2 * LX];
      }
      T4[i0 + j0 * LX] = s0;
      if (h1) T4[i1 + j1 * LX] = s1;
      if (h2) T4[i2 + j2 * LX] = s2;
    }
    __syncthreads();
    BSTAMP(5);
    // stage 7: V_new = (T4 ABK + Q) + T6 K
    ILP3_BEGIN(nx * nx)
      double a0s = 0, a1s = 0, a2s = 0, b0s = 0, b1s = 0, b2s = 0;
      const int i0 = e0 % nx, j0 = e0 / nx, i1 = f1 % nx, j1 = f1 / nx, i2 = f2 % nx, j2 = f2 / nx;
      for (int kk = 0; kk < nx; kk++) {
        a0s += T4[i0 + kk * LX] * ABK[kk + j0 * LX];
        a1s += T4[i1 + kk * LX] * ABK[kk + j1 * LX];
        a2s += T4[i2 + kk * LX] * ABK[kk + j2 * LX];
      }
      for (int b = 0; b < nu; b++) {
        b0s += T6[i0 + b * LX] * Kl[b + j0 * nu];
        b1s += T6[i1 + b * LX] * Kl[b + j1 * nu];
        b2s += T6[i2 + b * LX] * Kl[b + j2 * nu];
      }
      Vn[i0 + j0 * LX] = (a0s + q[i0] * q[j0]) + b0s;
      if (h1) Vn[i1 + j1 * LX] = (a1s + q[i1] * q[j1]) + b1s;
      if (h2) Vn[i2 + j2 * LX] = (a2s + q[i2] * q[j2]) + b2s;
    }
    __syncthreads();
    BSTAMP(6);
    // stage 8: z = (2y)' V_new ; v_new (reads the NEW V, Q14)
    for (int j = tid; j < nx; j += BW_THREADS) {
      double sm = 0;
      for (int i = 0; i < nx; i++) sm += (2 * y[i]) * Vn[i + j * LX];
      z[j] = sm;
    }
    __syncthreads();
    for (int j = tid; j < nx; j += BW_THREADS) {
      double ta = 0, tb = 0, td = 0;
      for (int i = 0; i < nx; i++) {
        ta += z[i] * ABK[i + j * LX];
        tb += v[i] * ABK[i + j * LX];
      }
      for (int b = 0; b < nu; b++) td += (2 * kR[b]) * Kl[b + j * nu];
      vn[j] = ((ta + tb) + q[j]) + td;
    }
    BSTAMP(7);
    // gains out
    for (int e = tid; e < nu * nx; e += BW_THREADS) Kg[pc * nu * nx + e] = Kl[e];
    for (int a = tid; a < nu; a += BW_THREADS) kg[pc * nu + a] = kl[a];
    __syncthreads();
    for (int i = tid; i < nx; i += BW_THREADS) v[i] = vn[i];  // V already holds V_new
    if (pref && n + 1 < P) {
#pragma unroll
      for (int t = 0; t < BW_PF; t++) {
        int i = tid + t * BW_THREADS;
        if (i < D) dl[i] = pf[t];
      }
    }
    __syncthreads();
    xa = xb;
    xb = xn;
    BSTAMP(8);
  }
  if (Vg)
    for (int e = tid; e < nx * nx; e += BW_THREADS) {
      int i = e % nx, j = e / nx;
      Vg[(size_t)s * nx * nx + e] = V[i + j * LX];
    }
  if (vg)
    for (int i = tid; i < nx; i += BW_THREADS) vg[(size_t)s * nx + i] = v[i];
}


}  // namespace ilqg
