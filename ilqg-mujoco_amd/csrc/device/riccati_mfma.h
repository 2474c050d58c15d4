// initV + Riccati backward pass (inc/ilqr.h:100-107,133-176) with the matrix
// products on the fp64 matrix cores (v_mfma_f64_16x16x4_f64) -- the
// "MFMA on the Quu/Qux block products where nu x nx is large enough" of the
// north star, for models whose nx x nx products dominate (humanoid: nx = 54,
// nu = 21: 1.23 MFLOP per step).
//
// One workgroup of eight wavefronts (two a SIMD) per seed; every matrix LDS-resident at an
// odd leading dimension (the 16 lanes of an MFMA operand fetch walk a row or a
// column: an odd stride keeps them on distinct banks).  Each product is a set
// of 16x16 output tiles dealt round-robin to the waves; K advances 4 per
// instruction; operands outside a matrix read as 0 (no padding in LDS).
// Stage order and every non-product expression are those of riccati.h
// (oracle/ilqr_ora.c ora_riccati_step); only the order of the additions inside
// each matrix product differs (the matrix core's), so K, k, V, v agree with the
// oracle to rounding, not bit for bit: tests/test_gpu_parity.py states the
// tolerance (ilqg_solver_set_riccati selects this path; the default stays the
// bit-exact one).
#pragma once
#include <hip/hip_runtime.h>

#include "dphys.h"
#include "kernels.h"

namespace ilqg {
namespace rmfma {

// eight wavefronts: two a SIMD, so one wave's LDS operand loads and barrier
// waits overlap the other's MFMAs (cfg 5's recursion 9.0 -> 8.0 ms against
// four, 7.9 -> 9.2 at sixteen, whose 128-VGPR budget spills:
// profiles/r06_mfma_waves.txt); ILQG_MFMA_WAVES rebuilds another count (A/B)
#ifndef ILQG_MFMA_WAVES
#define ILQG_MFMA_WAVES 8
#endif
constexpr int THREADS = 64 * ILQG_MFMA_WAVES;
constexpr int WAVES = THREADS / 64;
constexpr int SOLVE_WAVES = WAVES < 4 ? WAVES : 4;  // stage 5's waves
constexpr int MPF = 4096 / THREADS;  // record prefetch registers per thread: D <= 4096
constexpr int NU_MAX = 32;  // pivoted-LDLT permutation tables (static __shared__ below)
constexpr size_t STATIC_LDS_BYTES = 2 * NU_MAX * sizeof(int);

typedef double d4 __attribute__((ext_vector_type(4)));

// one 16x16 tile of C = sum_k a(i, k) b(k, j), i in [i0, i0+16), j in [j0, j0+16):
// lane l supplies a(i0 + l%16, k0 + l/16) and b(k0 + l/16, j0 + l%16); result
// entry q of lane l is C(i0 + l/16 + 4q, j0 + l%16)
// (k from kb, a multiple of 4: the terms below kb are zero products)
template <class GA, class GB>
__device__ __forceinline__ d4 tile(int i0, int j0, int K, const GA& ga, const GB& gb, int lane, int kb = 0) {
  const int r = lane & 15, kq = lane >> 4;
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  int k0 = kb;
  // four K steps a block: the block's eight operand reads issue together, then
  // its four MFMAs (the same accumulation sequence as one step at a time)
  for (; k0 + 16 <= K; k0 += 16) {
    double a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      a[u] = ga(i0 + r, k0 + 4 * u + kq);
      b[u] = gb(k0 + 4 * u + kq, j0 + r);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
  }
  for (; k0 < K; k0 += 4) {
    const double a = ga(i0 + r, k0 + kq);
    const double b = gb(k0 + kq, j0 + r);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  return acc;
}

// C (rows x cols) = A B over K, tiles dealt to the waves; out(i, j, value) stores
template <class GA, class GB, class OUT>
__device__ __forceinline__ void product(int rows, int cols, int K, const GA& ga, const GB& gb, const OUT& out,
                                        int wave, int lane, int kb = 0) {
  const int mt = (rows + 15) / 16, nt = (cols + 15) / 16;
  for (int t = wave; t < mt * nt; t += WAVES) {
    const int i0 = (t % mt) * 16, j0 = (t / mt) * 16;
    const d4 acc = tile(i0, j0, K, ga, gb, lane, kb);
    const int j = j0 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int i = i0 + (lane >> 4) + 4 * q;
      if (i < rows && j < cols) out(i, j, acc[q]);
    }
  }
}

// sum_{k<n} fa(k) fb(k), ascending from +0 (the oracle's loops), with eight
// terms' operands read ahead of their additions
template <class FA, class FB>
__device__ __forceinline__ double dot8(int n, const FA& fa, const FB& fb) {
  double s = 0;
  int k = 0;
  for (; k + 8 <= n; k += 8) {
    double a[8], b[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      a[q] = fa(k + q);
      b[q] = fb(k + q);
    }
#pragma unroll
    for (int q = 0; q < 8; q++) s += a[q] * b[q];
  }
  for (; k < n; k++) s += fa(k) * fb(k);
  return s;
}

// LDS (doubles) for (nv, nu): see the layout in backward_seed_mfma
__host__ __device__ inline size_t lds_doubles(int nv, int nu) {
  const size_t nx = 2 * (size_t)nv, LX = nx | 1, LU = (size_t)nu | 1;
  const size_t D = (size_t)nv * (2 * nv + nu) + 2 * nv + nu;
  const size_t x1 = nx * LU > nu * LX ? nx * LU : nu * LX;
  return 4 * nx * LX + nu * LX + x1 + nx * LU + (size_t)nu * nu + 7 * nx + 5 * (size_t)nu + D;
}

// Eigen-style LDLT with symmetric pivoting (oracle ora_ldlt_factor) and its
// solve: riccati.h ldlt_factor_wave (one wavefront) / ldlt_solve (per column)
// NU_ > 0: nu fixed at compile time (the humanoid's 21): the LDLT and its
// solves fully unrolled (riccati.h ldlt_factor_reg_t / ldlt_solve_bcast_t, the
// same operations); 0: any nu <= NU_MAX.  NV_ > 0: nv fixed too (27).
template <int NV_, int NU_, class MD>
__device__ inline void backward_seed_mfma(const MD& m, int nq, int nv_rt, int nu_rt, int P, double dt, double mu,
                                          const double* deriv, int Ds, TrajDev tr, double* Kg, double* kg,
                                          double* Vg, double* vg, int s, double* sh, RicFlags fl) {
  const int nu = NU_ > 0 ? NU_ : nu_rt;
  const int nv = NV_ > 0 ? NV_ : nv_rt;  // NV_ > 0: every loop bound and index a compile-time constant
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nx = 2 * nv, D = nv * (2 * nv + nu) + 2 * nv + nu;
  const int LX = nx | 1, LU = nu | 1;
  double* V = sh;            // nx x nx (ld LX); V_new from stage 8
  double* Vs = V + nx * LX;  // symmetrised V + mu I
  double* A = Vs + nx * LX;  // A; T4 from stage 7
  double* ABK = A + nx * LX;
  double* B = ABK + nx * LX;  // nx x nu (ld LX)
  double* X1 = B + nu * LX;   // T1 (nu x nx, ld LU); T6 (nx x nu, ld LX) from stage 6
  double* Y1 = X1 + (nx * LU > nu * LX ? nx * LU : nu * LX);  // T3, then K (nu x nx, ld LU)
  double* Mm = Y1 + nx * LU;  // nu x nu (ld nu): -2 B'VsB - 2R, then its LDLT factor
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
  double* tmp = r + nu;  // nu: LDLT scratch
  double* dl = tmp + nu;  // FD record of the current step, D doubles
  __shared__ int trn[NU_MAX], perm[NU_MAX];  // STATIC_LDS_BYTES
  double* T4 = A;
  double* Vn = V;
#ifdef ILQG_STAMPS
  unsigned long long bst_prev = 0;  // BSTAMP (riccati.hip): per-stage cycles, diagnostic build
#endif
  BSTAMP(-1);

  // initV at the terminal point dArray[0] (inc/ilqr.h:100-107)
  {
    const double* q0 = deriv + ((size_t)s * P) * Ds + 2 * nv * nv + nv * nu;
    // v0 = dgdx at the terminal point, or the caller's (an initV override)
    for (int i = tid; i < nx; i += THREADS) v[i] = fl.vinit ? vg[(size_t)s * nx + i] : q0[i];
    const double* d1 = deriv + ((size_t)s * P + (P > 1 ? 1 : 0)) * Ds;
    for (int i = tid; i < D; i += THREADS) dl[i] = d1[rec_src(i, nv, nu, fl.layout)];
    __syncthreads();
    for (int e = tid; e < nx * nx; e += THREADS) {
      const int i = e % nx, j = e / nx;
      V[i + j * LX] = fl.vinit ? Vg[(size_t)s * nx * nx + e] : v[i] * v[j];
    }
    __syncthreads();
  }
  for (int n = 1; n < P; n++) {
    const size_t pc = (size_t)s * P + n, pp = pc - 1;
    // next step's FD record, consumed at the end of this step: loaded after
    // the LDLT solves (stage 5), which need the registers
    double pf[MPF];
    auto prefetch = [&]() __attribute__((always_inline)) {
      if (n + 1 < P) {
        const double* dn1 = deriv + (pc + 1) * Ds;
#pragma unroll
        for (int t = 0; t < MPF; t++) {
          const int i = tid + t * THREADS;
          pf[t] = i < D ? dn1[rec_src(i, nv, nu, fl.layout)] : 0.0;
        }
      }
    };
    const double* dn = dl;
    // stage 1: symmetrise V (+ mu I), assemble A/B (differentiator.h:66-71,89-92), q, r, c
    // (columns dealt to the waves, rows to the lanes: no index division; q, c, r
    // on the last wave, which has the fewest columns)
    for (int j = wave; j < nx; j += WAVES)
      for (int i = lane; i < nx; i += 64) {
        const double sv = (V[i + j * LX] + V[j + i * LX]) / 2;
        Vs[i + j * LX] = i == j ? sv + mu : sv;
        double val;
        if (i < nv && j < nv) val = (i == j) ? 1 : 0;
        else if (i < nv) val = (i == j - nv) ? dt : 0;
        else if (j < nv) val = dn[(i - nv) + j * nv] * dt;
        else val = ((i - nv) == (j - nv) ? 1 : 0) + dn[nv * nv + (i - nv) + (j - nv) * nv] * dt;
        A[i + j * LX] = val;
      }
    for (int j = wave; j < nu; j += WAVES)
      for (int i = lane; i < nx; i += 64) B[i + j * LX] = (i < nv) ? 0 : dn[2 * nv * nv + (i - nv) + j * nv] * dt;
    if (wave == WAVES - 1) {
      for (int i = lane; i < nx; i += 64) {
        q[i] = dn[2 * nv * nv + nv * nu + i];
        // c = x*_{n-1} (-) x*_n (inc/ilqr.h:154-157; tangent space for quaternion joints)
        if (i < nv && nq != nv) {
          c[i] = dev::state_diff_dof(m, i, tr.qpos + pp * nq, tr.qpos + pc * nq);
        } else {
          const double xp = i < nv ? tr.qpos[pp * nq + i] : tr.qvel[pp * nv + i - nv];
          const double xc = i < nv ? tr.qpos[pc * nq + i] : tr.qvel[pc * nv + i - nv];
          c[i] = xp - xc;
        }
      }
      for (int a = lane; a < nu; a += 64) r[a] = dn[2 * nv * nv + nv * nu + nx + a];
    }
    __syncthreads();
    BSTAMP(0);
    // stage 2: T1 = B' Vs (nu x nx); B's rows below nv are zero (B = [0; dt dB]):
    // the products over them start at the last multiple of 4 at or below nv
    // (whole MFMA k-steps of zero terms skipped, which add exact zeros)
    const int kb = nv & ~3;
    product(
        nu, nx, nx, [&](int a, int k) { return (a < nu && k < nx) ? B[k + a * LX] : 0.0; },
        [&](int k, int j) { return (k < nx && j < nx) ? Vs[k + j * LX] : 0.0; },
        [&](int a, int j, double x) { X1[a + j * LU] = x; }, wave, lane, kb);
    __syncthreads();
    BSTAMP(1);
    // stage 3: Mm = -2 T1 B - 2 R ; T3 = T1 A ; w = v + 2 Vs c
    auto gT1 = [&](int a, int k) { return (a < nu && k < nx) ? X1[a + k * LU] : 0.0; };
    product(
        nu, nu, nx, gT1, [&](int k, int b) { return (k < nx && b < nu) ? B[k + b * LX] : 0.0; },
        [&](int a, int b, double x) { Mm[a + b * nu] = -2 * x - 2 * (r[a] * r[b]); }, wave, lane, kb);
    // (T3's tiles dealt from wave 4 on: Mm's went to waves 0-3; w on the last wave)
    product(
        nu, nx, nx, gT1, [&](int k, int j) { return (k < nx && j < nx) ? A[k + j * LX] : 0.0; },
        [&](int a, int j, double x) { Y1[a + j * LU] = x; }, (wave + 4) % WAVES, lane);
    if (wave == WAVES - 1)
      for (int i = lane; i < nx; i += 64) {
        const double sm = dot8(nx, [&](int j) { return Vs[i + j * LX]; }, [&](int j) { return c[j]; });
        w[i] = v[i] + 2 * sm;
      }
    __syncthreads();
    BSTAMP(2);
    // stage 4: LDLT of Mm (wave 0); col = B'w + r beside it (wave 1)
    // (and perm, the solves' gather order)
    if (wave == 0) {
      if constexpr (NU_ > 0) {
        if (fl.ldlt_lds == 1) {
          ldlt_factor_wave_t<NU_>(Mm, trn, tmp, lane);
          ldlt_perm(nu, trn, perm, lane);
        } else {
          ldlt_factor_reg_t<NU_>(Mm, trn, perm, tmp, lane, fl.ldlt_lds == 2);
        }
      } else {
        ldlt_factor_wave(nu, Mm, trn, tmp, lane);
        ldlt_perm(nu, trn, perm, lane);
      }
    }
    for (int a = tid - 64; a >= 0 && a < nu; a += THREADS) {
      const double sm = dot8(nx, [&](int kk) { return B[kk + a * LX]; }, [&](int kk) { return w[kk]; });
      col[a] = sm + r[a];
    }
    __syncthreads();
    BSTAMP(3);
    // stage 5: K = ldlt.solve(2 T3) column-parallel (in place), k = ldlt.solve(B'w + r)
    // (columns dealt over SOLVE_WAVES waves, one a SIMD: one solve per lane,
    // the vector in registers, ldlt_solve_reg; a second wave on a SIMD would
    // issue the whole instruction stream again for its few columns -- 8 waves
    // measured 26k cycles a step against 4's 16k)
    // (NU_ > 0: the doubling of T3 and the copy of col folded into the solve's
    // gather, the same values)
#ifndef ILQG_SOLVE_STRIDE
#define ILQG_SOLVE_STRIDE 1
#endif
    constexpr int SS = ILQG_SOLVE_STRIDE;  // the solving waves: every SS-th
    if (wave % SS == 0 && wave / SS < SOLVE_WAVES) {
      const int j = lane * SOLVE_WAVES + wave / SS;  // one column per thread: nx + 1 <= 64 SOLVE_WAVES (launch_backward_mfma)
      double* x = j < nx ? Y1 + j * LU : kl;
      if constexpr (NU_ > 0) {
#ifndef ILQG_SOLVE_BCAST
#define ILQG_SOLVE_BCAST 1
#endif
        if constexpr (ILQG_SOLVE_BCAST) ldlt_solve_bcast_t<NU_>(Mm, perm, j < nx ? x : col, x, j < nx, j < nx + 1, lane);
        else ldlt_solve_reg_t<NU_>(Mm, perm, j < nx ? x : col, x, j < nx, j < nx + 1);
      } else {
        if (j < nx)
          for (int a = 0; a < nu; a++) x[a] = 2 * x[a];
        else if (j == nx)
          for (int a = 0; a < nu; a++) x[a] = col[a];
        ldlt_solve_reg(nu, Mm, perm, x, j < nx + 1);
      }
    }
    __syncthreads();
    BSTAMP(4);
#ifndef ILQG_PF_STAGE
#define ILQG_PF_STAGE 9
#endif
    // (issued at stage 6, the record loads' registers collided with the
    // products' and the compiler waited for the loads there: vmcnt(0) before
    // stage 6's first MFMA, every step.  Issued at stage 9 they are waited for
    // at stage 10 -- the same 6.22-6.27 ms a launch as issuing them at stage 7,
    // profiles/r06_mfma_waves.txt)
    if constexpr (ILQG_PF_STAGE == 6) prefetch();
    // stage 6: ABK = A + B K ; T6 = K'R ; y = B k + c ; kR = k'R
    auto gK = [&](int a, int j) { return (a < nu && j < nx) ? Y1[a + j * LU] : 0.0; };
    product(
        nx, nx, nu, [&](int i, int a) { return (i < nx && a < nu) ? B[i + a * LX] : 0.0; }, gK,
        [&](int i, int j, double x) { ABK[i + j * LX] = A[i + j * LX] + x; }, wave, lane);
    product(
        nx, nu, nu, [&](int i, int a) { return (i < nx && a < nu) ? Y1[a + i * LU] : 0.0; },
        [&](int a, int b) { return (a < nu && b < nu) ? r[a] * r[b] : 0.0; },
        [&](int i, int b, double x) { X1[i + b * LX] = x; }, wave, lane);
    // (y on wave 0, kR on wave 1: every wave has dealt its tiles)
    if (wave == 0)
      for (int i = lane; i < nx; i += 64) {
        const double sm = dot8(nu, [&](int a) { return B[i + a * LX]; }, [&](int a) { return kl[a]; });
        y[i] = sm + c[i];
      }
    if (wave == 1)
      for (int b = lane; b < nu; b += 64)
        kR[b] = dot8(nu, [&](int a) { return kl[a]; }, [&](int a) { return r[a] * r[b]; });
    __syncthreads();
    BSTAMP(5);
    // stage 7: T4 = ABK' Vs (into A's buffer: A is dead)
    product(
        nx, nx, nx, [&](int i, int k) { return (i < nx && k < nx) ? ABK[k + i * LX] : 0.0; },
        [&](int k, int j) { return (k < nx && j < nx) ? Vs[k + j * LX] : 0.0; },
        [&](int i, int j, double x) { T4[i + j * LX] = x; }, wave, lane);
    __syncthreads();
    BSTAMP(6);
    // stage 8: V_new = (T4 ABK + q q') + T6 K (into V's buffer: V is dead)
    {
      const int mt = (nx + 15) / 16;
      for (int t = wave; t < mt * mt; t += WAVES) {
        const int i0 = (t % mt) * 16, j0 = (t / mt) * 16;
        const d4 a1 = tile(
            i0, j0, nx, [&](int i, int k) { return (i < nx && k < nx) ? T4[i + k * LX] : 0.0; },
            [&](int k, int j) { return (k < nx && j < nx) ? ABK[k + j * LX] : 0.0; }, lane);
        const d4 a2 = tile(
            i0, j0, nu, [&](int i, int b) { return (i < nx && b < nu) ? X1[i + b * LX] : 0.0; }, gK, lane);
        const int j = j0 + (lane & 15);
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
          const int i = i0 + (lane >> 4) + 4 * qq;
          if (i < nx && j < nx) Vn[i + j * LX] = (a1[qq] + q[i] * q[j]) + a2[qq];
        }
      }
    }
    __syncthreads();
    BSTAMP(7);
    if constexpr (ILQG_PF_STAGE == 9) prefetch();
    // stage 9: z = (2y)' V_new ; v_new (reads the NEW V, quirk Q14).  The
    // terms of v_new that do not read z -- v' ABK and (2 kR)' K -- beside z on
    // waves 1 and 2 (into w and c, dead since stages 4 and 6), the gains out
    // on the others; then z' ABK and the sum, in the oracle's order
    static_assert(WAVES >= 4, "stage 9 deals four roles to the waves");
    if (wave == 0) {
      for (int j = lane; j < nx; j += 64)
        z[j] = dot8(nx, [&](int i) { return 2 * y[i]; }, [&](int i) { return Vn[i + j * LX]; });
    } else if (wave == 1) {
      for (int j = lane; j < nx; j += 64)
        w[j] = dot8(nx, [&](int i) { return v[i]; }, [&](int i) { return ABK[i + j * LX]; });
    } else if (wave == 2) {
      for (int j = lane; j < nx; j += 64)
        c[j] = dot8(nu, [&](int b) { return 2 * kR[b]; }, [&](int b) { return Y1[b + j * LU]; });
    } else {
      // gains out (Eigen col-major K[a + j nu])
      for (int e = tid - 192; e < nu * nx; e += THREADS - 192) {
        const int a = e % nu, j = e / nu;
        Kg[pc * nu * nx + e] = Y1[a + j * LU];
      }
      for (int a = tid - 192; a < nu; a += THREADS - 192) kg[pc * nu + a] = kl[a];
    }
    __syncthreads();
    for (int j = tid; j < nx; j += THREADS) {
      const double ta = dot8(nx, [&](int i) { return z[i]; }, [&](int i) { return ABK[i + j * LX]; });
      vn[j] = ((ta + w[j]) + q[j]) + c[j];
    }
    __syncthreads();
    BSTAMP(8);
    for (int i = tid; i < nx; i += THREADS) v[i] = vn[i];
    if (n + 1 < P) {
#pragma unroll
      for (int t = 0; t < MPF; t++) {
        const int i = tid + t * THREADS;
        if (i < D) dl[i] = pf[t];
      }
    }
    __syncthreads();
    BSTAMP(9);
  }
  if (Vg)
    for (int e = tid; e < nx * nx; e += THREADS) {
      const int i = e % nx, j = e / nx;
      Vg[(size_t)s * nx * nx + e] = V[i + j * LX];
    }
  if (vg)
    for (int i = tid; i < nx; i += THREADS) vg[(size_t)s * nx + i] = v[i];
}

}  // namespace rmfma
}  // namespace ilqg
