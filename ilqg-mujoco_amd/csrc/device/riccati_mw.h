// initV + Riccati backward pass (inc/ilqr.h:100-107,133-176) for the
// register-formulation sizes (riccati_reg.h: pendulum 2/1, hopper 6/3) on a
// multi-wave workgroup with one lane per matrix entry.  Column j of every
// nx x nx matrix belongs to the NXP = 2^k >= NX lanes j NXP .. j NXP + NXP - 1
// (a column never straddles a wavefront), lane (i, j) = tid j NXP + i owning
// entry (i, j); the column's lanes past NX (and any lanes past NX NXP) are
// spare lanes for the small nu x nu products and y.
//
// The one-wave formulation gives each lane three rows of a column (≈11k
// cycles a hopper step, each stage a chain of 3 x 12-term sums per lane).
// Here a lane sums one entry, the stages are separated by LDS-only workgroup
// barriers (global loads -- the next record, the next state -- stay in flight
// across them), and a step is five stages:
//   A  Vs column j (each lane, from V); T1[a][j] (lanes i = a < NU); lane i = NU:
//      v_{n-1}[j] (the previous step's last stage, deferred to here) and w[j]
//   B  T3[a][j] (lanes i = a < NU); spare lanes: Mm, col
//   C  every lane: the pivoted LDLT of Mm, k and K[:, j] (2 T3[:, j]) solved
//      together (uniform); lane (i, j): ABK[i][j]; spare lanes: y
//   D  T4[i][j] = (ABK' Vs)[i][j]; T6 row i (registers)
//   E  Vn[i][j] = (T4 ABK + q q')[i][j] + (T6 K)[i][j]; lane (0, j): z[j] =
//      (2y)' Vn[:, j] gathered from its column's lanes; the next FD record and c
// Every scalar is riccati_reg.h's expression -- the oracle's (oracle/ilqr_ora.c
// ora_riccati_step_c, ora_ldlt_factor/solve) in the oracle's summation order --
// so K, k, V, v are bit-identical to the oracle and to the one-wave kernel.
//
// Streaming (done != nullptr): a launch of its own beside the FD sweep that
// produces the records (seed groups, capi.cpp iterate_groups): record p is read
// once done[s P + p] >= target, with sc1 loads (handoff.h); every wave polls
// for itself before its lanes load.
#pragma once
#include <hip/hip_runtime.h>

#include "riccati_reg.h"

namespace ilqg {

template <int NV, int NU>
struct RicMw {
  static constexpr int NX = 2 * NV;
  static constexpr bool ok = RicReg<NV, NU>::ok;
  static constexpr int LX = NX + 2;  // even: 16-byte aligned columns
  static constexpr int NXP = NX <= 4 ? 4 : (NX <= 8 ? 8 : 16);
  static constexpr int NCOL = NX * NXP;
  static constexpr int NSPIN = NX * (NXP - NX);  // spare lanes inside the columns
  static constexpr int NSPNEED = (NU * NU + NU) > NX ? (NU * NU + NU) : NX;
  static constexpr int THREADS = (NCOL + (NSPNEED > NSPIN ? NSPNEED - NSPIN : 0) + 63) / 64 * 64;
  static constexpr int D = NV * (2 * NV + NU) + 2 * NV + NU;
  static constexpr int DP = (D + 1) / 2 * 2;
  static constexpr int NPF = (D + THREADS - 1) / THREADS;
  // LDS offsets (doubles, all even)
  static constexpr int oV = 0, oABK = oV + NX * LX, oT4 = oABK + NX * LX, oT1 = oT4 + NX * LX,
                       oT3 = oT1 + NU * NX, oW = oT3 + (NU * NX + 1) / 2 * 2, oM = oW + NX,
                       oK = oM + (NU * NU + NU + 1) / 2 * 2, oZ = oK + (NU * NX + 1) / 2 * 2, oY = oZ + NX,
                       oVv = oY + NX, oC = oVv + 2 * NX, oDL = oC + 2 * NX, total = oDL + 2 * DP;
  static constexpr size_t bytes = (size_t)total * sizeof(double);
};

namespace rreg {
// workgroup barrier ordering LDS only: outstanding global loads stay in flight
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// ldlt_solve_r on two right-hand sides, their operations interleaved (each
// vector receives exactly ldlt_solve_r's operations in its order)
template <int N>
__device__ __forceinline__ void ldlt_solve2_r(const double (&L)[N * N], const int (&tr)[N], double (&x)[N],
                                              double (&y)[N]) {
  const double tol = 2.2250738585072014e-308;
  sf<0, N>(RL(kk) {
    constexpr int k = RK(kk);
    if (tr[k] != k) {
      swap_rt<N>(x, k, tr[k]);
      swap_rt<N>(y, k, tr[k]);
    }
  });
  sf<0, N>(RL(ii) {
    constexpr int i = RK(ii);
    sf<0, i>(RL(jj) {
      x[i] -= L[i + RK(jj) * N] * x[RK(jj)];
      y[i] -= L[i + RK(jj) * N] * y[RK(jj)];
    });
  });
  sf<0, N>(RL(ii) {
    constexpr int i = RK(ii);
    const bool nz = fabs(L[i + i * N]) > tol;
    const double qx = x[i] / L[i + i * N], qy = y[i] / L[i + i * N];
    x[i] = nz ? qx : 0.0;
    y[i] = nz ? qy : 0.0;
  });
  sf<0, N>(RL(ii) {
    constexpr int i = N - 1 - RK(ii);
    sf<i + 1, N>(RL(jj) {
      x[i] -= L[RK(jj) + i * N] * x[RK(jj)];
      y[i] -= L[RK(jj) + i * N] * y[RK(jj)];
    });
  });
  sf<0, N>(RL(kk) {
    constexpr int k = N - 1 - RK(kk);
    if (tr[k] != k) {
      swap_rt<N>(x, k, tr[k]);
      swap_rt<N>(y, k, tr[k]);
    }
  });
}
}  // namespace rreg

template <int NV, int NU, class MD>
__device__ inline void backward_seed_mw(const MD& m, int P, double dt, double mu, const double* deriv, int Ds,
                                        TrajDev tr, double* Kg, double* kg, double* Vg, double* vg, int s, int tid,
                                        double* sh, const unsigned* done, unsigned target, unsigned* fault,
                                        RicFlags fl) {
  using R = RicMw<NV, NU>;
  constexpr int NX = R::NX, LX = R::LX, NXP = R::NXP, D = R::D, DP = R::DP, T = R::THREADS, NPF = R::NPF;
  using namespace rreg;
  (void)m;
  double* Vb = sh + R::oV;
  double* ABKb = sh + R::oABK;
  double* T4b = sh + R::oT4;
  double* T1b = sh + R::oT1;
  double* T3b = sh + R::oT3;
  double* Wb = sh + R::oW;
  double* Mb = sh + R::oM;
  double* Kb = sh + R::oK;
  double* Zb = sh + R::oZ;
  double* Yb = sh + R::oY;
  double* Vv = sh + R::oVv;   // v_n in buffer n & 1
  double* Cb = sh + R::oC;    // c of step n in buffer (n - 1) & 1
  double* DLb = sh + R::oDL;  // FD record of step n in buffer n & 1
  const int i = tid % NXP, j = tid / NXP;  // lane (i, j)
  const bool mat = tid < R::NCOL && i < NX;
  const int sp = tid < R::NCOL ? (i >= NX ? j * (NXP - NX) + (i - NX) : -1) : R::NSPIN + (tid - R::NCOL);
  const int jc = j < NX ? j : 0;  // the column index clamped for the spare lanes past the columns
#ifdef ILQG_STAMPS
  unsigned long long bst_prev = 0;
#endif

  int ready_upto = -1;
  auto ready = [&](int p) __attribute__((always_inline)) {
    if (!done || p <= ready_upto) return;
    ready_upto = bw_wait_window(done + (size_t)s * P, p, P, target, fault);
  };
  auto ld = [&](const double* a) -> double __attribute__((always_inline)) { return done ? ld_sc1(a) : *a; };
  auto fetch_rec = [&](size_t pt, double (&pf)[NPF]) __attribute__((always_inline)) {
    const double* src = deriv + pt * Ds;
    sf<0, NPF>(RL(tt) {
      const int e = tid + RK(tt) * T;
      pf[RK(tt)] = e < D ? ld(src + rec_src(e, NV, NU, fl.layout)) : 0.0;
    });
  };
  auto park_rec = [&](const double (&pf)[NPF], double* dst) __attribute__((always_inline)) {
    sf<0, NPF>(RL(tt) {
      const int e = tid + RK(tt) * T;
      if (e < D) dst[e] = pf[RK(tt)];
    });
  };
  // nominal state component tid (< NX) of a point: [qpos | qvel] (nq == nv)
  auto xload = [&](size_t pt) -> double __attribute__((always_inline)) {
    return tid < NV ? tr.qpos[pt * NV + tid] : (tid < NX ? tr.qvel[pt * NV + tid - NV] : 0.0);
  };

  // ---- initV at the terminal point dArray[0] (inc/ilqr.h:100-107) ----
  {
    ready(0);
    const double* q0 = deriv + ((size_t)s * P) * Ds + 2 * NV * NV + NV * NU;
    // v0 = dgdx at the terminal point, or the caller's (an initV override)
    const double v0 = tid < NX ? (fl.vinit ? vg[(size_t)s * NX + tid] : ld(q0 + tid)) : 0.0;
    if (tid < NX) Vv[tid] = v0;  // v_0, buffer 0
    if (P > 1) {
      ready(1);
      double pf[NPF];
      fetch_rec((size_t)s * P + 1, pf);
      park_rec(pf, DLb + DP);  // step 1's record, buffer 1
    }
    lds_barrier();
    if (mat) Vb[i + j * LX] = fl.vinit ? Vg[(size_t)s * NX * NX + i + j * NX] : Vv[i] * Vv[j];  // V = v'v
  }
  double xa = 0, xb = 0;
  xa = xload((size_t)s * P);
  if (P > 1) xb = xload((size_t)s * P + 1);
  if (tid < NX) Cb[tid] = xa - xb;  // c of step 1
  lds_barrier();
  BSTAMP(-1);

  // the previous step's values its deferred last stage (v_{n-1}) reads
  double abk_p[NX], Kc_p[NU], kR_p[NU], qj_p = 0;
  sf<0, NX>(RL(kk) { abk_p[RK(kk)] = 0; });
  sf<0, NU>(RL(aa) { Kc_p[RK(aa)] = 0; kR_p[RK(aa)] = 0; });
  // v_{n-1}[j] = ((z_{n-1}' ABK[:, j] + v_{n-2}' ABK[:, j]) + q[j]) + 2 kR K[:, j]
  // (ilqr.h:175, quirk Q14: z from the NEW V), on lane (NU, j)
  auto v_prev = [&](const double* vold) -> double __attribute__((always_inline)) {
    double zz[NX], vv[NX];
    lds_row<NX>(zz, Zb);
    lds_row<NX>(vv, vold);
    double ta = 0, tb = 0, td = 0;
    sf<0, NX>(RL(kk) { ta += zz[RK(kk)] * abk_p[RK(kk)]; });
    sf<0, NX>(RL(kk) { tb += vv[RK(kk)] * abk_p[RK(kk)]; });
    sf<0, NU>(RL(bb) { td += (2 * kR_p[RK(bb)]) * Kc_p[RK(bb)]; });
    return ((ta + tb) + qj_p) + td;
  };

  for (int n = 1; n < P; n++) {
    const size_t pc = (size_t)s * P + n;
    const double* cc = Cb + ((n - 1) & 1) * NX;  // step n's c
    double* cnext = Cb + (n & 1) * NX;
    const double* dl = DLb + (n & 1) * DP;
    // next step's record and state, one step ahead (in flight until stage E)
    double xn = 0;
    if (n + 1 < P) xn = xload(pc + 1);
    double pf[NPF];
    if (n + 1 < P) {
      ready(n + 1);
      fetch_rec(pc + 1, pf);
    }
    // record offsets: B block (deriv[2nv^2 + (i - nv) + a nv], differentiator.h:89-92,
    // quirk Q1), A's lower blocks (:66-71), q, r (ilqr.h:157-158)
    constexpr int oB = 2 * NV * NV, oQ = 2 * NV * NV + NV * NU, oR = oQ + NX;
    double r[NU];
    sf<0, NU>(RL(aa) { r[RK(aa)] = dl[oR + RK(aa)]; });
    auto bcol = [&](int a_, double (&bl)[NV]) __attribute__((always_inline)) {
      lds_row<NV>(bl, dl + oB + a_ * NV);
      sf<0, NV>(RL(ii) { bl[RK(ii)] = bl[RK(ii)] * dt; });
    };
    // A[ai][aj] (differentiator.h:66-71), the oracle's expression
    auto aval = [&](int ai, int aj) -> double __attribute__((always_inline)) {
      if (ai < NV) {
        if (aj < NV) return (ai == aj) ? 1.0 : 0.0;
        return (ai == aj - NV) ? dt : 0.0;
      }
      if (aj < NV) return dl[(ai - NV) + aj * NV] * dt;
      return ((ai - NV) == (aj - NV) ? 1.0 : 0.0) + dl[NV * NV + (ai - NV) + (aj - NV) * NV] * dt;
    };
    // ---- A: Vs column j; T1[a][j] (lane i = a); v_{n-1}[j] and w[j] (lane i = NU) ----
    double vs[NX];
    if (mat) {
      double vc[NX];
      lds_row<NX>(vc, Vb + j * LX);
      sf<0, NX>(RL(kk) {
        constexpr int k = RK(kk);
        vs[k] = (vc[k] + Vb[j + k * LX]) / 2;
      });
      // V.diagonal() += mu (inc/ilqr.h:165-166, quirk Q13): entry (j, j)
      sf<0, NX>(RL(kk) {
        const double d = vs[RK(kk)] + mu;
        vs[RK(kk)] = (RK(kk) == j) ? d : vs[RK(kk)];
      });
      if (i < NU) {
        double bl[NV];
        bcol(i, bl);
        double t1 = 0;
        sf<0, NX>(RL(kk) {
          constexpr int k = RK(kk);
          if constexpr (k < NV) t1 += 0.0 * vs[k];
          else t1 += bl[k - NV] * vs[k];
        });
        T1b[i * NX + j] = t1;  // T1[a][kk] at a NX + kk
      } else if (i == NU) {
        double vj;
        if (n >= 2) {
          vj = v_prev(Vv + (n & 1) * NX);  // from v_{n-2}
          Vv[((n - 1) & 1) * NX + j] = vj;
        } else {
          vj = Vv[j];
        }
        double c[NX];
        lds_row<NX>(c, cc);
        double sm = 0;
        sf<0, NX>(RL(kk) { sm += vs[RK(kk)] * c[RK(kk)]; });
        Wb[j] = vj + 2 * sm;
      }
    }
    lds_barrier();
    BSTAMP(0);
    // ---- B: T3[a][j] (lane i = a); spare lanes Mm, col ----
    if (mat) {
      if (i < NU) {
        double t1r[NX];
        lds_row<NX>(t1r, T1b + i * NX);
        // A column j: [delta or dt delta ; dt * deriv block column]
        double al[NV];
        lds_row<NV>(al, dl + (j < NV ? j * NV : NV * NV + (j - NV) * NV));
        double t3 = 0;
        sf<0, NX>(RL(kk) {
          constexpr int k = RK(kk);
          double av;
          if constexpr (k < NV) av = j < NV ? ((k == j) ? 1.0 : 0.0) : ((k == j - NV) ? dt : 0.0);
          else av = j < NV ? al[k - NV] * dt : ((k - NV) == (j - NV) ? 1.0 : 0.0) + al[k - NV] * dt;
          t3 += t1r[k] * av;
        });
        T3b[i + j * NU] = t3;
      }
    } else if (sp >= 0 && sp < NU * NU) {
      const int a = sp % NU, b = sp / NU;
      double t1r[NX], bl[NV];
      lds_row<NX>(t1r, T1b + a * NX);
      bcol(b, bl);
      double sm = 0;
      sf<0, NX>(RL(kk) {
        constexpr int k = RK(kk);
        if constexpr (k < NV) sm += t1r[k] * 0.0;
        else sm += t1r[k] * bl[k - NV];
      });
      Mb[sp] = -2 * sm - 2 * (dl[oR + a] * dl[oR + b]);
    } else if (sp >= NU * NU && sp < NU * NU + NU) {
      const int a = sp - NU * NU;
      double wv[NX], bl[NV];
      lds_row<NX>(wv, Wb);
      bcol(a, bl);
      double sm = 0;
      sf<0, NX>(RL(kk) {
        constexpr int k = RK(kk);
        if constexpr (k < NV) sm += 0.0 * wv[k];
        else sm += bl[k - NV] * wv[k];
      });
      Mb[sp] = sm + dl[oR + a];
    }
    lds_barrier();
    BSTAMP(1);
    // ---- C: LDLT, k and K[:, j] (uniform); ABK[i][j]; spare lanes y ----
    double Lm[NU * NU], kf[NU], Kc[NU];
    int trn[NU];
    sf<0, NU * NU>(RL(ee) { Lm[RK(ee)] = Mb[RK(ee)]; });
    sf<0, NU>(RL(aa) {
      kf[RK(aa)] = Mb[NU * NU + RK(aa)];
      Kc[RK(aa)] = 2 * T3b[RK(aa) + jc * NU];
    });
    ldlt_factor_r<NU>(Lm, trn);
    ldlt_solve2_r<NU>(Lm, trn, kf, Kc);
    if (mat) {
      double sm = 0;
      sf<0, NU>(RL(aa) {
        const double bi = i < NV ? 0.0 : dl[oB + (i - NV) + RK(aa) * NV] * dt;
        sm += bi * Kc[RK(aa)];
      });
      ABKb[i + j * LX] = aval(i, j) + sm;
      if (i == 0) {
        sf<0, NU>(RL(aa) {
          Kb[RK(aa) + j * NU] = Kc[RK(aa)];
          Kg[pc * NU * NX + RK(aa) + j * NU] = Kc[RK(aa)];
        });
      }
    } else if (sp >= 0 && sp < NX) {
      // y = B k + c (ilqr.h:174), one entry per spare lane
      const int yi = sp;
      double sm = 0;
      sf<0, NU>(RL(aa) {
        const double bi = yi < NV ? 0.0 : dl[oB + (yi - NV) + RK(aa) * NV] * dt;
        sm += bi * kf[RK(aa)];
      });
      Yb[yi] = sm + cc[yi];
    }
    if (tid == 0) sf<0, NU>(RL(aa) { kg[pc * NU + RK(aa)] = kf[RK(aa)]; });
    // kR = k'R (uniform), read by v_n's stage in the next step
    sf<0, NU>(RL(bb) {
      double sm = 0;
      sf<0, NU>(RL(aa) { sm += kf[RK(aa)] * (r[RK(aa)] * r[RK(bb)]); });
      kR_p[RK(bb)] = sm;
    });
    lds_barrier();
    BSTAMP(2);
    // ---- D: T4[i][j]; T6 row i (registers) ----
    double T6r[NU];
    if (mat) {
      double ac[NX];
      lds_row<NX>(ac, ABKb + i * LX);
      double sm = 0;
      sf<0, NX>(RL(kk) { sm += ac[RK(kk)] * vs[RK(kk)]; });
      T4b[i * LX + j] = sm;  // row-major
      double kc[NU];
      sf<0, NU>(RL(aa) { kc[RK(aa)] = Kb[RK(aa) + i * NU]; });
      sf<0, NU>(RL(bb) {
        double t = 0;
        sf<0, NU>(RL(aa) { t += kc[RK(aa)] * (r[RK(aa)] * r[RK(bb)]); });
        T6r[RK(bb)] = t;
      });
    }
    lds_barrier();
    BSTAMP(3);
    // ---- E: Vn[i][j] (into V's buffer); z[j] on lane (0, j); next record, c ----
    const double qj = dl[oQ + jc];
    double vn = 0;
    lds_row<NX>(abk_p, ABKb + jc * LX);  // ABK column j, for this step's v (deferred)
    if (mat) {
      double tr4[NX];
      lds_row<NX>(tr4, T4b + i * LX);
      double s5 = 0, s7 = 0;
      sf<0, NX>(RL(kk) { s5 += tr4[RK(kk)] * abk_p[RK(kk)]; });
      sf<0, NU>(RL(bb) { s7 += T6r[RK(bb)] * Kc[RK(bb)]; });
      vn = (s5 + dl[oQ + i] * qj) + s7;
      Vb[i + j * LX] = vn;
    }
    {
      // z[j] = (2y)' Vn[:, j] (ilqr.h:175): the column's entries from its lanes
      double vcol[NX];
      const int base = (tid & 63) & ~(NXP - 1);
      sf<0, NX>(RL(kk) { vcol[RK(kk)] = __shfl(vn, base + RK(kk)); });
      if (mat && i == 0) {
        double y[NX];
        lds_row<NX>(y, Yb);
        double sm = 0;
        sf<0, NX>(RL(kk) { sm += (2 * y[RK(kk)]) * vcol[RK(kk)]; });
        Zb[j] = sm;
      }
    }
    qj_p = qj;
    sf<0, NU>(RL(aa) { Kc_p[RK(aa)] = Kc[RK(aa)]; });
    if (n + 1 < P) {
      if (tid < NX) cnext[tid] = xb - xn;
      park_rec(pf, DLb + ((n + 1) & 1) * DP);
    }
    xa = xb;
    xb = xn;
    lds_barrier();
    BSTAMP(4);
  }
  // the last step's v (its deferred stage)
  if (P > 1 && mat && i == NU) {
    const double vj = v_prev(Vv + (P & 1) * NX);  // from v_{P-2}
    Vv[((P - 1) & 1) * NX + j] = vj;
  }
  lds_barrier();
  const double* vfin = Vv + ((P - 1) & 1) * NX;
  if (Vg && mat) Vg[(size_t)s * NX * NX + i + j * NX] = Vb[i + j * LX];
  if (vg && tid < NX) vg[(size_t)s * NX + tid] = vfin[tid];
}

}  // namespace ilqg
