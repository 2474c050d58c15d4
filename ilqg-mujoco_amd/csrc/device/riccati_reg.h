// initV + Riccati backward pass (inc/ilqr.h:100-107,133-176) for compile-time
// (NV, NU) with NX = 2 NV a multiple of 4 and <= 16, NU <= 4 -- the bundled
// pendulum (2, 1) and hopper (6, 3) -- on one 64-lane wavefront, with the
// per-lane state in VGPRs and LDS used only to exchange the products one
// stage needs from another.  Included by riccati.h; backward_seed dispatches
// here for those sizes.
//
// Layout.  Lanes 0 .. 4 NX - 1 form NX quads; quad j owns column j of every
// nx x nx matrix, and its lane g (0..3) the rows i = g, g+4, g+8, ... (RP =
// NX / 4 of them).  Each quad lane keeps the whole column j of Vs in
// registers (it recomputes it from V rather than exchanging it: Vs is
// symmetric bit for bit, (a + b)/2 == (b + a)/2, so column j is also row j,
// which is what w and T1 need).  The spare lanes 4 NX .. 63 compute the small
// nu x nu products.  One step:
//   A  Vs column j; T1[g][j] = (B'Vs)[g][j]; w[j] = v[j] + 2 (Vs c)[j]     -> LDS
//   B  spare lanes: Mm = -2 T1 B - 2 R, col = B'w + r; quads: T3[g][j]    -> LDS
//   C  every lane: Eigen's pivoted LDLT of Mm in registers (uniform), k;
//      quad j: K[:, j] (T3 column gathered over the quad by DPP), ABK rows -> LDS
//   D  T4 = ABK' Vs (rows R_g of column j), T6 = K' R                      -> LDS
//   E  Vn = (T4 ABK + q q') + T6 K (rows R_g of column j)                 -> LDS (V)
//   F  z = (2y)' Vn                                                        -> LDS
//   G  v_new = ((z ABK + v ABK) + q') + 2 kR K (Q14: the NEW V)            -> LDS
// Every scalar is the oracle's expression (oracle/ilqr_ora.c
// ora_riccati_step_c, ora_ldlt_factor/solve) with the oracle's summation
// order, on one lane; only where it is computed changed.  Synchronisation
// is wave-scope (team_sync): one wavefront executes its LDS accesses in order.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace ilqg {
namespace rreg {

template <int B, int E, typename F>
__device__ __forceinline__ void sf(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sf<B + 1, E>(f);
  }
}
#define RK(v) decltype(v)::value
#define RL(v) [&](auto v) __attribute__((always_inline))

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lane (quad base + S) of the caller's quad, to every lane of the quad
template <int S>
__device__ __forceinline__ double quad_bcast(double x) {
  constexpr int ctrl = S | (S << 2) | (S << 4) | (S << 6);  // quad_perm [S,S,S,S]
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), ctrl, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// n contiguous doubles from 16-byte aligned LDS as b128 reads
template <int N>
__device__ __forceinline__ void lds_row(double (&d)[N], const double* p) {
  static_assert(N % 2 == 0, "even rows");
  sf<0, N / 2>(RL(hh) {
    const double2 t = reinterpret_cast<const double2*>(p)[RK(hh)];
    d[2 * RK(hh)] = t.x;
    d[2 * RK(hh) + 1] = t.y;
  });
}

// Eigen's pivoted LDLT (oracle ora_ldlt_factor) of an N x N matrix held in
// registers, m[i + j N] (column-major, lower triangle used); every index a
// compile-time constant, the pivot a runtime select.  Uniform on every lane.
template <int N>
__device__ __forceinline__ void ldlt_factor_r(double (&m)[N * N], int (&tr)[N]) {
  bool stop = false;
  sf<0, N>(RL(kk) {
    constexpr int k = RK(kk);
    if (stop) {
      tr[k] = k;
      return;
    }
    int big = k;
    double bigv = fabs(m[k + k * N]);
    sf<k + 1, N>(RL(ii) {
      constexpr int i = RK(ii);
      const double a = fabs(m[i + i * N]);
      if (a > bigv) {
        bigv = a;
        big = i;
      }
    });
    tr[k] = big;
    // symmetric pivot swap (oracle order), once per candidate b == big
    sf<k + 1, N>(RL(bb) {
      constexpr int b = RK(bb);
      if (big == b) {
        double t;
        sf<0, k>(RL(jj) {
          constexpr int j = RK(jj);
          t = m[k + j * N]; m[k + j * N] = m[b + j * N]; m[b + j * N] = t;
        });
        sf<0, N - b - 1>(RL(ii) {
          constexpr int r = b + 1 + RK(ii);
          t = m[r + k * N]; m[r + k * N] = m[r + b * N]; m[r + b * N] = t;
        });
        t = m[k + k * N]; m[k + k * N] = m[b + b * N]; m[b + b * N] = t;
        sf<k + 1, b>(RL(ii) {
          constexpr int i = RK(ii);
          t = m[i + k * N]; m[i + k * N] = m[b + i * N]; m[b + i * N] = t;
        });
      }
    });
    if constexpr (k > 0) {
      double temp[k];
      sf<0, k>(RL(jj) { temp[RK(jj)] = m[RK(jj) + RK(jj) * N] * m[k + RK(jj) * N]; });
      double s = 0;
      sf<0, k>(RL(jj) { s += m[k + RK(jj) * N] * temp[RK(jj)]; });
      m[k + k * N] -= s;
      sf<k + 1, N>(RL(ii) {
        constexpr int i = RK(ii);
        double si = 0;
        sf<0, k>(RL(jj) { si += m[i + RK(jj) * N] * temp[RK(jj)]; });
        m[i + k * N] -= si;
      });
    }
    if constexpr (k == 0) {
      if (!(fabs(m[0]) > 0)) {
        tr[0] = 0;
        stop = true;
        return;
      }
    }
    if constexpr (N - k - 1 > 0) {
      const double d = m[k + k * N];
      if (fabs(d) > 0) sf<k + 1, N>(RL(ii) { m[RK(ii) + k * N] /= d; });
    }
  });
}

// x <- transposition-permuted L'DL solve (oracle ora_ldlt_solve)
template <int N>
__device__ __forceinline__ void swap_rt(double (&x)[N], int a, int b) {
  // x[a] <-> x[b] with a compile-time-unrolled select (a, b runtime)
  double xa = x[0], xb = x[0];
  sf<0, N>(RL(ii) {
    xa = (a == RK(ii)) ? x[RK(ii)] : xa;
    xb = (b == RK(ii)) ? x[RK(ii)] : xb;
  });
  sf<0, N>(RL(ii) {
    if (RK(ii) == a) x[RK(ii)] = xb;
    if (RK(ii) == b) x[RK(ii)] = xa;
  });
}
template <int N>
__device__ __forceinline__ void ldlt_solve_r(const double (&L)[N * N], const int (&tr)[N], double (&x)[N]) {
  const double tol = 2.2250738585072014e-308;
  sf<0, N>(RL(kk) {
    constexpr int k = RK(kk);
    if (tr[k] != k) swap_rt<N>(x, k, tr[k]);
  });
  sf<0, N>(RL(ii) {
    constexpr int i = RK(ii);
    sf<0, i>(RL(jj) { x[i] -= L[i + RK(jj) * N] * x[RK(jj)]; });
  });
  sf<0, N>(RL(ii) {
    constexpr int i = RK(ii);
    if (fabs(L[i + i * N]) > tol) x[i] /= L[i + i * N];
    else x[i] = 0;
  });
  sf<0, N>(RL(ii) {
    constexpr int i = N - 1 - RK(ii);
    sf<i + 1, N>(RL(jj) { x[i] -= L[RK(jj) + i * N] * x[RK(jj)]; });
  });
  sf<0, N>(RL(kk) {
    constexpr int k = N - 1 - RK(kk);
    if (tr[k] != k) swap_rt<N>(x, k, tr[k]);
  });
}

}  // namespace rreg

template <int NV, int NU>
struct RicReg {
  static constexpr int NX = 2 * NV;
  static constexpr bool ok = NV > 0 && NU > 0 && NX % 4 == 0 && NX <= 16 && NU <= 4 && 4 * NX + NU * NU + NU <= 64;
  static constexpr int LX = NX + 2;  // even: every column starts 16-byte aligned
  static constexpr int RP = NX / 4;  // rows per quad lane
  static constexpr int D = NV * (2 * NV + NU) + 2 * NV + NU;
  static constexpr int DP = (D + 1) / 2 * 2;
  // LDS offsets (doubles, all even)
  static constexpr int oV = 0, oABK = oV + NX * LX, oT4 = oABK + NX * LX, oT1 = oT4 + NX * LX,
                       oW = oT1 + NU * NX, oM = oW + NX, oK = oM + (NU * NU + NU + 1) / 2 * 2,
                       oZ = oK + (NU * NX + 1) / 2 * 2, oY = oZ + NX, oVv = oY + NX, oC = oVv + 2 * NX, oDL = oC + 2 * NX,
                       total = oDL + DP;
  static constexpr size_t bytes = (size_t)total * sizeof(double);
};

template <int NV, int NU, class MD>
__device__ inline void backward_seed_reg(const MD& m, int P, double dt, double mu, const double* deriv, int Ds,
                                         TrajDev tr, double* Kg, double* kg, double* Vg, double* vg, int s, int tid,
                                         double* sh, const unsigned* done, unsigned target, unsigned* fault,
                                         RicFlags fl) {
  using R = RicReg<NV, NU>;
  constexpr int NX = R::NX, LX = R::LX, RP = R::RP, D = R::D;
  using namespace rreg;
  (void)m;
  double* Vb = sh + R::oV;
  double* ABKb = sh + R::oABK;
  double* T4b = sh + R::oT4;
  double* T1b = sh + R::oT1;
  double* Wb = sh + R::oW;
  double* Mb = sh + R::oM;
  double* Kb = sh + R::oK;
  double* Zb = sh + R::oZ;
  double* Yb = sh + R::oY;
  double* Vv = sh + R::oVv;  // v, two buffers by step parity
  double* Cb = sh + R::oC;   // c = x*_{n-1} - x*_n, two buffers by step parity
  double* dl = sh + R::oDL;
  const bool quad = tid < 4 * NX;
  const int j = tid >> 2, g = tid & 3;  // quad lane: column j, rows g + 4 r
  const int sp = tid - 4 * NX;          // spare lane index
#ifdef ILQG_STAMPS
  unsigned long long bst_prev = 0;
#endif

  int ready_upto = -1;
  auto ready = [&](int p) __attribute__((always_inline)) {
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
  auto ld = [&](const double* a) -> double __attribute__((always_inline)) { return done ? ld_sc1(a) : *a; };
  constexpr int NPF = (D + 63) / 64;
  auto fetch_rec = [&](size_t pt, double (&pf)[NPF]) __attribute__((always_inline)) {
    const double* src = deriv + pt * Ds;
    sf<0, NPF>(RL(tt) {
      const int i = tid + RK(tt) * 64;
      pf[RK(tt)] = i < D ? ld(src + rec_src(i, NV, NU, fl.layout)) : 0.0;
    });
  };
  auto park_rec = [&](const double (&pf)[NPF]) __attribute__((always_inline)) {
    sf<0, NPF>(RL(tt) {
      const int i = tid + RK(tt) * 64;
      if (i < D) dl[i] = pf[RK(tt)];
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
    double v0 = tid < NX ? (fl.vinit ? vg[(size_t)s * NX + tid] : ld(q0 + tid)) : 0.0;
    if (tid < NX) Vv[tid] = v0;  // parity 0 buffer: v before step 1
    if (P > 1) {
      ready(1);
      double pf[NPF];
      fetch_rec((size_t)s * P + 1, pf);
      park_rec(pf);
    }
    wsync();
    if (quad && fl.vinit) {
      sf<0, RP>(RL(rr) {
        const int i = g + 4 * RK(rr);
        Vb[i + j * LX] = Vg[(size_t)s * NX * NX + i + j * NX];
      });
    } else if (quad) {
      double vv[NX];
      lds_row<NX>(vv, Vv);
      sf<0, RP>(RL(rr) {
        const int i = g + 4 * RK(rr);
        Vb[i + j * LX] = vv[i] * vv[j];  // V = v'v (col-major)
      });
    }
  }
  double xa = 0, xb = 0;
  xa = xload((size_t)s * P);
  if (P > 1) xb = xload((size_t)s * P + 1);
  if (tid < NX) Cb[tid] = xa - xb;  // c for step 1 (parity 1 buffer below is step 2's)
  wsync();
  BSTAMP(-1);

  for (int n = 1; n < P; n++) {
    const size_t pc = (size_t)s * P + n;
    const int par = n & 1;
    const double* cc = Cb + (par ^ 1) * NX;   // step n's c (step 1 in buffer 0)
    double* cnext = Cb + par * NX;
    const double* vold = Vv + (par ^ 1) * NX;  // v entering step n
    double* vnew = Vv + par * NX;
    // next step's record and state, one step ahead
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
    // B[i][a] * dt for a runtime column a: the lower NV rows (upper rows are 0)
    auto bcol = [&](int a_, double (&bl)[NV]) __attribute__((always_inline)) {
      lds_row<NV>(bl, dl + oB + a_ * NV);
      sf<0, NV>(RL(ii) { bl[RK(ii)] = bl[RK(ii)] * dt; });
    };
    // A[i][j] (differentiator.h:66-71), i, j runtime, the oracle's expression
    auto aval = [&](int i, int jc) -> double __attribute__((always_inline)) {
      if (i < NV) {
        if (jc < NV) return (i == jc) ? 1.0 : 0.0;
        return (i == jc - NV) ? dt : 0.0;
      }
      if (jc < NV) return dl[(i - NV) + jc * NV] * dt;
      return ((i - NV) == (jc - NV) ? 1.0 : 0.0) + dl[NV * NV + (i - NV) + (jc - NV) * NV] * dt;
    };
    // ---- A: Vs column j, T1[g][j], w[j] ----
    double vs[NX];
    if (quad) {
      double vc[NX];
      lds_row<NX>(vc, Vb + j * LX);
      sf<0, NX>(RL(ii) {
        constexpr int i = RK(ii);
        vs[i] = (vc[i] + Vb[j + i * LX]) / 2;
      });
      // V.diagonal() += mu (inc/ilqr.h:165-166, quirk Q13): entry (j, j)
      sf<0, NX>(RL(ii) {
        const double d = vs[RK(ii)] + mu;
        vs[RK(ii)] = (RK(ii) == j) ? d : vs[RK(ii)];
      });
      if (g < NU) {
        double bl[NV];
        bcol(g, bl);
        double t1 = 0;
        sf<0, NX>(RL(kk) {
          constexpr int k = RK(kk);
          if constexpr (k < NV) t1 += 0.0 * vs[k];
          else t1 += bl[k - NV] * vs[k];
        });
        T1b[g * NX + j] = t1;  // T1[a][kk] at a NX + kk
      }
      if (g == (NU < 4 ? NU : 0)) {
        double c[NX];
        lds_row<NX>(c, cc);
        double sm = 0;
        sf<0, NX>(RL(jj) { sm += vs[RK(jj)] * c[RK(jj)]; });
        Wb[j] = vold[j] + 2 * sm;
      }
    }
    wsync();
    BSTAMP(0);
    // ---- B: spare lanes Mm, col; quads T3[g][j] ----
    double t3 = 0;
    if (quad) {
      if (g < NU) {
        double t1r[NX];
        lds_row<NX>(t1r, T1b + g * NX);
        // A column j: [delta or dt delta ; dt * deriv block column]
        double al[NV];
        lds_row<NV>(al, dl + (j < NV ? j * NV : NV * NV + (j - NV) * NV));
        sf<0, NX>(RL(kk) {
          constexpr int k = RK(kk);
          double av;
          if constexpr (k < NV) av = j < NV ? ((k == j) ? 1.0 : 0.0) : ((k == j - NV) ? dt : 0.0);
          else av = j < NV ? al[k - NV] * dt : ((k - NV) == (j - NV) ? 1.0 : 0.0) + al[k - NV] * dt;
          t3 += t1r[k] * av;
        });
      }
    } else if (sp < NU * NU) {
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
    } else if (sp < NU * NU + NU) {
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
    wsync();
    BSTAMP(1);
    // ---- C: LDLT (uniform), k; K column j, ABK rows; spare lanes y ----
    double Lm[NU * NU], kf[NU];
    int trn[NU];
    sf<0, NU * NU>(RL(ee) { Lm[RK(ee)] = Mb[RK(ee)]; });
    sf<0, NU>(RL(aa) { kf[RK(aa)] = Mb[NU * NU + RK(aa)]; });
    ldlt_factor_r<NU>(Lm, trn);
    ldlt_solve_r<NU>(Lm, trn, kf);
    double Kc[NU];
    if (quad) {
      // T3 column j from quad lanes 0 .. NU-1
      sf<0, NU>(RL(aa) { Kc[RK(aa)] = 2 * quad_bcast<RK(aa)>(t3); });
      ldlt_solve_r<NU>(Lm, trn, Kc);
      sf<0, RP>(RL(rr) {
        const int i = g + 4 * RK(rr);
        double sm = 0;
        sf<0, NU>(RL(aa) {
          const double bi = i < NV ? 0.0 : dl[oB + (i - NV) + RK(aa) * NV] * dt;
          sm += bi * Kc[RK(aa)];
        });
        ABKb[i + j * LX] = aval(i, j) + sm;
      });
      if (g == 0) {
        sf<0, NU>(RL(aa) {
          Kb[RK(aa) + j * NU] = Kc[RK(aa)];
          Kg[pc * NU * NX + RK(aa) + j * NU] = Kc[RK(aa)];
        });
      }
    } else if (sp < NX) {
      // y = B k + c (ilqr.h:174), one entry per spare lane
      const int i = sp;
      double sm = 0;
      sf<0, NU>(RL(aa) {
        const double bi = i < NV ? 0.0 : dl[oB + (i - NV) + RK(aa) * NV] * dt;
        sm += bi * kf[RK(aa)];
      });
      Yb[i] = sm + cc[i];
    }
    if (tid == 0) sf<0, NU>(RL(aa) { kg[pc * NU + RK(aa)] = kf[RK(aa)]; });
    // kR = k'R (uniform)
    double kR[NU];
    sf<0, NU>(RL(bb) {
      double sm = 0;
      sf<0, NU>(RL(aa) { sm += kf[RK(aa)] * (r[RK(aa)] * r[RK(bb)]); });
      kR[RK(bb)] = sm;
    });
    wsync();
    BSTAMP(2);
    // ---- D: T4 rows R_g of column j; T6 rows R_g ----
    double T6r[RP][NU];
    if (quad) {
      sf<0, RP>(RL(rr) {
        const int i = g + 4 * RK(rr);
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
          T6r[RK(rr)][RK(bb)] = t;
        });
      });
    }
    wsync();
    BSTAMP(3);
    // ---- E: Vn rows R_g of column j (into V's buffer) ----
    double abk[NX];
    if (quad) {
      lds_row<NX>(abk, ABKb + j * LX);
      const double qj = dl[oQ + j];
      sf<0, RP>(RL(rr) {
        const int i = g + 4 * RK(rr);
        double tr4[NX];
        lds_row<NX>(tr4, T4b + i * LX);
        double s5 = 0, s7 = 0;
        sf<0, NX>(RL(kk) { s5 += tr4[RK(kk)] * abk[RK(kk)]; });
        sf<0, NU>(RL(bb) { s7 += T6r[RK(rr)][RK(bb)] * Kc[RK(bb)]; });
        Vb[i + j * LX] = (s5 + dl[oQ + i] * qj) + s7;
      });
    }
    wsync();
    BSTAMP(4);
    // ---- F: z[j] = (2y)' Vn[:, j] ----
    if (quad && g == 0) {
      double vc[NX], y[NX];
      lds_row<NX>(vc, Vb + j * LX);
      lds_row<NX>(y, Yb);
      double sm = 0;
      sf<0, NX>(RL(ii) { sm += (2 * y[RK(ii)]) * vc[RK(ii)]; });
      Zb[j] = sm;
    }
    wsync();
    BSTAMP(5);
    // ---- G: v_new[j]; next step's c, record ----
    if (quad && g == 0) {
      double zz[NX], vv[NX];
      lds_row<NX>(zz, Zb);
      lds_row<NX>(vv, vold);
      double ta = 0, tb = 0, td = 0;
      sf<0, NX>(RL(ii) { ta += zz[RK(ii)] * abk[RK(ii)]; });
      sf<0, NX>(RL(ii) { tb += vv[RK(ii)] * abk[RK(ii)]; });
      sf<0, NU>(RL(bb) { td += (2 * kR[RK(bb)]) * Kc[RK(bb)]; });
      vnew[j] = ((ta + tb) + dl[oQ + j]) + td;
    }
    if (n + 1 < P) {
      if (tid < NX) cnext[tid] = xb - xn;
      park_rec(pf);
    }
    xa = xb;
    xb = xn;
    wsync();
    BSTAMP(6);
    BSTEP_LOG(s, n);
  }
  const double* vfin = Vv + ((P - 1) & 1) * NX;
  if (P == 1) vfin = Vv;
  if (Vg && quad)
    sf<0, RP>(RL(rr) {
      const int i = g + 4 * RK(rr);
      Vg[(size_t)s * NX * NX + i + j * NX] = Vb[i + j * LX];
    });
  if (vg && tid < NX) vg[(size_t)s * NX + tid] = vfin[tid];
}

}  // namespace ilqg
