/* Line-search certification study (VERDICT r5 "Next" #2).  STUDY TOOL, not product.
 *
 * The FD sweep's Newton line searches (oracle/mjsub.c linesearch, restating
 * MuJoCo 2.0's exact line search at tolerance 0, src/mjderivative.cpp:241-242)
 * run 62.5 % of their calls to LS_ITER = 50, mostly as bisection levels.  A
 * bisection level's midpoint is fixed by the bracket alone; only the SIGN of
 * d1 there (lo or hi moves), the break test |d1| < gtol and the next level's
 * Newton-candidate test need d1.  If all three can be decided from a cheap
 * rigorous bound, the level's row sums could be skipped without changing a
 * bit.  This study measures, over the bench workload's sweep, how many
 * bisection levels are decidable at all:
 *
 *   d1 is recomputed in long double (64-bit mantissa) from the same fp64
 *   inputs (the "true" value of the expression the oracle evaluates), and the
 *   fp64 evaluation's rounding error is bounded by
 *     e = (ne + 4) u (|g1| + |g2 a| + sum_i |D_i| |Jv_i| (|jar_i| + |a Jv_i|))
 *   (u = 2^-53; rows whose activation x = jar + a Jv lies within that bound of 0
 *   are included in the sum either way).  A level is decidable when
 *     sign:  |d1_true| > e
 *     break: |d1_true| - e >= gtol
 *     next:  the next level's candidate alpha - d1/d2 is outside the new
 *            bracket by more than e/|d2| + 4 ulp(alpha) (so it bisects again;
 *            a Newton step needs the exact d1) -- or this was the last level.
 * Any certification scheme (a piecewise-linear root with interval bounds) can
 * at best skip the decidable levels.
 */
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#define MAXNE 64
static int s_ne;
static double s_Jv[MAXNE], s_jar[MAXNE], s_D[MAXNE], s_g1, s_g2, s_gtol;
static long n_calls, n_iters, n_bis, n_dec, n_sign, n_brk, n_next, n_full;
static long n_bis_ne[4], n_dec_ne[4];
static int pend_valid;           /* the previous level was a bisection awaiting its "next" test */
static int pend_sign, pend_brk;  /* its sign / break certificates */
static double pend_lo, pend_hi, pend_alpha, pend_d1t, pend_e, pend_d2;
static int pend_ne_cls;
static int call_iters;

static int ne_cls(int ne) { return ne <= 4 ? 0 : ne <= 8 ? 1 : ne <= 16 ? 2 : 3; }

void ora_ls_study_begin(int ne, const double* Jv, const double* jar, const double* D, double g1, double g2,
                        double d1, double d2, double gtol) {
  (void)d1; (void)d2;
  s_ne = ne < MAXNE ? ne : MAXNE;
  memcpy(s_Jv, Jv, s_ne * sizeof(double));
  memcpy(s_jar, jar, s_ne * sizeof(double));
  memcpy(s_D, D, s_ne * sizeof(double));
  s_g1 = g1; s_g2 = g2; s_gtol = gtol;
  pend_valid = 0;
  call_iters = 0;
  n_calls++;
}

static void settle(int next_ok) {
  if (!pend_valid) return;
  int dec = pend_sign && pend_brk && next_ok;
  n_bis++; n_bis_ne[pend_ne_cls]++;
  n_sign += pend_sign; n_brk += pend_brk; n_next += next_ok;
  if (dec) { n_dec++; n_dec_ne[pend_ne_cls]++; }
  pend_valid = 0;
}

void ora_ls_study_iter(int it, int bisect, double lo, double hi, double a, double d1, double d2) {
  n_iters++;
  call_iters++;
  /* the previous bisection level's "next" certificate: this level's decision */
  if (pend_valid) {
    /* the candidate the oracle formed from the previous level's d1 */
    long double cand = (long double)pend_alpha - pend_d1t / (long double)pend_d2;
    long double err = pend_e / fabs(pend_d2) + 4.0L * nextafter(fabs(pend_alpha), INFINITY) - 4.0L * fabs(pend_alpha);
    /* new bracket after the previous level */
    double nlo = pend_d1t < 0 ? pend_alpha : pend_lo, nhi = pend_d1t < 0 ? pend_hi : pend_alpha;
    int outside = (cand <= nlo - err) || (cand >= nhi + err);
    settle(bisect && outside);
  }
  if (!bisect) return;
  long double s = (long double)s_g1 + (long double)s_g2 * a, bound = fabs(s_g1) + fabs(s_g2 * a);
  for (int i = 0; i < s_ne; i++) {
    long double x = (long double)s_jar[i] + (long double)a * s_Jv[i];
    long double mag = fabsl((long double)s_D[i] * s_Jv[i]) * (fabs(s_jar[i]) + fabs(a * s_Jv[i]));
    if (x < 0) s += (long double)s_D[i] * x * s_Jv[i];
    bound += mag;
  }
  long double e = (s_ne + 4) * ldexpl(1.0L, -53) * bound;
  static int ndump = 0;
  if (getenv("LS_STUDY_DUMP") && (getenv("LS_STUDY_BIG") ? fabsl(s) > e : 1) && ndump++ < 40)
    fprintf(stderr, "it %d ne %d a %.17g lo %.17g hi %.17g d1 %.6Le d1_64 %.6e e %.3Le gtol %.3e d2 %.3e g1 %.3e\n", it, s_ne,
            a, lo, hi, s, d1, e, s_gtol, d2, s_g1);
  pend_valid = 1;
  pend_sign = fabsl(s) > e && ((s < 0) == (d1 < 0));
  pend_brk = fabsl(s) - e >= s_gtol;
  pend_lo = lo; pend_hi = hi; pend_alpha = a; pend_d1t = (double)s; pend_e = (double)e; pend_d2 = d2;
  pend_ne_cls = ne_cls(s_ne);
  if (it == 49) settle(1);
}

void ora_ls_study_end(void) {
  if (pend_valid) settle(1);  /* the search ended (break or LS_ITER): no next level */
  if (call_iters == 50) n_full++;
}

void ora_ls_study_report(char* out, int cap) {
  snprintf(out, cap,
           "{\"calls\": %ld, \"calls_to_ls_iter\": %ld, \"iterations\": %ld, \"bisection_levels\": %ld, "
           "\"decidable_levels\": %ld, \"sign_certified\": %ld, \"break_certified\": %ld, \"next_certified\": %ld, "
           "\"bisection_levels_by_ne\": {\"<=4\": %ld, \"5-8\": %ld, \"9-16\": %ld, \">16\": %ld}, "
           "\"decidable_by_ne\": {\"<=4\": %ld, \"5-8\": %ld, \"9-16\": %ld, \">16\": %ld}}",
           n_calls, n_full, n_iters, n_bis, n_dec, n_sign, n_brk, n_next, n_bis_ne[0], n_bis_ne[1], n_bis_ne[2],
           n_bis_ne[3], n_dec_ne[0], n_dec_ne[1], n_dec_ne[2], n_dec_ne[3]);
}

void ora_ls_study_reset(void) {
  n_calls = n_iters = n_bis = n_dec = n_sign = n_brk = n_next = n_full = 0;
  memset(n_bis_ne, 0, sizeof n_bis_ne);
  memset(n_dec_ne, 0, sizeof n_dec_ne);
}
