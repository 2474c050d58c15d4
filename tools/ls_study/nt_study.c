/* Newton factor speculation study (STUDY TOOL): in the rollout's constraint
 * solves, how often does the active set a full step (alpha = 1) would give
 * equal the active set after the line search, when that set differs from the
 * one the current Hessian factor was built for (a rebuild)?  A helper wave
 * could build the alpha = 1 factor while the primary runs the line search.
 * Hooked into oracle/mjsub.c solver_newton (-DORA_NT_STUDY). */
#include <stdio.h>
#include <string.h>
static long n_iter, n_rebuild, n_hit, n_alpha1;
void ora_nt_study_iter(int ne, const double* jar, const double* Jv, double alpha, const int* state) {
  n_iter++;
  if (alpha == 0) return;
  int rebuild = 0, hit = 1;
  for (int i = 0; i < ne; i++) {
    int now = (jar[i] + alpha * Jv[i]) < 0, one = (jar[i] + Jv[i]) < 0;
    if (now != (state[i] != 0)) rebuild = 1; /* efc_state: the set the current factor was built for */
    if (now != one) hit = 0;
  }
  n_alpha1 += alpha == 1.0;
  if (rebuild) {
    n_rebuild++;
    n_hit += hit;
  }
}
void ora_nt_study_report(char* out, int cap) {
  snprintf(out, cap, "{\"newton_iterations\": %ld, \"alpha_exactly_1\": %ld, \"rebuilds\": %ld, \"rebuilds_predicted_by_alpha1_set\": %ld}",
           n_iter, n_alpha1, n_rebuild, n_hit);
}
void ora_nt_study_reset(void) { n_iter = n_rebuild = n_hit = n_alpha1 = 0; }
