/* ORACLE / TEST INFRASTRUCTURE ONLY: flat accessors so tests can drive the
   oracle through ctypes without mirroring struct layouts. */
#include "ilqr_ora.h"
#ifdef __cplusplus
extern "C" {  /* the instrumented C++ build (flops/) keeps C names */
#endif

void ora_model_info(const mjModel* m, int* out, double* dt) {
  out[0] = m->nq; out[1] = m->nv; out[2] = m->nu; out[3] = m->nbody; out[4] = m->njnt;
  out[5] = m->ngeom; out[6] = m->nconmax; out[7] = m->njmax; out[8] = m->nstack; out[9] = m->nbuffer;
  *dt = (double)m->opt.timestep;
}
mjtNum* ora_d_field(mjData* d, int which) {
  switch (which) {
    case 0: return d->qpos;
    case 1: return d->qvel;
    case 2: return d->ctrl;
    case 3: return d->qacc;
    case 4: return d->qacc_warmstart;
    case 5: return d->qfrc_applied;
    case 6: return d->xfrc_applied;
    case 7: return &d->time;
    case 8: return d->qfrc_bias;
    case 9: return d->qM;
    case 10: return d->qacc_smooth;
    case 11: return d->efc_J;
    case 12: return d->xpos;
    case 13: return d->efc_D;
    case 14: return d->efc_aref;
    default: return 0;
  }
}
int ora_d_int(const mjData* d, int which) {
  switch (which) {
    case 0: return d->ncon;
    case 1: return d->nefc;
    case 2: return d->solver_iter;
    case 3: return d->maxuse_stack;
    default: return -1;
  }
}
void ora_set_solver(mjModel* m, int iterations, double tolerance) {
  m->opt.iterations = iterations;
  m->opt.tolerance = tolerance;
}
void ora_get_solver(const mjModel* m, int* iterations, double* tolerance) {
  *iterations = m->opt.iterations;
  *tolerance = (double)m->opt.tolerance;
}
#ifdef __cplusplus
}
#endif
