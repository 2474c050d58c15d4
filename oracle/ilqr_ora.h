/* ORACLE / TEST INFRASTRUCTURE ONLY.  See ilqr_ora.c. */
#pragma once
#include "mujoco/mujoco.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef mjtNum (*stepCostFn_t)(const mjData*);
typedef void (*ora_calc_fn)(mjModel*, mjData*, mjtNum*, stepCostFn_t);

/* diagonal-quadratic + linear cost over (qpos, qvel, ctrl):
   c = sum_i w_i (x_i - t_i)^2 + l_i x_i, terms in (q, v, u) order, i ascending */
typedef struct {
  int nq, nv, nu;
  mjtNum wq[64], tq[64], lq[64];
  mjtNum wv[64], tv[64], lv[64];
  mjtNum wu[64], tu[64], lu[64];
} ora_cost_desc;

typedef struct {
  mjModel* m;
  int N, nv, nu, nx, D;
  mjData* d;
  mjData** dArray;      /* dArray[N] = initial, dArray[0] = terminal (Q11) */
  mjtNum* deriv;        /* (N+1) x D, one FD record per point */
  mjtNum *V, *v;        /* nx x nx col-major, nx */
  mjtNum *K, *k;        /* (N+1) x nu x nx col-major, (N+1) x nu */
  mjtNum mu;
  stepCostFn_t cost;
  ora_calc_fn calc;
  long cout_lines;
} ora_ilqr;

void ora_set_nthread(int n);
void ora_set_fd_eps(double eps); /* FD step (default 1e-6, mjderivative.cpp:39) */
int ora_get_nthread(void);
void ora_cpMjData(const mjModel* m, mjData* dst, const mjData* src);
mjtNum ora_cost_pendulum(const mjData* d);
void ora_set_cost_desc(const ora_cost_desc* desc);
mjtNum ora_cost_desc_fn(const mjData* d);
mjtNum ora_cost_eval_desc(const ora_cost_desc* c, const mjtNum* qpos, const mjtNum* qvel, const mjtNum* ctrl);

void ora_calcMJDerivatives(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t cost);
void ora_calcMJDerivatives_tuned(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t cost,
                                 mjData** pool, int npool);
void ora_set_layout(int layout); /* 0 reference (quirk Q1), 1 corrected */
int ora_get_layout(void);
void ora_assemble_AB(int nv, int nu, mjtNum dt, const mjtNum* deriv, mjtNum* A, mjtNum* B);
int ora_ldlt_factor(int n, mjtNum* mat, int* transp);
void ora_ldlt_solve(int n, const mjtNum* L, const int* transp, mjtNum* x);
void ora_riccati_step(int nv, int nu, mjtNum dt, mjtNum mu, const mjtNum* deriv,
                      const mjtNum* xprev, const mjtNum* xcur, mjtNum* V, mjtNum* v,
                      mjtNum* K, mjtNum* kff);

void ora_riccati_step_c(int nv, int nu, mjtNum dt, mjtNum mu, const mjtNum* deriv, const mjtNum* c,
                        mjtNum* V, mjtNum* v, mjtNum* K, mjtNum* kff);
void ora_state_diff(const mjModel* m, const mjtNum* qa, const mjtNum* va, const mjtNum* qb, const mjtNum* vb,
                    mjtNum* dx);

ora_ilqr* ora_ilqr_create(mjModel* m, const mjData* dmain, int N, stepCostFn_t cost, ora_calc_fn calc);
void ora_ilqr_free(ora_ilqr* s);
void ora_ilqr_setDInit(ora_ilqr* s, const mjData* dinit);
void ora_ilqr_forwardPass(ora_ilqr* s);
void ora_ilqr_fd_point(ora_ilqr* s, int n);
void ora_calc_none(mjModel* m, mjData* d, mjtNum* deriv, stepCostFn_t cost);
void ora_ilqr_backwardPass(ora_ilqr* s);
void ora_ilqr_backwardPass_v0(ora_ilqr* s, const mjtNum* V0, const mjtNum* v0);
void ora_ilqr_iterate(ora_ilqr* s);
void ora_ilqr_iterate_v0(ora_ilqr* s, const mjtNum* V0, const mjtNum* v0);
void ora_ilqr_forward_candidates(ora_ilqr* s, int A, const mjtNum* alphas, int select_mode, mjtNum* costs,
                                 int* selected);
void ora_ilqr_iterate_ls(ora_ilqr* s, int A, const mjtNum* alphas, int select_mode, mjtNum* costs, int* selected);
void ora_ilqr_set_gains(ora_ilqr* s, const mjtNum* K, const mjtNum* k);
void ora_ilqr_get_traj(const ora_ilqr* s, mjtNum* time, mjtNum* qpos, mjtNum* qvel, mjtNum* warm,
                       mjtNum* ctrl);

#ifdef __cplusplus
}
#endif
