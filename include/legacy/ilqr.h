// Legacy ILQR<nv,nu,N> (reference: inc/ilqr.h:14-188) over the MI355X path.
//
// Same typedefs, constructor, public members and methods, so callers such as
// src/inverted_pendulum/inverted_pendulum.cpp compile unchanged:
//   ILQR<nv,nu,N>(m, dmain, stepCostFn); setDInit(d); iterate();
//   dArray[N]->ctrl (the first control of the optimised trajectory).
// The passes run on the GPU (include/ilqg_amd.h, one seed, reference
// semantics: alpha = 1; mu is the public member, read by every backwardPass).  dArray / K / k / V / v are host mirrors,
// uploaded before and refreshed after every pass.  Eigen is not required: the
// matrices are column-major ilqg_legacy::Mat (Eigen's storage order) and the
// *_mt maps ilqg_legacy::Map views.
//
// initV is virtual, as in the reference (inc/ilqr.h:100,142): backwardPass
// calls it, and the V / v it leaves (the terminal FD's v = dgdx, V = v'v by
// default, or whatever an override sets) seed the device recursion
// (ilqg_solver_set_value).  backwardPass runs the FD sweep over every point
// first (the sweep does not depend on V), so the default initV reads the
// terminal record the sweep already formed instead of launching its own FD;
// if an override changes any dArray[n] the sweep is run again, as the
// reference would differentiate the changed state.
//
// Unlike the reference, every ILQR instance owns its own state (the
// reference's function-static references in backwardPass, inc/ilqr.h:137-140,
// would alias two instances of one <nv,nu,N>), and the destructor frees it.
#pragma once

#include <new>

#include "differentiator.h"
#include "ilqg_legacy.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"
#include "util.h"

template <int nv, int nu, int N>
class ILQR {
 public:
  // typedefs for env matrices/vectors (inc/ilqr.h:19-23)
  typedef ilqg_legacy::Mat<2 * nv, 2 * nv> A_t;
  typedef ilqg_legacy::Mat<2 * nv, nu> B_t;
  typedef ilqg_legacy::Mat<2 * nv, 1> x_t;
  typedef ilqg_legacy::Mat<nu, 1> u_t;
  // typedefs for env maps (inc/ilqr.h:24-33)
  typedef ilqg_legacy::Map<nv, nv> dqdq_mt;
  typedef ilqg_legacy::Map<nv, nu> dqdu_mt;
  typedef ilqg_legacy::Map<nv, 1> qpos_mt;
  typedef ilqg_legacy::Map<nv, 1> qvel_mt;
  typedef ilqg_legacy::Map<nv, 1> ctrl_mt;
  typedef ilqg_legacy::Map<2 * nv, 1> x_mt;
  typedef ilqg_legacy::Map<nu, 1> u_mt;
  typedef ilqg_legacy::Map<1, 2 * nv> q_mt;
  typedef ilqg_legacy::Map<1, nu> r_mt;
  // typedefs specific to iLQR (inc/ilqr.h:34-40)
  typedef ilqg_legacy::Mat<nu, 2 * nv> K_t;
  typedef ilqg_legacy::Mat<nu, 1> k_t;
  typedef ilqg_legacy::Mat<2 * nv, 2 * nv> V_t;
  typedef ilqg_legacy::Mat<1, 2 * nv> v_t;
  typedef ilqg_legacy::Mat<2 * nv, 2 * nv> Q_t;
  typedef ilqg_legacy::Mat<nu, nu> R_t;

  mjModel* m;
  mjData* d = NULL;
  Differentiator<nv, nu>* differentiator;
  mjData* dArray[N + 1];  // dArray[N]: initial state, dArray[0]: terminal state
  V_t* V;
  v_t* v;
  K_t K[N + 1];  // K/k[0] are never computed (inc/ilqr.h:56); zero here (quirk Q12)
  k_t k[N + 1];
  // (qpos, qvel) and ctrl of d; xStar / uStar are re-seated per point by
  // forwardPass and left on dArray[0] (inc/ilqr.h:59-62,90-93,124-125)
  x_mt* x;
  u_mt* u;
  x_mt* xStar;
  u_mt* uStar;
  mjtNum mu = 1000.0;  // inc/ilqr.h:65; uploaded by every backwardPass (ilqr.h:166)

  ILQR(mjModel* m, mjData* dmain, stepCostFn_t& stepCostFn) : m(m), core_(m, N, stepCostFn) {
    static_assert(sizeof(K_t) == sizeof(mjtNum) * nu * 2 * nv, "K must be dense");
    d = mj_makeData(m);
    setDInit(dmain);
    differentiator = new Differentiator<nv, nu>(m, d, stepCostFn);
    for (int n = N; n >= 0; n--) dArray[n] = mj_makeData(m);
    // initial passive rollout on the device (inc/ilqr.h:82-87); d then holds
    // the state one step past dArray[0], as the reference's loop leaves it
    core_.init(dmain, dArray);
    step_past_terminal();
    x = new x_mt(d->qpos);
    u = new u_mt(d->ctrl);
    xStar = new x_mt(d->qpos);
    uStar = new u_mt(d->ctrl);
    V = new V_t;
    v = new v_t;
  }
  virtual ~ILQR() {
    for (int n = 0; n <= N; n++) mj_deleteData(dArray[n]);
    mj_deleteData(d);
    delete differentiator;
    delete x;
    delete u;
    delete xStar;
    delete uStar;
    delete V;
    delete v;
  }
  ILQR(const ILQR&) = delete;
  ILQR& operator=(const ILQR&) = delete;

  // inc/ilqr.h:100-107: FD at the terminal point (on the GPU), v = dgdx, V = v'v.
  // Inside backwardPass the sweep's record of dArray[0] is that FD (the same
  // bits); called elsewhere, or after dArray[0] changed, it runs its own.
  virtual void initV() {
    differentiator->setMJData(dArray[0]);
    if (core_.deriv_current(0, dArray[0])) {
      mju_copy(differentiator->deriv, core_.deriv(0), Differentiator<nv, nu>::kD);
      differentiator->assemble();
    } else {
      differentiator->updateDerivatives();
    }
    for (int i = 0; i < 2 * nv; i++) (*v)(0, i) = (*differentiator->dgdx)(0, i);
    for (int j = 0; j < 2 * nv; j++)
      for (int i = 0; i < 2 * nv; i++) (*V)(i, j) = (*v)(0, i) * (*v)(0, j);
  }

  void setDInit(mjData* dInit) { cpMjData(m, d, dInit); }

  // inc/ilqr.h:116-130: u = K[n](x - x*) + k[n] + u*, store, mj_step, n = N..0
  // (on the device, from the state in d)
  void forwardPass() {
    core_.set_dinit(d);
    core_.forward(dArray, K[0].data(), k[0].data());
    step_past_terminal();
    new (xStar) x_mt(dArray[0]->qpos);
    new (uStar) u_mt(dArray[0]->ctrl);
  }

  // inc/ilqr.h:133-176: the FD sweep over dArray, initV (virtual), then the
  // Riccati recursion n = 1..N with the current mu on the device; the
  // differentiator is left at dArray[N] with its A / B, as the reference's last
  // updateDerivatives leaves it
  void backwardPass() {
    core_.sweep(dArray);
    initV();
    // the reference differentiates dArray[n] inside its loop, after initV
    // (inc/ilqr.h:142-154): an initV override that changed any point since the
    // sweep gets those points differentiated again at their new state
    if (!core_.traj_current(dArray)) core_.sweep(dArray);
    core_.riccati(mu, K[0].data(), k[0].data(), V->data(), v->data());
    differentiator->setMJData(dArray[N]);
    mju_copy(differentiator->deriv, core_.deriv(N), Differentiator<nv, nu>::kD);
    differentiator->assemble();
  }

  // inc/ilqr.h:179-186
  void iterate() {
    forwardPass();
    setDInit(dArray[N]);
    backwardPass();
  }

 private:
  // d = dArray[0] stepped once: the reference's rollout loops (inc/ilqr.h:82-87,
  // 121-129) end with d one mj_step past the terminal point
  void step_past_terminal() {
    cpMjData(m, d, dArray[0]);
    mj_step(m, d);
  }
  ilqg_legacy::SolverCore core_;
};
