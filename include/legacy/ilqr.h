// Legacy ILQR<nv,nu,N> (reference: inc/ilqr.h:14-188) over the MI355X path.
//
// Same constructor, public members and methods, so callers such as
// src/inverted_pendulum/inverted_pendulum.cpp compile unchanged:
//   ILQR<nv,nu,N>(m, dmain, stepCostFn); setDInit(d); iterate();
//   dArray[N]->ctrl (the first control of the optimised trajectory).
// The passes run on the GPU (include/ilqg_amd.h, one seed, reference
// semantics: alpha = 1, mu = 1000).  dArray / K / k / V / v are host mirrors,
// uploaded before and refreshed after every pass.  Eigen is not required: K, k,
// V, v are column-major ilqg_legacy::Mat with Eigen's storage order.
// Unlike the reference, every ILQR instance owns its own state (the
// reference's function-static references in backwardPass, inc/ilqr.h:137-140,
// would alias two instances of one <nv,nu,N>).
#pragma once

#include "differentiator.h"
#include "ilqg_legacy.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"
#include "util.h"

template <int nv, int nu, int N>
class ILQR {
 public:
  typedef ilqg_legacy::Mat<nu, 2 * nv> K_t;
  typedef ilqg_legacy::Mat<nu, 1> k_t;
  typedef ilqg_legacy::Mat<2 * nv, 2 * nv> V_t;
  typedef ilqg_legacy::Mat<1, 2 * nv> v_t;

  mjModel* m;
  mjData* d = NULL;
  Differentiator<nv, nu>* differentiator;
  mjData* dArray[N + 1];  // dArray[N]: initial state, dArray[0]: terminal state
  V_t* V;
  v_t* v;
  K_t K[N + 1];
  k_t k[N + 1];
  mjtNum mu = 1000.0;  // the device solver is created with this value

  ILQR(mjModel* m, mjData* dmain, stepCostFn_t& stepCostFn) : m(m), core_(m, N, stepCostFn) {
    static_assert(sizeof(K_t) == sizeof(mjtNum) * nu * 2 * nv, "K must be dense");
    d = mj_makeData(m);
    cpMjData(m, d, dmain);
    differentiator = new Differentiator<nv, nu>(m, d, stepCostFn);
    for (int n = N; n >= 0; n--) dArray[n] = mj_makeData(m);
    V = new V_t;
    v = new v_t;
    core_.init(dmain, dArray);
  }
  virtual ~ILQR() {
    for (int n = 0; n <= N; n++) mj_deleteData(dArray[n]);
    mj_deleteData(d);
    delete differentiator;
    delete V;
    delete v;
  }

  // initV runs on the device at the start of backwardPass (inc/ilqr.h:100-107)
  virtual void initV() {}

  void setDInit(mjData* dInit) {
    cpMjData(m, d, dInit);
    core_.set_dinit(d);
  }

  void forwardPass() { core_.forward(dArray, K[0].data(), k[0].data()); }

  void backwardPass() { core_.backward(dArray, K[0].data(), k[0].data(), V->data(), v->data()); }

  void iterate() {
    core_.iterate(dArray, K[0].data(), k[0].data(), V->data(), v->data());
    cpMjData(m, d, dArray[N]);
  }

 private:
  ilqg_legacy::SolverCore core_;
};
