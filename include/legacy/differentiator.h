// Legacy Differentiator<nv,nu> (reference: inc/differentiator.h:9-95) over the
// GPU FD sweep.  Same public members and methods; the Eigen maps become
// pointers into `deriv` and column-major ilqg_legacy::Mat for A and B.
#pragma once

#include "ilqg_legacy.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"

template <int nv, int nu>
class Differentiator {
 public:
  typedef ilqg_legacy::Mat<2 * nv, 2 * nv> A_t;
  typedef ilqg_legacy::Mat<2 * nv, nu> B_t;

  mjModel* m;
  mjData* d;
  mjtNum* deriv;       // nv*(2nv+nu) + 2nv + nu, mjderivative.cpp layout
  mjtNum* dqaccdq;     // deriv + 0          (read column-major, differentiator.h:57)
  mjtNum* dqaccdqvel;  // deriv + nv*nv
  mjtNum* dqaccdctrl;  // deriv + 2*nv*nv
  mjtNum* dgdx;        // deriv + nv*(2nv+nu), 2nv entries (qpos then qvel)
  mjtNum* dgdu;        // dgdx + 2nv, nu entries
  mjtNum* x;           // d->qpos (qvel follows in memory)
  mjtNum* u;           // d->ctrl
  A_t* A;
  B_t* B;

  Differentiator(mjModel* m, mjData* d, stepCostFn_t& stepCostFn) : m(m), d(d), stepCostFn_(stepCostFn) {
    deriv = static_cast<mjtNum*>(mju_malloc(sizeof(mjtNum) * (nv * (2 * nv + nu) + 2 * nv + nu)));
    mju_zero(deriv, nv * (2 * nv + nu) + 2 * nv + nu);
    dqaccdq = deriv;
    dqaccdqvel = deriv + nv * nv;
    dqaccdctrl = deriv + 2 * nv * nv;
    dgdx = deriv + nv * (2 * nv + nu);
    dgdu = dgdx + 2 * nv;
    A = new A_t;
    B = new B_t;
    setMJData(d);
  }
  ~Differentiator() {
    mju_free(deriv);
    delete A;
    delete B;
  }

  void setMJData(mjData* dnew) {
    d = dnew;
    x = d->qpos;
    u = d->ctrl;
  }

  // calcMJDerivatives at d, then A = [[I, dt I], [dt M_q, I + dt M_v]],
  // B = [[0], [dt M_u]] with M_* the column-major views of the row-major blocks
  // (differentiator.h:66-71,89-92, quirk Q1 kept).
  void updateDerivatives() {
    calcMJDerivatives(m, d, deriv, stepCostFn_);
    const mjtNum dt = m->opt.timestep;
    for (int j = 0; j < 2 * nv; j++)
      for (int i = 0; i < 2 * nv; i++) {
        mjtNum val;
        if (i < nv && j < nv) val = (i == j) ? 1 : 0;
        else if (i < nv) val = (i == j - nv) ? dt : 0;
        else if (j < nv) val = dqaccdq[(i - nv) + j * nv] * dt;
        else val = ((i - nv) == (j - nv) ? 1 : 0) + dqaccdqvel[(i - nv) + (j - nv) * nv] * dt;
        (*A)(i, j) = val;
      }
    for (int j = 0; j < nu; j++)
      for (int i = 0; i < 2 * nv; i++) (*B)(i, j) = (i < nv) ? 0 : dqaccdctrl[(i - nv) + j * nv] * dt;
  }

 private:
  stepCostFn_t stepCostFn_;
};
