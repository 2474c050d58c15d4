// Legacy Differentiator<nv,nu> (reference: inc/differentiator.h:9-95) over the
// GPU FD sweep.  Same typedefs, public members and methods; the Eigen types
// become ilqg_legacy::Mat (owned, column-major) and ilqg_legacy::Map (views
// into `deriv` / mjData, column-major, re-seatable with placement new).
#pragma once

#include <new>

#include "ilqg_legacy.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"

template <int nv, int nu, int N>
class ILQR;

template <int nv, int nu>
class Differentiator {
 public:
  // typedefs for env matrices/vectors (differentiator.h:14-18)
  typedef ilqg_legacy::Mat<2 * nv, 2 * nv> A_t;
  typedef ilqg_legacy::Mat<2 * nv, nu> B_t;
  typedef ilqg_legacy::Mat<2 * nv, 1> x_t;
  typedef ilqg_legacy::Mat<nu, 1> u_t;
  // typedefs for env maps (differentiator.h:19-28)
  typedef ilqg_legacy::Map<nv, nv> dqdq_mt;
  typedef ilqg_legacy::Map<nv, nu> dqdu_mt;
  typedef ilqg_legacy::Map<nv, 1> qpos_mt;
  typedef ilqg_legacy::Map<nv, 1> qvel_mt;
  typedef ilqg_legacy::Map<nv, 1> ctrl_mt;
  typedef ilqg_legacy::Map<2 * nv, 1> x_mt;
  typedef ilqg_legacy::Map<nu, 1> u_mt;
  typedef ilqg_legacy::Map<1, 2 * nv> q_mt;
  typedef ilqg_legacy::Map<1, nu> r_mt;

  mjModel* m;
  mjData* d;
  mjtNum* deriv;  // nv*(2nv+nu) + 2nv + nu doubles, src/mjderivative.cpp layout
  // column-major views of the row-major deriv blocks (differentiator.h:57-59, quirk Q1)
  dqdq_mt* dqaccdq;
  dqdq_mt* dqaccdqvel;
  dqdu_mt* dqaccdctrl;
  stepCostFn_t& stepCostFn;  // bound to the caller's variable, as the reference's
  q_mt* dgdx;                // cost gradient w.r.t. (qpos, qvel)
  r_mt* dgdu;                // ... and ctrl
  x_mt* x;                   // (qpos, qvel) of d: qvel follows qpos in memory
  u_mt* u;                   // ctrl of d
  A_t* A;
  B_t* B;

  Differentiator(mjModel* m, mjData* d, stepCostFn_t& stepCostFn) : m(m), d(d), stepCostFn(stepCostFn) {
    deriv = static_cast<mjtNum*>(mju_malloc(sizeof(mjtNum) * kD));
    mju_zero(deriv, kD);
    dqaccdq = new dqdq_mt(deriv);
    dqaccdqvel = new dqdq_mt(deriv + nv * nv);
    dqaccdctrl = new dqdu_mt(deriv + 2 * nv * nv);
    dgdx = new q_mt(deriv + 2 * nv * nv + nv * nu);
    dgdu = new r_mt(deriv + 2 * nv * nv + nv * nu + 2 * nv);
    x = new x_mt(d->qpos);
    u = new u_mt(d->ctrl);
    A = new A_t;
    B = new B_t;
    // invariant parts (differentiator.h:66-71): A top = [I, dt I], B top = 0
    const mjtNum dt = m->opt.timestep;
    for (int i = 0; i < nv; i++) {
      (*A)(i, i) = 1;
      (*A)(i, nv + i) = dt;
    }
  }
  ~Differentiator() {
    mju_free(deriv);
    delete dqaccdq;
    delete dqaccdqvel;
    delete dqaccdctrl;
    delete dgdx;
    delete dgdu;
    delete x;
    delete u;
    delete A;
    delete B;
  }
  Differentiator(const Differentiator&) = delete;
  Differentiator& operator=(const Differentiator&) = delete;

  void setMJData(mjData* dStar) {
    d = dStar;
    new (x) x_mt(d->qpos);
    new (u) u_mt(d->ctrl);
  }

  // calcMJDerivatives at d (on the GPU), then A/B (differentiator.h:85-93)
  void updateDerivatives() {
    calcMJDerivatives(m, d, deriv, stepCostFn);
    assemble();
  }

 private:
  template <int, int, int>
  friend class ILQR;
  static constexpr int kD = nv * (2 * nv + nu) + 2 * nv + nu;

  // A lower = [dt M_q, I + dt M_v], B lower = dt M_u with M_* the column-major
  // views of the row-major blocks (differentiator.h:89-92, quirk Q1 kept)
  void assemble() {
    const mjtNum dt = m->opt.timestep;
    for (int j = 0; j < nv; j++)
      for (int i = 0; i < nv; i++) {
        (*A)(nv + i, j) = (*dqaccdq)(i, j) * dt;
        (*A)(nv + i, nv + j) = (i == j ? 1 : 0) + (*dqaccdqvel)(i, j) * dt;
      }
    for (int j = 0; j < nu; j++)
      for (int i = 0; i < nv; i++) (*B)(nv + i, j) = (*dqaccdctrl)(i, j) * dt;
  }
};
