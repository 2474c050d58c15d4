// Legacy-boundary check program (tests/test_legacy.py): a caller that touches
// every public type, member and method SURVEY.md §8b lists for
// Differentiator<nv,nu> (/root/reference/inc/differentiator.h:14-93) and
// ILQR<nv,nu,N> (/root/reference/inc/ilqr.h:19-186), and an ILQR subclass that
// overrides the virtual initV (inc/ilqr.h:100,142).  Built against
// include/legacy and libilqg_mujoco.so by ilqg-mujoco_amd/Makefile.
//
//   legacy_members model.xml members   reference semantics of the members (GPU)
//   legacy_members model.xml initv N   N iterate() of the initV-override subclass;
//                                      prints K, k, V, v and the trajectory as hex
//   legacy_members model.xml mu X N    N iterate() of a plain ILQR whose public mu
//                                      was set to X first (inc/ilqr.h:65,166); same output
//   legacy_members model.xml mutate    one iterate() of a subclass whose initV changes
//                                      dArray[N/2] after the default; same output
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "differentiator.h"
#include "ilqr.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"
#include "update.h"
#include "util.h"

namespace {

constexpr int kNv = 2, kNu = 1, kN = 20;

// inc/inverted_pendulum/cost.h:7-17
mjtNum stepCost(const mjData* d) {
  return 1.0 * d->qpos[0] * d->qpos[0] + 10.0 * d->qpos[1] * d->qpos[1] + 1.0 * d->qvel[0] * d->qvel[0] +
         10.0 * d->qvel[1] * d->qvel[1] + 1.0 * d->ctrl[0] * d->ctrl[0];
}

// the terminal value an override installs: V0(i, j) = 0.5 (i + 1) delta_ij + 0.125 (i + j), v0(i) = i - 1.5
template <int nv, int nu, int N>
class FixedTerminal : public ILQR<nv, nu, N> {
 public:
  using Base = ILQR<nv, nu, N>;
  FixedTerminal(mjModel* m, mjData* d, stepCostFn_t& fn) : Base(m, d, fn) {}
  int calls = 0;
  void initV() override {
    calls++;
    for (int j = 0; j < 2 * nv; j++) {
      (*this->v)(0, j) = j - 1.5;
      for (int i = 0; i < 2 * nv; i++) (*this->V)(i, j) = (i == j ? 0.5 * (i + 1) : 0.0) + 0.125 * (i + j);
    }
  }
};

// the default terminal value, then a later point changed (qvel[0] of
// dArray[N / 2] += 1e-3): the recursion must differentiate that point at its
// new state, as the reference's loop would (inc/ilqr.h:142-154)
template <int nv, int nu, int N>
class MutatingTerminal : public ILQR<nv, nu, N> {
 public:
  using Base = ILQR<nv, nu, N>;
  MutatingTerminal(mjModel* m, mjData* d, stepCostFn_t& fn) : Base(m, d, fn) {}
  void initV() override {
    Base::initV();
    this->dArray[N / 2]->qvel[0] += 1e-3;
  }
};

int fails = 0;
void expect(bool ok, const char* what) {
  if (!ok) {
    fprintf(stderr, "FAIL: %s\n", what);
    fails++;
  }
}

void hex(const char* tag, const mjtNum* a, int n) {
  printf("%s", tag);
  for (int i = 0; i < n; i++) printf(" %a", a[i]);
  printf("\n");
}

int members(mjModel* m, mjData* d0) {
  stepCostFn_t fn = stepCost;
  // ---- Differentiator<nv,nu>: typedefs, members, methods ----
  using D = Differentiator<kNv, kNu>;
  D::A_t a0;
  D::B_t b0;
  D::x_t x0;
  D::u_t u0;
  (void)a0; (void)b0; (void)x0; (void)u0;
  D* df = new D(m, d0, fn);
  expect(df->m == m && df->d == d0, "Differentiator m / d");
  expect(df->x->data() == d0->qpos && df->u->data() == d0->ctrl, "Differentiator x / u bound to d");
  expect(df->stepCostFn == fn, "Differentiator stepCostFn is the caller's");
  expect(df->dqaccdq->data() == df->deriv && df->dqaccdqvel->data() == df->deriv + kNv * kNv &&
             df->dqaccdctrl->data() == df->deriv + 2 * kNv * kNv &&
             df->dgdx->data() == df->deriv + 2 * kNv * kNv + kNv * kNu &&
             df->dgdu->data() == df->dgdx->data() + 2 * kNv,
         "Differentiator maps into deriv (differentiator.h:57-61)");
  df->updateDerivatives();
  const mjtNum dt = m->opt.timestep;
  for (int i = 0; i < kNv; i++)
    for (int j = 0; j < kNv; j++) {
      expect((*df->A)(kNv + i, j) == (*df->dqaccdq)(i, j) * dt, "A lower-left = dt * col-major dqaccdq (Q1)");
      expect((*df->A)(i, j) == (i == j ? 1 : 0) && (*df->A)(i, kNv + j) == (i == j ? dt : 0), "A top = [I, dt I]");
    }
  for (int i = 0; i < kNv; i++) expect((*df->B)(kNv + i, 0) == (*df->dqaccdctrl)(i, 0) * dt, "B lower");
  mjData* d1 = mj_makeData(m);
  cpMjData(m, d1, d0);
  mj_step(m, d1);
  df->setMJData(d1);
  expect(df->d == d1 && df->x->data() == d1->qpos && df->u->data() == d1->ctrl, "setMJData re-seats x / u");
  ilqg_legacy::Map<1, 2 * kNv> q(df->deriv + 2 * kNv * kNv + kNv * kNu);
  (void)q;
  delete df;

  // ---- ILQR<nv,nu,N>: typedefs, members, methods ----
  using L = ILQR<kNv, kNu, kN>;
  L::A_t la; L::B_t lb; L::x_t lx; L::u_t lu; L::Q_t lq; L::R_t lr;
  L::K_t lK; L::k_t lk; L::V_t lV; L::v_t lv;
  (void)la; (void)lb; (void)lx; (void)lu; (void)lq; (void)lr; (void)lK; (void)lk; (void)lV; (void)lv;
  L::dqdq_mt* mp = nullptr; L::dqdu_mt* mu_ = nullptr; L::qpos_mt* mq = nullptr; L::qvel_mt* mv = nullptr;
  L::ctrl_mt* mc = nullptr; L::x_mt* mx = nullptr; L::u_mt* mu2 = nullptr; L::q_mt* mq2 = nullptr;
  L::r_mt* mr = nullptr;
  (void)mp; (void)mu_; (void)mq; (void)mv; (void)mc; (void)mx; (void)mu2; (void)mq2; (void)mr;
  L* il = new L(m, d0, fn);
  expect(il->m == m && il->mu == 1000.0, "ILQR m / mu");
  expect(il->x->data() == il->d->qpos && il->u->data() == il->d->ctrl, "ILQR x / u bound to d (ilqr.h:90-91)");
  expect(il->xStar->data() == il->d->qpos && il->uStar->data() == il->d->ctrl, "ILQR xStar / uStar after ctor");
  // after the ctor d is one step past dArray[0] (ilqr.h:82-87)
  mjData* t = mj_makeData(m);
  cpMjData(m, t, il->dArray[0]);
  mj_step(m, t);
  expect(!memcmp(t->qpos, il->d->qpos, sizeof(mjtNum) * m->nq) && !memcmp(t->qvel, il->d->qvel, sizeof(mjtNum) * m->nv),
         "ctor leaves d one step past the terminal point");
  il->setDInit(d0);
  il->forwardPass();
  expect(il->xStar->data() == il->dArray[0]->qpos && il->uStar->data() == il->dArray[0]->ctrl,
         "forwardPass leaves xStar / uStar on dArray[0] (ilqr.h:124-125)");
  il->setDInit(il->dArray[kN]);
  il->backwardPass();
  expect(il->differentiator->d == il->dArray[kN], "backwardPass leaves the differentiator at dArray[N]");
  // the differentiator's A / B are dArray[N]'s linearisation: recompute it
  L::A_t Aend = *il->differentiator->A;
  L::B_t Bend = *il->differentiator->B;
  il->differentiator->updateDerivatives();
  expect(!memcmp(Aend.data(), il->differentiator->A->data(), sizeof(Aend)) &&
             !memcmp(Bend.data(), il->differentiator->B->data(), sizeof(Bend)),
         "differentiator A / B after backwardPass = updateDerivatives at dArray[N]");
  il->initV();  // the base initV is callable
  il->iterate();
  for (int n = 1; n <= kN; n++) expect(il->K[n](0, 0) == il->K[n](0, 0), "K finite");
  expect((*il->V)(0, 0) == (*il->V)(0, 0) && (*il->v)(0, 0) == (*il->v)(0, 0), "V / v finite");
  delete il;
  mj_deleteData(t);
  mj_deleteData(d1);
  if (!fails) printf("members ok\n");
  return fails ? 1 : 0;
}

template <class IL>
void dump(const mjModel* m, IL& il) {
  for (int n = 0; n <= kN; n++) hex("K", il.K[n].data(), kNu * 2 * kNv);
  for (int n = 0; n <= kN; n++) hex("k", il.k[n].data(), kNu);
  hex("V", il.V->data(), 4 * kNv * kNv);
  hex("v", il.v->data(), 2 * kNv);
  for (int n = 0; n <= kN; n++) {
    hex("qpos", il.dArray[n]->qpos, m->nq);
    hex("qvel", il.dArray[n]->qvel, m->nv);
    hex("ctrl", il.dArray[n]->ctrl, m->nu);
  }
}

int initv(mjModel* m, mjData* d0, int iters) {
  stepCostFn_t fn = stepCost;
  FixedTerminal<kNv, kNu, kN> il(m, d0, fn);
  il.setDInit(d0);
  for (int i = 0; i < iters; i++) il.iterate();
  if (il.calls != iters) {
    fprintf(stderr, "FAIL: backwardPass called initV %d times for %d iterations\n", il.calls, iters);
    return 1;
  }
  dump(m, il);
  return 0;
}

int mutate(mjModel* m, mjData* d0) {
  stepCostFn_t fn = stepCost;
  MutatingTerminal<kNv, kNu, kN> il(m, d0, fn);
  il.setDInit(d0);
  il.iterate();
  dump(m, il);
  return 0;
}

int mu(mjModel* m, mjData* d0, mjtNum value, int iters) {
  stepCostFn_t fn = stepCost;
  ILQR<kNv, kNu, kN> il(m, d0, fn);
  il.mu = value;  // the public member, read by every backwardPass
  il.setDInit(d0);
  for (int i = 0; i < iters; i++) il.iterate();
  dump(m, il);
  return 0;
}
}  // namespace

int main(int argc, const char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: legacy_members model.xml members | initv [iters] | mu value [iters] | mutate\n");
    return 2;
  }
  mj_activate("mjkey.txt");
  char error[1000] = "";
  mjModel* m = mj_loadXML(argv[1], 0, error, 1000);
  if (!m) mju_error_s("Load model error: %s", error);
  if (m->nv != kNv || m->nu != kNu) mju_error("legacy_members drives the inverted pendulum (nv=2, nu=1)");
  mjData* d = mj_makeData(m);
  for (int i = 0; i < 10; i++) mj_step(m, d);  // inverted_pendulum.cpp:12-13
  int rc = !strcmp(argv[2], "members") ? members(m, d)
           : !strcmp(argv[2], "mu")    ? mu(m, d, argc > 3 ? atof(argv[3]) : 1000.0, argc > 4 ? atoi(argv[4]) : 1)
           : !strcmp(argv[2], "mutate") ? mutate(m, d)
                                       : initv(m, d, argc > 3 ? atoi(argv[3]) : 1);
  mj_deleteData(d);
  mj_deleteModel(m);
  return rc;
}
