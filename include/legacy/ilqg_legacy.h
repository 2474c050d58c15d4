// Support types for the legacy C++ boundary (ilqr.h / differentiator.h):
// a small fixed-size column-major matrix (the reference's Eigen members'
// storage order) and the non-template solver core in libilqg_mujoco.so that
// drives the MI355X path (include/ilqg_amd.h).
#pragma once

#include <cstddef>

#include "mjderivative.h"
#include "mujoco/mujoco.h"

struct ilqg_cost;

namespace ilqg_legacy {

// Column-major R x C storage, like Eigen::Matrix<mjtNum, R, C> (the types of
// ILQR::K / k / V / v and Differentiator::A / B in the reference).
template <int R, int C>
struct Mat {
  mjtNum a[R * C] = {};
  mjtNum& operator()(int i, int j) { return a[i + j * R]; }
  const mjtNum& operator()(int i, int j) const { return a[i + j * R]; }
  // vectors (R == 1 or C == 1): coefficient i, as Eigen's v(i)
  mjtNum& operator()(int i) { return a[i]; }
  const mjtNum& operator()(int i) const { return a[i]; }
  mjtNum* data() { return a; }
  const mjtNum* data() const { return a; }
  static constexpr int rows() { return R; }
  static constexpr int cols() { return C; }
  static constexpr int size() { return R * C; }
};

// Column-major R x C view of caller memory, like Eigen::Map<Eigen::Matrix<
// mjtNum, R, C>> (the reference's *_mt typedefs, inc/ilqr.h:25-33,
// inc/differentiator.h:20-28).  Re-seated with placement new, as the
// reference does (`new (x) x_mt(d->qpos)`, inc/differentiator.h:80).
template <int R, int C>
struct Map {
  mjtNum* p;
  explicit Map(mjtNum* data) : p(data) {}
  mjtNum& operator()(int i, int j) const { return p[i + j * R]; }
  mjtNum& operator()(int i) const { return p[i]; }
  mjtNum* data() const { return p; }
  static constexpr int rows() { return R; }
  static constexpr int cols() { return C; }
  static constexpr int size() { return R * C; }
};

// Register a device cost descriptor for a host cost callback: ILQR / calcMJDerivatives
// then evaluate the cost on the GPU instead of calling `fn` on the host.  The
// descriptor must reproduce fn bit for bit (e.g. inc/inverted_pendulum/cost.h is
// wq = {1,10}, wv = {1,10}, wu = {1}); the arrays are copied.
void register_cost(stepCostFn_t fn, const ilqg_cost* desc, int nq, int nv, int nu);

// Cost-gradient entries of one FD record by host evaluation of fn, exactly as
// src/mjderivative.cpp:72,78-206 forms them (one-sided, perturbed state, eps 1e-6).
void host_cost_columns(const mjModel* m, const mjData* dmain, stepCostFn_t fn, mjtNum* deriv);

// The non-template part of ILQR<nv,nu,N>: one device solver (1 seed, 1
// candidate, reference semantics) plus host mirrors of its trajectory.
class SolverCore {
 public:
  SolverCore(mjModel* m, int N, stepCostFn_t fn);
  ~SolverCore();
  SolverCore(const SolverCore&) = delete;
  SolverCore& operator=(const SolverCore&) = delete;

  // ILQR ctor: d = dmain, passive rollout into dArray (inc/ilqr.h:69-97)
  void init(const mjData* dmain, mjData* const* dArray);
  void set_dinit(const mjData* dinit);                    // inc/ilqr.h:110-113
  void forward(mjData* const* dArray, const mjtNum* K, const mjtNum* k);  // inc/ilqr.h:116-130
  // the FD sweep of backwardPass: calcMJDerivatives at every point of dArray
  // (inc/ilqr.h:153-154 for n = 1..N, :102-103 for initV's n = 0), with the
  // host cost callback's gradient entries when no device cost is registered
  void sweep(mjData* const* dArray);
  // the Riccati recursion n = 1..N (inc/ilqr.h:144-175) with Levenberg-
  // Marquardt constant mu (read per pass, as ilqr.h:166 reads the member) from
  // the V0 / v0 that initV left in V / v (uploaded, ilqg_solver_set_value);
  // K, k, V, v out
  void riccati(mjtNum mu, mjtNum* K, mjtNum* k, mjtNum* V, mjtNum* v);
  // the FD record (calcMJDerivatives layout) of point n from the last sweep:
  // n = 0 and n = N always, every n when a host cost callback is in use
  const mjtNum* deriv(int n) const;
  // whether the last sweep's record of point n is the linearisation at d's
  // current state (dArray[n] unchanged since the sweep)
  bool deriv_current(int n, const mjData* d) const;
  // deriv_current at every point: dArray unchanged since the last sweep
  bool traj_current(mjData* const* dArray) const;

 private:
  void push_traj(mjData* const* dArray);
  void pull_traj(mjData* const* dArray);
  struct Impl;
  Impl* p_;
};

}  // namespace ilqg_legacy
