// Host-only exercise of the C/C++ host code under AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_sanitize.py builds and runs it):
// the product's MJCF compiler, setConst and blob writer (csrc/model) on every
// bundled model, the blob read back by the oracle (mj_loadBlob), and the
// oracle's physics, FD driver and iLQR restatement on it.  No GPU involved.
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "model.h"
#include "ilqr_ora.h"

using namespace ilqg;

static int run(const std::string& path, int H) {
  HostModel hm;
  std::string err;
  if (!compile_mjcf_file(path, hm, err)) {
    std::fprintf(stderr, "%s: %s\n", path.c_str(), err.c_str());
    return 1;
  }
  set_const(hm);
  std::vector<unsigned char> blob = write_blob(hm);
  char e[256] = {0};
  mjModel* m = mj_loadBlob(blob.data(), blob.size(), e, sizeof(e));
  if (!m) {
    std::fprintf(stderr, "%s: mj_loadBlob: %s\n", path.c_str(), e);
    return 1;
  }
  mjData* d = mj_makeData(m);
  for (int i = 0; i < 30; i++) mj_step(m, d);
  mj_forward(m, d);
  const int nv = m->nv, nu = m->nu, D = nv * (2 * nv + nu) + 2 * nv + nu;
  std::vector<mjtNum> deriv(D);
  ora_set_nthread(2);
  ora_cost_desc c{};
  c.nq = m->nq; c.nv = nv; c.nu = nu;
  for (int i = 0; i < m->nq && i < 64; i++) c.wq[i] = 1.0;
  for (int i = 0; i < nv && i < 64; i++) c.wv[i] = 0.1;
  for (int i = 0; i < nu && i < 64; i++) c.wu[i] = 0.01;
  ora_set_cost_desc(&c);
  ora_calcMJDerivatives(m, d, deriv.data(), ora_cost_desc_fn);
  ora_ilqr* il = ora_ilqr_create(m, d, H, ora_cost_desc_fn, ora_calcMJDerivatives);
  ora_ilqr_setDInit(il, d);
  ora_ilqr_iterate(il);
  const mjtNum alphas[3] = {1.0, 0.5, 0.25};
  mjtNum costs[3];
  int sel = 0;
  ora_ilqr_iterate_ls(il, 3, alphas, 1, costs, &sel);
  double s = 0;
  for (int i = 0; i < D; i++) s += std::fabs(deriv[i]);
  std::printf("%s: nq=%d nv=%d nu=%d |deriv|=%.6g cost=%.6g\n", path.c_str(), m->nq, nv, nu, s, costs[sel]);
  ora_ilqr_free(il);
  mj_deleteData(d);
  mj_deleteModel(m);
  return 0;
}

int main(int argc, char** argv) {
  int rc = 0;
  for (int i = 1; i < argc; i++) rc |= run(argv[i], 12);
  // a malformed document must fail cleanly, not read out of bounds
  HostModel hm;
  std::string err;
  if (compile_mjcf_string("<mujoco><worldbody><body pos=\"0 0", hm, err)) rc |= 1;
  if (compile_mjcf_string("", hm, err)) rc |= 1;
  return rc;
}
