// ilqg_headless: the cmd/basic.cpp main loop without rendering (SURVEY.md
// §8f row 4), driving an inverted-pendulum MPC controller through the legacy
// C++ boundary (include/legacy: mujoco.h, ilqr.h) on the MI355X path.
//
//   ilqg_headless model.xml [frames=60] [--device-cost]
//
// Per frame, like the reference's controller (src/inverted_pendulum/
// inverted_pendulum.cpp:19-30): setDInit(d); 10 x iterate(); apply the first
// control of the optimised trajectory; mj_step.  The initial state is the
// model's reset state after 10 passive steps (inverted_pendulum.cpp:12-13).
// Each frame prints time, qpos, qvel, ctrl as C99 hex floats so runs can be
// compared bit for bit.  --device-cost registers the cost's diagonal-quadratic
// descriptor so the cost samples run on the GPU instead of the host callback.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ilqg_amd.h"
#include "ilqr.h"
#include "mjderivative.h"
#include "mujoco/mujoco.h"

namespace {

constexpr int kNv = 2, kNu = 1, kN = 20, kIters = 10;

// quadratic pendulum cost: weights 1, 10 on (cart, pole) position and velocity, 1 on ctrl
mjtNum pendulum_cost(const mjData* d) {
  mjtNum c = 1.0 * d->qpos[0] * d->qpos[0] + 10.0 * d->qpos[1] * d->qpos[1] + 1.0 * d->qvel[0] * d->qvel[0] +
             10.0 * d->qvel[1] * d->qvel[1] + 1.0 * d->ctrl[0] * d->ctrl[0];
  return c;
}

void print_frame(int f, const mjModel* m, const mjData* d) {
  printf("frame %d %a", f, d->time);
  for (int i = 0; i < m->nq; i++) printf(" %a", d->qpos[i]);
  for (int i = 0; i < m->nv; i++) printf(" %a", d->qvel[i]);
  for (int i = 0; i < m->nu; i++) printf(" %a", d->ctrl[i]);
  printf("\n");
}

}  // namespace

int main(int argc, const char** argv) {
  if (argc < 2) {
    printf(" USAGE:  ilqg_headless modelfile.xml [frames] [--device-cost]\n");
    return 0;
  }
  int frames = 60;
  bool device_cost = false;
  for (int i = 2; i < argc; i++) {
    if (!strcmp(argv[i], "--device-cost")) device_cost = true;
    else frames = atoi(argv[i]);
  }
  mj_activate("mjkey.txt");
  char error[1000] = "Could not load binary model";
  mjModel* m = mj_loadXML(argv[1], 0, error, 1000);
  if (!m) mju_error_s("Load model error: %s", error);
  if (m->nv != kNv || m->nu != kNu) mju_error("ilqg_headless drives the inverted pendulum (nv=2, nu=1)");
  mjData* d = mj_makeData(m);

  stepCostFn_t cost = pendulum_cost;
  if (device_cost) {
    const double wq[2] = {1.0, 10.0}, wv[2] = {1.0, 10.0}, wu[1] = {1.0};
    ilqg_cost desc{};
    desc.wq = wq;
    desc.wv = wv;
    desc.wu = wu;
    ilqg_legacy::register_cost(cost, &desc, m->nq, m->nv, m->nu);
  }
  for (int i = 0; i < 10; i++) mj_step(m, d);
  ILQR<kNv, kNu, kN>* ilqr = new ILQR<kNv, kNu, kN>(m, d, cost);

  print_frame(0, m, d);
  for (int f = 1; f <= frames; f++) {
    ilqr->setDInit(d);
    for (int i = 0; i < kIters; i++) ilqr->iterate();
    mju_copy(d->ctrl, ilqr->dArray[kN]->ctrl, kNu);
    mj_step(m, d);
    print_frame(f, m, d);
  }
  delete ilqr;
  mj_deleteData(d);
  mj_deleteModel(m);
  mj_deactivate();
  return 0;
}
