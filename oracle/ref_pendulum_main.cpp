// ORACLE / TEST INFRASTRUCTURE ONLY.
// Drives the reference's own controller class (InvertedPendulum,
// src/inverted_pendulum/inverted_pendulum.cpp, compiled unmodified from
// /root/reference against the product's legacy headers include/legacy/) through
// the cmd/basic.cpp main loop without rendering, and prints every frame as hex
// floats.  Linked against the product's libilqg_mujoco.so: this is the
// drop-in check "the reference's caller code runs on the MI355X path".
#include <cstdio>
#include <cstdlib>

#include "inverted_pendulum/inverted_pendulum.h"
#include "mujoco/mujoco.h"

static void print_frame(int f, const mjModel* m, const mjData* d) {
  printf("frame %d %a", f, d->time);
  for (int i = 0; i < m->nq; i++) printf(" %a", d->qpos[i]);
  for (int i = 0; i < m->nv; i++) printf(" %a", d->qvel[i]);
  for (int i = 0; i < m->nu; i++) printf(" %a", d->ctrl[i]);
  printf("\n");
}

int main(int argc, const char** argv) {
  if (argc < 2) return 2;
  const int frames = argc > 2 ? atoi(argv[2]) : 3;
  char error[1000] = "Could not load binary model";
  mjModel* m = mj_loadXML(argv[1], 0, error, 1000);
  if (!m) mju_error_s("Load model error: %s", error);
  mjData* d = mj_makeData(m);
  InvertedPendulum ip(m, d);
  print_frame(0, m, d);
  for (int f = 1; f <= frames; f++) {
    ip.forward();
    print_frame(f, m, d);
  }
  return 0;
}
