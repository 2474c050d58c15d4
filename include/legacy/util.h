// Legacy state copy (reference: inc/util.h:6, src/util.cpp:4-14).
#pragma once

#include "mujoco/mujoco.h"

// copies time, qpos, qvel, qacc, qacc_warmstart, qfrc_applied, xfrc_applied, ctrl
void cpMjData(const mjModel* m, mjData* d_dest, const mjData* d_src);
