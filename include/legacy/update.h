// Legacy simulation helpers (reference: inc/update.h:6-8, src/update.cpp).
#pragma once

#include "mujoco/mujoco.h"

void forwardStep(mjModel* model, mjData* data);   // one mj_step
void forwardFrame(mjModel* model, mjData* data);  // mj_step until 1/60 s of simulated time passed
