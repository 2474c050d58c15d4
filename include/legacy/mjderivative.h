// Legacy FD entry point (reference: inc/mjderivative.h:5,7), served by the GPU
// sweep of libilqg_amd (ilqg_fd_batch) plus host evaluation of the user's cost
// callback for the 1 + 2nv + nu cost samples.
#pragma once

#include "mujoco/mujoco.h"

typedef mjtNum (*stepCostFn_t)(const mjData*);

// deriv: caller-owned, nv*(2nv+nu) + 2nv + nu doubles, laid out as the
// reference writes it (src/mjderivative.cpp:88,107,120,138,174,202).
// Not re-entrant per (model) just like the reference; errors go to mju_error.
void calcMJDerivatives(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t stepCostFn);
