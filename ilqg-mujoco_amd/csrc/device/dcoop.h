// Cooperative device physics: ONE WAVEFRONT PER EVALUATION, workspace in LDS.
//
// The same MuJoCo-2.0 pipeline as dphys.h (and oracle/mjsub.c), re-mapped for
// latency: the 64 lanes of a workgroup split every stage over its independent
// outputs -- bodies, joints, dofs, geom pairs, constraint rows, matrix entries
// -- while each scalar is still produced by exactly one lane with the oracle's
// expression and summation order, so results stay bit-identical.  Inherently
// serial recursions (kinematic chain, com velocities, triangular solves,
// ordered reductions) run on lane 0 out of LDS.  All control flow that
// reaches a barrier is uniform across the workgroup (broadcast through LDS).
#pragma once

#include "dphys.h"
#include "dsmall.h"

namespace ilqg {
namespace coop {

using real = double;
#include "dcoop_impl.h"

}  // namespace coop
}  // namespace ilqg

