// fp32 instance of the cooperative device physics (dcoop_impl.h with
// real = float) for the fp32 FD sweep of BASELINE.json configs[4] (humanoid,
// "fp32 FD with fp64 Riccati"): half the LDS per evaluation team.  Nothing
// on the bit-exact fp64 path includes it.
#pragma once

#include "dphys.h"
#include "dsmall.h"

namespace ilqg {
namespace coopf {

using namespace coop;  // dsmall.h: team_sync, register rows, broadcasts
using real = float;
#include "dcoop_impl.h"

}  // namespace coopf
}  // namespace ilqg
