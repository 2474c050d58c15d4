// ORACLE / TEST INFRASTRUCTURE ONLY.
// C-linkage shim over the reference's own FD driver, compiled unmodified from
// /root/reference/src/{mjderivative,util,update}.cpp by oracle/Makefile into
// oracle/_ref/libilqg_ref.so (never copied into this repo).  It lets tests
// call the reference's calcMJDerivatives (mjderivative.h:7), cpMjData
// (util.h:6) and forwardStep/forwardFrame (update.h:6-8) through ctypes.
#include "mujoco/mujoco.h"
#include "mjderivative.h"
#include "util.h"
#include "update.h"

extern "C" {
void ref_calcMJDerivatives(mjModel* m, mjData* dmain, mjtNum* deriv, stepCostFn_t fn) {
  calcMJDerivatives(m, dmain, deriv, fn);
}
void ref_cpMjData(const mjModel* m, mjData* dst, const mjData* src) { cpMjData(m, dst, src); }
void ref_forwardStep(mjModel* m, mjData* d) { forwardStep(m, d); }
void ref_forwardFrame(mjModel* m, mjData* d) { forwardFrame(m, d); }
}
