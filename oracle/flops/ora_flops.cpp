// ORACLE / TEST INFRASTRUCTURE ONLY: the counters of the instrumented build (counted.h).
#include "counted.h"

extern "C" {
ora_flop_counts ora_flops = {0, 0, 0, 0, 0, 0};
void ora_flops_get(unsigned long long* out) {
  out[0] = ora_flops.add; out[1] = ora_flops.mul; out[2] = ora_flops.div;
  out[3] = ora_flops.sqrt; out[4] = ora_flops.cmp; out[5] = ora_flops.trans;
}
void ora_flops_reset(void) { ora_flops = ora_flop_counts{0, 0, 0, 0, 0, 0}; }
}
