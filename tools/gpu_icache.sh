#!/bin/bash
# Instruction-fetch counters (SQC I-cache) for the bench's kernels, plus the
# diagnostic stage stamps; each GPU step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ic
mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ \
  --output-format csv -d $OUT/p1 -o run -- $CMD > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d $OUT/p2 -o run -- $CMD > $OUT/p2.log 2>&1 &&
echo done
