#!/bin/bash
# SQ (instruction-mix / stall) counters for the bench's kernels, one rocprofv3
# --pmc pass per counter group, each under its own time limit, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
CMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --output-format csv -d $OUT/p1 -o run -- $CMD > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_SMEM \
  --output-format csv -d $OUT/p2 -o run -- $CMD > $OUT/p2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS \
  --output-format csv -d $OUT/p3 -o run -- $CMD > $OUT/p3.log 2>&1 &&
echo done
