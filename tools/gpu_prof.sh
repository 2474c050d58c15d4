#!/bin/bash
# rocprofv3 evidence for the bench command: kernel-trace stats, then one PMC
# pass per TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
# Each profiled run has its own time limit; the steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD \
  > $OUT/trace.json 2> $OUT/trace.err &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD \
  > $OUT/fetch.json 2> $OUT/fetch.err &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD \
  > $OUT/write.json 2> $OUT/write.err &&
find $OUT -name "*.csv" | sort
