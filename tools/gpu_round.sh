#!/bin/bash
# One GPU-box session: gpu tests, smoke, bench, rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STAGE=${1:-all}
if [[ $STAGE == all || $STAGE == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [[ $STAGE == all || $STAGE == prof ]]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
  find $OUT/prof -name "*kernel_stats*" | head
fi
