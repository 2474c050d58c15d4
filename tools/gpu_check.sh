#!/bin/bash
# Quick GPU check: the full -m gpu suite, smoke(), one default bench line.
# Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
tail -3 $OUT/pytest_gpu.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
tail -1 $OUT/smoke.log &&
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
echo done
