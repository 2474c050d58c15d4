#!/bin/bash
# cfg 5 evidence: the humanoid bench line (with its CPU baseline), a rocprofv3
# kernel-trace summary of the cfg-5 kernels, and the fp32-FD tolerance tests
# with their measured deviations printed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cfg5
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -s -k "fp32 or cfg5" --timeout 240 --timeout-method thread > $OUT/fp32_tests.log 2>&1 || { echo "fp32 tests failed"; tail -30 $OUT/fp32_tests.log; exit 1; }
grep -E "passed|failed|fp32 FD|relative|costs" $OUT/fp32_tests.log | tail -12
timeout -k 10 400 python bench.py --workload humanoid_cfg5 --steps 5 --warmup 1 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err || { echo "cfg5 bench failed"; tail -20 $OUT/bench_cfg5.err; exit 1; }
cat $OUT/bench_cfg5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --workload humanoid_cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/trace.log; exit 1; }
echo done
