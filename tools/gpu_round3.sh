#!/bin/bash
# Round-3 evidence in one GPU session: full GPU suite, smoke, the default bench
# (with the CPU baseline), rocprofv3 kernel-trace stats, FETCH/WRITE PMC passes
# and stage stamps.  Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r3
mkdir -p $OUT
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
tail -1 $OUT/pytest_gpu.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD > $OUT/trace.json 2> $OUT/trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.json 2> $OUT/fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.json 2> $OUT/write.err &&
python3 tools/pmc_summary.py $OUT $OUT/pmc_traffic.json &&
timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
echo done
