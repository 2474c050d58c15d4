#!/bin/bash
# Round-4 evidence in one GPU session: full GPU suite, smoke, the default bench
# (with the CPU baseline), rocprofv3 kernel-trace stats, FETCH/WRITE PMC
# passes (summary tagged with the kernel-source hash and GIT_HEAD), stage
# stamps and the fused-sweep timeline on the diagnostic build, the cfg-5 line.
# Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4}
mkdir -p $OUT
CMD="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
DIAG=ilqg-mujoco_amd/lib/libilqg_amd_diag.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
tail -1 $OUT/pytest_gpu.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
cat $OUT/bench.json &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $CMD > $OUT/trace.json 2> $OUT/trace.err &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $CMD > $OUT/fetch.json 2> $OUT/fetch.err &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $CMD > $OUT/write.json 2> $OUT/write.err &&
python3 tools/pmc_summary.py $OUT $OUT/pmc_traffic.json > /dev/null &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 -u tools/fused_timeline.py 8 > $OUT/timeline.log 2>&1 &&
timeout -k 10 400 python bench.py --workload humanoid_cfg5 --steps 5 --warmup 1 > $OUT/bench_cfg5.json 2> $OUT/bench_cfg5.err &&
cat $OUT/bench_cfg5.json &&
echo done
