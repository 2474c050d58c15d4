#!/bin/bash
# Fused-sweep ticket planner A/B: GPU tests, bench lines with the planner off /
# on at a few thresholds, then the diagnostic build's stamps and timelines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-plan}
mkdir -p $OUT
DIAG=ilqg-mujoco_amd/lib/libilqg_amd_diag.so
B="python bench.py --no-cpu-baseline --steps 20"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
tail -2 $OUT/pytest_gpu.log &&
timeout -k 10 300 env ILQG_PLAN=0 $B > $OUT/bench_plan0.json 2> $OUT/bench_plan0.err &&
timeout -k 10 300 env ILQG_PLAN=1 $B > $OUT/bench_plan1.json 2> $OUT/bench_plan1.err &&
timeout -k 10 300 env ILQG_PLAN_K=2 $B > $OUT/bench_k2.json 2> $OUT/bench_k2.err &&
timeout -k 10 300 env ILQG_PLAN_K=5 $B > $OUT/bench_k5.json 2> $OUT/bench_k5.err &&
timeout -k 10 300 env ILQG_PLAN_P0=2 $B > $OUT/bench_p02.json 2> $OUT/bench_p02.err &&
for f in plan0 plan1 k2 k5 p02; do python3 -c "import json,sys; d=json.load(open('$OUT/bench_$f.json')); k=d['kernels']; print('$f', round(d['value'],1), 'rollout', round(k['rollout']['avg_ms'],3), 'fd_backward', round(k['fd_backward']['avg_ms'],3))"; done &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG ILQG_PLAN=0 python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan0.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan1.log 2>&1 &&
head -20 $OUT/timeline_plan1.log &&
echo done
