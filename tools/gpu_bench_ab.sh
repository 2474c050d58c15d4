#!/bin/bash
# Bench lines per library / environment (no tests), the selection probe, then
# the diagnostic build's stamps and fused-sweep timelines.
#   tools/gpu_bench_ab.sh OUTDIR "NAME:ENV=.. ENV2=.." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p $OUT
LIB=ilqg-mujoco_amd/lib
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 300 env $envs python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -5 $OUT/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); k=d['kernels']; print('$name', round(d['value'],1), 'rollout', round(k['rollout']['avg_ms'],3), 'fd_backward', round(k['fd_backward']['avg_ms'],3))"
done
timeout -k 10 120 python tools/select_probe.py 12 > $OUT/select_probe.log 2>&1
DIAG=$LIB/libilqg_amd_diag.so
if [ -f $DIAG ]; then
timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG ILQG_PLAN=0 python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan0.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan1.log 2>&1
fi
echo done
