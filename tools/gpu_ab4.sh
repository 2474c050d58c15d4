#!/bin/bash
# Rollout-sensitive GPU tests against one library, then bench lines per
# library / environment, then the diagnostic build's stamps (hopper and
# humanoid).
#   tools/gpu_ab4.sh OUTDIR TESTLIB "NAME:ENV=.. ENV2=.." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
TESTLIB=$2
shift 2
mkdir -p $OUT
LIB=ilqg-mujoco_amd/lib
if [ "$TESTLIB" != "-" ]; then
  timeout -k 10 900 env ILQG_LIB=$TESTLIB python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 300 env $envs python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -5 $OUT/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); k=d['kernels']; print('$name', round(d['value'],1), 'rollout', round(k['rollout']['avg_ms'],3), 'fd_backward', round(k['fd_backward']['avg_ms'],3))"
done
if [ "$TESTLIB" != "-" ]; then
  timeout -k 10 300 env ILQG_LIB=$TESTLIB python bench.py --workload humanoid_cfg5 --no-cpu-baseline --steps 3 > $OUT/cfg5.json 2> $OUT/cfg5.err || { echo "cfg5 failed"; tail -5 $OUT/cfg5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/cfg5.json')); k=d['kernels']; print('cfg5', round(d['value'],2), {n: round(v['avg_ms'],2) for n, v in k.items() if v['launches']})"
fi
DIAG=$LIB/libilqg_amd_diag.so
if [ -f $DIAG ]; then
timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py humanoid > $OUT/stamps_humanoid.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG ILQG_PLAN=0 python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan0.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan1.log 2>&1
fi
echo done
