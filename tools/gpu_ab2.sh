#!/bin/bash
# Round-4 A/B: full GPU suite on the product library, the rollout-sensitive
# parity tests on the uniform-stage variant, then bench lines per library /
# environment, the selection probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
LIB=ilqg-mujoco_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 env ILQG_LIB=$LIB/libilqg_amd_rollu.so python -u -m pytest tests/test_gpu_parity.py tests/test_layout.py -m gpu -x -q --timeout 300 --timeout-method thread -k "iterate or bench_workload or step_batch or linesearch or cfg4 or edge or corrected or set_value or multiseed" > $OUT/pytest_rollu.log 2>&1 || { tail -5 $OUT/pytest_rollu.log; exit 1; }
tail -1 $OUT/pytest_rollu.log
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 300 env $envs python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -5 $OUT/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); k=d['kernels']; print('$name', round(d['value'],1), 'rollout', round(k['rollout']['avg_ms'],3), 'fd_backward', round(k['fd_backward']['avg_ms'],3))"
done
timeout -k 10 120 python tools/select_probe.py 12 > $OUT/select_probe.log 2>&1
DIAG=$LIB/libilqg_amd_diag.so
timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py > $OUT/stamps.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG ILQG_PLAN=0 python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan0.log 2>&1 &&
timeout -k 10 300 env ILQG_LIB=$DIAG python3 -u tools/fused_timeline.py 8 > $OUT/timeline_plan1.log 2>&1
echo done
