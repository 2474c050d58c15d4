#!/bin/bash
# Quick GPU check after a kernel change: parity tests, a short bench, stage stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --no-cpu-baseline --steps ${STEPS:-10} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', round(d['value'],1), {k: round(v['avg_ms'],2) for k,v in d['kernels'].items()})"
if [[ -n "$STAMPS" ]]; then
  timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python3 tools/stamps.py > $OUT/stamps.log 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps.log; exit 1; }
  timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python3 tools/fused_diag.py 8 4 > $OUT/fused_diag.log 2>&1 || { echo "fused_diag failed"; tail -20 $OUT/fused_diag.log; exit 1; }
fi
