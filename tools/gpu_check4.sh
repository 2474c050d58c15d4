#!/bin/bash
# Full GPU suite, the hopper bench line, the cfg-5 bench line and the
# humanoid stage stamps (diagnostic build).   tools/gpu_check4.sh OUTDIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); k=d['kernels']; print('hopper', round(d['value'],1), {n: round(v['avg_ms'],3) for n, v in k.items() if v['launches']})"
timeout -k 10 300 python bench.py --workload humanoid_cfg5 --no-cpu-baseline --steps 3 > $OUT/cfg5.json 2> $OUT/cfg5.err || { echo "cfg5 failed"; tail -5 $OUT/cfg5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/cfg5.json')); k=d['kernels']; print('cfg5', round(d['value'],2), {n: round(v['avg_ms'],2) for n, v in k.items() if v['launches']})"
timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so python3 tools/stamps.py humanoid > $OUT/stamps_humanoid.log 2>&1
echo done
