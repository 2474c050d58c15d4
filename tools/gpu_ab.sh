#!/bin/bash
# GPU tests + bench A/B over environment settings.
#   tools/gpu_ab.sh OUTDIR "NAME1:ENV1=a ENV2=b" "NAME2:..." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  timeout -k 10 300 env $envs python bench.py --no-cpu-baseline --steps 20 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -5 $OUT/bench_$name.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$name.json')); k=d['kernels']; print('$name', round(d['value'],1), 'rollout', round(k['rollout']['avg_ms'],3), 'fd_backward', round(k['fd_backward']['avg_ms'],3))"
done
echo done
