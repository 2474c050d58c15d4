#!/bin/bash
# GPU tests, a short bench and one WRITE_SIZE PMC pass of the bench command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT/write
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py --no-cpu-baseline --steps ${STEPS:-10} > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print('value', round(d['value'],1), {k: round(v['avg_ms'],2) for k,v in d['kernels'].items()})"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/write/w.json 2> $OUT/write/w.err || { echo "pmc failed"; tail -20 $OUT/write/w.err; exit 1; }
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/write/run_counter_collection.csv")):
    k = r["Kernel_Name"]
    if "fd_fused" in k or "rollout2" in k:
        acc[k[:60]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, "launches", len(v), "avg WRITE_SIZE KB", round(sum(v) / len(v), 1))
PY
