#!/bin/bash
# One parameterised GPU-box session (replaces the per-round gpu_*.sh scripts).
#
#   tools/gpu.sh OUTDIR STEP [STEP ...]
#
# Steps run in order, each GPU step under its own time limit; the first
# failure ends the session (nothing more touches the GPU after it).
#   tests[=LIB]          full -m gpu suite (optionally against ILQG_LIB=LIB)
#   testk=EXPR           -m gpu tests selected by -k EXPR
#   smoke                __graft_entry__.smoke()
#   bench                default bench line (with the CPU baseline)
#   ab=NAME[,ENV=V...]   REPS (default 3) bench lines, 20 steps, no CPU leg;
#                        ENV=V pairs may include ILQG_LIB=...
#   cfg5[=NAME,ENV=V...] REPS cfg-5 humanoid bench lines (ENV may include ILQG_LIB=...)
#   cfg5cpu              one cfg-5 bench line with its CPU baseline (cfg5_bench.json)
#   cfg5trace            rocprofv3 kernel trace of a short cfg-5 bench (the pipeline's timeline)
#   resources            tools/resource_report.py of the library (no GPU)
#   prof                 rocprofv3 kernel-trace stats + FETCH/WRITE PMC passes
#   stamps[=MODEL[:mfma]] stage stamps on the diagnostic build
#   timeline             fused-sweep timeline on the diagnostic build
#   sq                   SQ instruction-mix / stall counters (3 passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
shift
mkdir -p "$OUT"
REPS=${REPS:-3}
DIAG=ilqg-mujoco_amd/lib/libilqg_amd_diag.so
PCMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }
summ() {  # one-line summary of a bench JSON
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels',{}); print(sys.argv[2], round(d['value'],2), {n: round(v['avg_ms'],3) for n, v in k.items() if v.get('launches')})" "$1" "$2"
}
for step in "$@"; do
  key=${step%%=*}; arg=""
  [[ $step == *=* ]] && arg=${step#*=}
  case $key in
  tests)
    envs=""; [ -n "$arg" ] && envs="ILQG_LIB=$arg"
    timeout -k 10 1000 env $envs python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > $OUT/tests.log 2>&1 || fail tests $OUT/tests.log
    tail -1 $OUT/tests.log ;;
  testk)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -k "$arg" --timeout 300 --timeout-method thread \
      > $OUT/testk.log 2>&1 || fail testk $OUT/testk.log
    tail -1 $OUT/testk.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || fail smoke $OUT/smoke.log
    tail -1 $OUT/smoke.log ;;
  bench)
    timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || fail bench $OUT/bench.err
    cat $OUT/bench.json ;;
  ab)
    name=${arg%%,*}; envs=""; [[ $arg == *,* ]] && envs=${arg#*,}; envs=${envs//,/ }
    for r in $(seq 1 $REPS); do
      f=$OUT/ab_${name}_$r.json
      timeout -k 10 300 env $envs python bench.py --no-cpu-baseline --steps 20 > $f 2> $f.err || fail "ab $name" $f.err
      summ $f "$name#$r"
    done ;;
  cfg5)
    name=${arg%%,*}; name=${name:-default}; envs=""; [[ $arg == *,* ]] && envs=${arg#*,}; envs=${envs//,/ }
    for r in $(seq 1 $REPS); do
      f=$OUT/cfg5_${name}_$r.json
      timeout -k 10 400 env $envs python bench.py --workload humanoid_cfg5 --no-cpu-baseline --steps 5 > $f 2> $f.err || fail cfg5 $f.err
      summ $f "cfg5 $name#$r"
    done ;;
  cfg5cpu)
    timeout -k 10 600 python bench.py --workload humanoid_cfg5 --steps 5 > $OUT/cfg5_bench.json 2> $OUT/cfg5_bench.err \
      || fail cfg5cpu $OUT/cfg5_bench.err
    summ $OUT/cfg5_bench.json "cfg5 (with cpu_baseline)" ;;
  cfg5trace)
    timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/cfg5trace -o run -- \
      python3 bench.py --workload humanoid_cfg5 --steps 2 --warmup 1 --no-cpu-baseline \
      > $OUT/cfg5trace.json 2> $OUT/cfg5trace.err || fail cfg5trace $OUT/cfg5trace.err
    echo "cfg5trace ok" ;;
  resources)
    python3 tools/resource_report.py > $OUT/resource_usage.txt || fail resources
    echo "resources ok" ;;
  prof)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $PCMD \
      > $OUT/trace.json 2> $OUT/trace.err || fail trace $OUT/trace.err
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $PCMD \
      > $OUT/fetch.json 2> $OUT/fetch.err || fail fetch $OUT/fetch.err
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $PCMD \
      > $OUT/write.json 2> $OUT/write.err || fail write $OUT/write.err
    python3 tools/pmc_summary.py $OUT $OUT/pmc_traffic.json || fail pmc_summary ;;
  stamps)
    m=${arg:-hopper}  # MODEL or MODEL:mfma (the backward section on the MFMA engine)
    timeout -k 10 300 env ILQG_LIB=$DIAG python3 tools/stamps.py ${m//:/ } > $OUT/stamps_${m//:/_}.log 2>&1 || fail stamps $OUT/stamps_${m//:/_}.log
    echo "stamps $m ok" ;;
  timeline)
    timeout -k 10 300 env ILQG_LIB=$DIAG python3 -u tools/fused_timeline.py 8 > $OUT/timeline.log 2>&1 || fail timeline $OUT/timeline.log
    echo "timeline ok" ;;
  sq)
    SCMD="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
    timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
      --output-format csv -d $OUT/sq1 -o run -- $SCMD > $OUT/sq1.log 2>&1 || fail sq1 $OUT/sq1.log
    timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS \
      --output-format csv -d $OUT/sq2 -o run -- $SCMD > $OUT/sq2.log 2>&1 || fail sq2 $OUT/sq2.log
    echo "sq ok" ;;
  *) fail "unknown step $step" ;;
  esac
done
echo done
