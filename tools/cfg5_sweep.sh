# cfg 5 pipeline knobs (ILQG_PIPE_*), one bench line each: bash tools/cfg5_sweep.sh OUT
export TMPDIR=/tmp
O=gpurun_out/${1:-r5x}
mkdir -p $O
run() {  # name env...
  n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --workload humanoid_cfg5 --no-cpu-baseline --steps 4 > $O/$n.json 2> $O/$n.err || { echo "fail $n"; tail -5 $O/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$n.json')); print('$n', round(d['value'],2), {k: round(v['avg_ms'],2) for k,v in d['kernels'].items() if v['launches']})"
}
run c16 ILQG_PIPE_CHUNK=16
run c8 ILQG_PIPE_CHUNK=8
run c12 ILQG_PIPE_CHUNK=12
run c24 ILQG_PIPE_CHUNK=24
run c16k8 ILQG_PIPE_CHUNK=16 ILQG_PIPE_KEEP=8
run c16k16 ILQG_PIPE_CHUNK=16 ILQG_PIPE_KEEP=16
run c16xcd ILQG_PIPE_CHUNK=16 ILQG_PIPE_LOW=2
run c16spread ILQG_PIPE_CHUNK=16 ILQG_PIPE_LOW=0
run c16flat ILQG_PIPE_CHUNK=16 ILQG_PIPE_FLAT=1
run c16b ILQG_PIPE_CHUNK=16
