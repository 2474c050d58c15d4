export TMPDIR=/tmp
mkdir -p gpurun_out/r5f
run() {  # name env...
  n=$1; shift
  timeout -k 10 300 env "$@" python bench.py --workload humanoid_cfg5 --no-cpu-baseline --steps 4 > gpurun_out/r5f/$n.json 2> gpurun_out/r5f/$n.err || { echo "fail $n"; tail -5 gpurun_out/r5f/$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r5f/$n.json')); print('$n', round(d['value'],2), {k: round(v['avg_ms'],2) for k,v in d['kernels'].items() if v['launches']})"
}
run c12 ILQG_PIPE_CHUNK=12
run c16 ILQG_PIPE_CHUNK=16
run c24 ILQG_PIPE_CHUNK=24
run c16flat ILQG_PIPE_CHUNK=16 ILQG_PIPE_FLAT=1
run c16k8 ILQG_PIPE_CHUNK=16 ILQG_PIPE_KEEP=8
run c16x ILQG_PIPE_CHUNK=16 ILQG_PIPE_KEEP=32 ILQG_PIPE_LOW=1
run c16y ILQG_PIPE_CHUNK=16 ILQG_PIPE_KEEP=32
run c16r ILQG_PIPE_CHUNK=16
