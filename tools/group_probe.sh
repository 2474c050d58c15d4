set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/grp.log
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "seed_groups or fused_sweep" > gpurun_out/grp_test.log 2>&1 || { tail -30 gpurun_out/grp_test.log; exit 1; }
tail -2 gpurun_out/grp_test.log
run() { # label env... -- groups
  local label=$1; shift
  env PROBE_LABEL="$label" "$@" timeout -k 10 120 python3 -u tools/group_probe.py $GS >> gpurun_out/grp.log 2>&1 || { cat gpurun_out/grp.log; exit 1; }
}
GS="1" run "prio"
timeout -k 10 60 python3 tools/fd_probe.py "prio" >> gpurun_out/grp.log 2>&1 || exit 1
GS="2 4" run "roll64 hwq8" GPU_MAX_HW_QUEUES=8 ILQG_ROLL_CUS=64
GS="2 4" run "roll64 notoken hwq12" GPU_MAX_HW_QUEUES=12 ILQG_ROLL_CUS=64 ILQG_GROUP_TOKEN=0
cat gpurun_out/grp.log
