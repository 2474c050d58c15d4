#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STAMPS=1 bash tools/gpu_quick.sh || exit 1
timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag0.so python3 tools/stamps.py > $OUT/stamps0.log 2>&1 || exit 1
timeout -k 10 300 env ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag0.so python3 tools/fused_diag.py 8 4 > $OUT/fused_diag0.log 2>&1 || exit 1
