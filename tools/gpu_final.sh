#!/bin/bash
# Round-end evidence in one GPU session: gpu tests + smoke + bench (with CPU
# baseline) + rocprofv3 kernel stats (gpu_round.sh), the FETCH/WRITE PMC passes
# (gpu_prof.sh) and the diagnostic stage stamps.  Steps chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_round.sh all &&
bash tools/gpu_prof.sh &&
python3 tools/pmc_summary.py gpurun_out/prof gpurun_out/pmc_traffic.json &&
ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps.log 2>&1 &&
ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so timeout -k 10 120 python3 -u tools/fused_diag.py 8 1 > gpurun_out/fdiag.log 2>&1 &&
echo done
