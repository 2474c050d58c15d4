set -o pipefail
cd $GRAFT_REPO_ROOT
for lag in 8 32 64 128 500; do ILQG_FD_LAG=$lag timeout -k 10 60 python3 tools/fd_probe.py "lag=$lag" >> gpurun_out/fdp.log 2>&1 || exit 1; done
ILQG_FD_CV=6 ILQG_FD_LAG=64 timeout -k 10 60 python3 tools/fd_probe.py "cv=6 lag=64" >> gpurun_out/fdp.log 2>&1 || exit 1
ILQG_FUSED=0 timeout -k 10 60 python3 tools/fd_probe.py "unfused" >> gpurun_out/fdp.log 2>&1 || exit 1
