cd $GRAFT_REPO_ROOT
: > gpurun_out/fdiag.log
for lag in 501 250 100 32; do ILQG_FD_LAG=$lag timeout -k 10 60 python3 tools/fd_probe.py "lag=$lag" >> gpurun_out/fdiag.log 2>&1 || exit 1; done
ILQG_FD_CV=2 ILQG_FD_LAG=100 timeout -k 10 60 python3 tools/fd_probe.py "cv=2 lag=100" >> gpurun_out/fdiag.log 2>&1 || exit 1
cat gpurun_out/fdiag.log
