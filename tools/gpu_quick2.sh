cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 -u tools/group_probe.py 1 > gpurun_out/gp.log 2>&1 || { cat gpurun_out/gp.log; exit 1; }
cat gpurun_out/gp.log
ILQG_LIB=ilqg-mujoco_amd/lib/libilqg_amd_diag.so timeout -k 10 120 python3 tools/stamps.py > gpurun_out/stamps.log 2>&1 || { cat gpurun_out/stamps.log; exit 1; }
head -45 gpurun_out/stamps.log
