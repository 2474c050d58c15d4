cd $GRAFT_REPO_ROOT
: > gpurun_out/fdiag.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "fused_sweep or fd_batch" > gpurun_out/grp_test.log 2>&1 || { tail -30 gpurun_out/grp_test.log; exit 1; }
tail -1 gpurun_out/grp_test.log
for g in 0 1; do ILQG_FD_GIMG=$g timeout -k 10 60 python3 tools/fd_probe.py "gimg=$g" >> gpurun_out/fdiag.log 2>&1 || exit 1; done
cat gpurun_out/fdiag.log
