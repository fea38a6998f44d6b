cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05i
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow_giveup.py tests/test_gpu_flow_order.py tests/test_gpu_lean.py tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05i/pytest.log 2>&1 || { tail -25 gpurun_out/r05i/pytest.log; exit 1; }
tail -2 gpurun_out/r05i/pytest.log
bash tools/prof_pair.sh
