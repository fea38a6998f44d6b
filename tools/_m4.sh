cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m4
DOFS_LIB=$PWD/exp/P/libdofs_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_bench_config.py tests/test_gpu_lean.py tests/test_gpu_replay_modes.py tests/test_gpu_knobs.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread > gpurun_out/m4/pytest_P.log 2>&1
echo "pytest rc=$?"; grep -c PASSED gpurun_out/m4/pytest_P.log; grep FAILED gpurun_out/m4/pytest_P.log | head -20
