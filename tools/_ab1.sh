cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05c
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_knobs.py tests/test_gpu_bench_config.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05c/pytest.log 2>&1 || { tail -5 gpurun_out/r05c/pytest.log; exit 1; }
tail -2 gpurun_out/r05c/pytest.log
VARIANTS="L128=A L256=A,DOFS_FLOW_LONG=256 L512=A,DOFS_FLOW_LONG=512" N=2 bash tools/ab_env.sh
