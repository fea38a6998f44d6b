cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05k
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_bench_config.py tests/test_gpu_replay_modes.py tests/test_gpu_knobs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05k/pytest.log 2>&1 || { tail -25 gpurun_out/r05k/pytest.log; exit 1; }
tail -2 gpurun_out/r05k/pytest.log
DOFS_SERIAL=1 DOFS_LIB=$PWD/denseopticalflowsegmentation3d_amd/_build/prof/libdofs_hip.so timeout -k 10 300 python tools/flow_stats.py 112 2 > gpurun_out/r05k/flow1080_prof.log 2>&1 || exit 1
tail -2 gpurun_out/r05k/flow1080_prof.log | cut -c1-400
VARIANTS="A=A B=B C=C" N=3 bash tools/ab_env.sh
