cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05g
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_intraframe.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05g/pytest.log 2>&1 || { tail -15 gpurun_out/r05g/pytest.log; exit 1; }
tail -2 gpurun_out/r05g/pytest.log
DOFS_SERIAL=1 H=2160 W=3840 timeout -k 10 300 python tools/flow_stats.py 1 3 > gpurun_out/r05g/flow4k.log 2>&1 || exit 1
DOFS_SERIAL=1 DOFS_LIB=$PWD/denseopticalflowsegmentation3d_amd/_build/prof/libdofs_hip.so H=2160 W=3840 timeout -k 10 300 python tools/flow_stats.py 1 3 > gpurun_out/r05g/flow4k_prof.log 2>&1 || exit 1
tail -2 gpurun_out/r05g/flow4k.log | cut -c1-300
tail -2 gpurun_out/r05g/flow4k_prof.log | cut -c1-400
timeout -k 10 300 python tools/bench_intraframe.py --model 4 > gpurun_out/r05g/intra.json 2>&1 || exit 1
tail -1 gpurun_out/r05g/intra.json | cut -c1-500
