cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m9
DOFS_LIB=$PWD/exp/S/libdofs_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_krt_dnc.py tests/test_gpu_determinism.py -x -q --timeout 300 --timeout-method thread > gpurun_out/m9/pytest.log 2>&1 || { tail -25 gpurun_out/m9/pytest.log; exit 1; }
tail -1 gpurun_out/m9/pytest.log
DOFS_LIB=$PWD/denseopticalflowsegmentation3d_amd/_build/krt/libdofs_hip.so timeout -k 10 300 python tools/krt_timing.py 112 3 > gpurun_out/m9/krt_timing.log 2>&1 || exit 1
grep -A2 '"sweep' gpurun_out/m9/krt_timing.log | grep us_per | head -8
VARIANTS="E=E S=S L1=L1 L2=L2" N=2 bash tools/ab_env.sh
