cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_knobs.py tests/test_gpu_bench_config.py tests/test_gpu_parity.py tests/test_gpu_lean.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05d/pytest.log 2>&1 || { tail -15 gpurun_out/r05d/pytest.log; exit 1; }
tail -2 gpurun_out/r05d/pytest.log
for v in A B; do DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 300 python tools/bench_intraframe.py --model 4 > gpurun_out/r05d/intra_$v.json 2>&1 || exit 1; tail -1 gpurun_out/r05d/intra_$v.json | cut -c1-400; done
VARIANTS="A=A B=B B512=B,DOFS_FLOW_LONG=512 B128=B,DOFS_FLOW_LONG=128" N=2 bash tools/ab_env.sh
