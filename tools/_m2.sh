cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m2
for i in 1 2 3 4; do
for v in E B; do
  DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_flow_giveup.py tests/test_gpu_bench_config.py -q --timeout 240 --timeout-method thread > gpurun_out/m2/s_$v$i.log 2>&1
  echo "$v$i rc=$? $(tail -1 gpurun_out/m2/s_$v$i.log)"
done
done
