set -u
for v in R2 R2W6; do
  DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py > gpurun_out/par_$v.log 2>&1 || { echo "parity $v failed"; tail -20 gpurun_out/par_$v.log; exit 1; }
  tail -1 gpurun_out/par_$v.log
done
VARIANTS="F R2 R2W6" N=3 bash tools/ab.sh
