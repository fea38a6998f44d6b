# KLeafPos writes the replay inputs (StepIn): parity on the variant library, then a same-box A/B against HEAD's
set -u
v=${V:-LP}
DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_preorder_modes.py tests/test_gpu_krt_dnc.py > gpurun_out/par_$v.log 2>&1 || { echo "parity $v failed"; tail -30 gpurun_out/par_$v.log; exit 1; }
tail -1 gpurun_out/par_$v.log
VARIANTS="${VS:-F $v}" N=${N:-3} bash tools/ab.sh
