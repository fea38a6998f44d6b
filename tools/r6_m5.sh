# Round 6 check 5: workgroup shapes of stage B beside stage A — short replay workers of 8 (F, default), 4 (S4) and
# 2 (S2) waves, KLift / KSlotEvent at >= 4 waves per SIMD (W4). Replay parity on S2 first.
set -u
export TMPDIR=/tmp
DOFS_LIB=$PWD/exp/S2/libdofs_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_bench_config.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/m5_pytest.log 2>&1 || { tail -20 gpurun_out/m5_pytest.log; exit 1; }
tail -1 gpurun_out/m5_pytest.log
VARIANTS="F S4 S2 W4" N=2 bash tools/ab.sh || exit 1
