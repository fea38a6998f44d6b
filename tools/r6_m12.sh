# Tiled round 0 (FT) and the same with physically contiguous workspaces (FC) against HEAD (HB): three
# variants back to back, so each meets both of the box's run-to-run modes
set -u
DOFS_LIB=$PWD/exp/FC/libdofs_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_bench_config.py > gpurun_out/par_FC.log 2>&1 || { echo "parity FC failed"; tail -30 gpurun_out/par_FC.log; exit 1; }
tail -1 gpurun_out/par_FC.log
VARIANTS="HB=HB FT=FT FC=FC" N=${N:-4} bash tools/ab_env.sh
grep -h "contiguous" gpurun_out/abe_FC1.log | sort | uniq -c | head
