# The KRT sweep's records without an initialisation pass (NI: phase D writes whole root records; with the
# single-pixel flags no find reads a record D has not written): GPU suite on the variant, then an A/B
set -u
v=${V:-NI}
DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_$v.log 2>&1 || { echo "suite $v failed"; tail -30 gpurun_out/suite_$v.log; exit 1; }
tail -1 gpurun_out/suite_$v.log
DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 600 python tools/stress_determinism.py 12 - 0 > gpurun_out/stress_$v.log 2>&1 || { tail -5 gpurun_out/stress_$v.log; exit 1; }
tail -1 gpurun_out/stress_$v.log
TINY=1 VARIANTS="H0 $v" N=${N:-4} bash tools/ab.sh
