# Borůvka record hook by pointer (no finds, no CAS; mutual pairs resolved by the edge flag's atomic OR):
# the whole GPU suite on the variant library, then a same-box A/B against HEAD's
set -u
v=${V:-PH}
DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_$v.log 2>&1 || { echo "suite $v failed"; tail -30 gpurun_out/suite_$v.log; exit 1; }
tail -1 gpurun_out/suite_$v.log
VARIANTS="${VS:-F $v}" N=${N:-3} bash tools/ab.sh
