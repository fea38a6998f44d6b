# The MST offsets scanned frame-locally by a fixed per-frame total (FS, no rebase pass): GPU suite on
# the variant, then an A/B against HEAD with a memory-query process before each run
set -u
v=${V:-FS}
DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/suite_$v.log 2>&1 || { echo "suite $v failed"; tail -30 gpurun_out/suite_$v.log; exit 1; }
tail -1 gpurun_out/suite_$v.log
TINY=1 VARIANTS="H1 $v H2" N=${N:-3} bash tools/ab.sh
