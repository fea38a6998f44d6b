cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m8
DOFS_LIB=$PWD/denseopticalflowsegmentation3d_amd/_build/krt/libdofs_hip.so timeout -k 10 300 python tools/krt_timing.py 112 3 > gpurun_out/m8/krt_timing.log 2>&1 || { tail -5 gpurun_out/m8/krt_timing.log; exit 1; }
tail -30 gpurun_out/m8/krt_timing.log
