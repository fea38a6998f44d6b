cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05h
DOFS_SERIAL=1 DOFS_LIB=$PWD/denseopticalflowsegmentation3d_amd/_build/prof/libdofs_hip.so H=2160 W=3840 timeout -k 10 300 python tools/flow_stats.py 1 2 > gpurun_out/r05h/flow4k_prof.log 2>&1 || exit 1
tail -2 gpurun_out/r05h/flow4k_prof.log | cut -c1-500
