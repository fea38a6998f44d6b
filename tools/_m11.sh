cd $GRAFT_REPO_ROOT
M=$PWD/denseopticalflowsegmentation3d_amd/_build/measure/libdofs_hip.so
timeout -k 10 300 python tools/batch_loop.py 112 8 || exit 1
DOFS_LIB=$M DOFS_SKIP_B=1 timeout -k 10 300 python tools/batch_loop.py 112 8 || exit 1
DOFS_LIB=$M DOFS_SKIPMASK=3 timeout -k 10 300 python tools/batch_loop.py 112 8 || exit 1
DOFS_SERIAL=1 timeout -k 10 300 python tools/batch_loop.py 112 8 || exit 1
