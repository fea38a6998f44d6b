cd $GRAFT_REPO_ROOT
M=$PWD/denseopticalflowsegmentation3d_amd/_build/measure/libdofs_hip.so
for d in 0 15000 30000 0 15000 30000; do
  DOFS_LIB=$M DOFS_B_DELAY=$d timeout -k 10 300 python tools/batch_loop.py 112 8 | sed "s/^/delay $d us: /" || exit 1
done
