cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05j
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05j/pytest.log 2>&1 || { tail -25 gpurun_out/r05j/pytest.log; exit 1; }
tail -2 gpurun_out/r05j/pytest.log
VARIANTS="A=A B=B" N=3 bash tools/ab_env.sh
