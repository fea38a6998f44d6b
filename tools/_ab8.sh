cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05l
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05l/pytest.log 2>&1 || { tail -25 gpurun_out/r05l/pytest.log; exit 1; }
tail -2 gpurun_out/r05l/pytest.log
VARIANTS="B=B C=C D=D E=E" N=2 bash tools/ab_env.sh
