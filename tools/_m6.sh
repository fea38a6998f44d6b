cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/m6/pytest.log 2>&1 || { tail -25 gpurun_out/m6/pytest.log; exit 1; }
tail -1 gpurun_out/m6/pytest.log
timeout -k 10 400 python -u tools/stress_determinism.py 30 > gpurun_out/m6/stress.log 2>&1 || { tail -5 gpurun_out/m6/stress.log; exit 1; }
tail -1 gpurun_out/m6/stress.log
VARIANTS="B=B E=E" N=2 bash tools/ab_env.sh
