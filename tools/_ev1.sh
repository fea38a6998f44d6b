cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05m/pytest.log 2>&1 || { tail -25 gpurun_out/r05m/pytest.log; exit 1; }
tail -2 gpurun_out/r05m/pytest.log
bash tools/round_evidence.sh
