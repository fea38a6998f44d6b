set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05a/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python bench.py --cpu-frames 0 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err
echo "exit $?"
tail -3 gpurun_out/r05a/pytest_gpu.log
cat gpurun_out/r05a/bench.json | head -c 600
