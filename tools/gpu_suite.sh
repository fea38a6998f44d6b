#!/bin/bash
# One gpurun call: the GPU test suite, then a short bench (no CPU baseline), each step under its own time
# limit; logs under gpurun_out/$1/. Usage (from the repo root, on the GPU box): bash tools/gpu_suite.sh TAG [pytest args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
tag=${1:-run}
shift
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$out/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$out/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --cpu-frames 0 > "$out/bench.json" 2> "$out/bench.err"
rc=$?
head -c 400 "$out/bench.json"
exit $rc
