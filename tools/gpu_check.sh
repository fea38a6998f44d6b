#!/bin/bash
# One GPU session: parity tests, the default bench line, a rocprofv3 kernel-trace summary.
# Stops at the first step that faults, aborts or times out (exit >= 2 other than pytest's 1).
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
    return 0
}
export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread ${TESTS:-}
fi
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ -n "${ROCPROF:-}" ]; then
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-stages --no-h2d
fi
exit 0
