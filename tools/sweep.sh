#!/bin/bash
# Environment-knob sweep on one GPU box: optional parity suite, then the bench once per value of one
# knob (repeated REPS times, values interleaved so box drift hits all of them alike), printing the
# value, the median step and the stage times of each run. Replaces the round-1 one-off sweep scripts.
#   VAR=DOFS_LONG_PATH VALUES="256 128 512" bash tools/sweep.sh
#   VAR=B VALUES="64 96 128" bash tools/sweep.sh          (B: frames per batch, passed as --batch)
#   VAR=DOFS_FLOW_LONG VALUES="128 512" BENCH_ARGS="--steps 6 --warmup 2" REPS=2 PARITY=1 bash tools/sweep.sh
# Knobs read by the library: dofs_knobs.h (DESIGN.md §5 "Runtime knobs"); any other DOFS_* name makes
# dofs_create fail.
set -u
: "${VAR:?VAR=knob name}" "${VALUES:?VALUES=space-separated values}"
REPS=${REPS:-1}
ARGS=${BENCH_ARGS:---cpu-frames 0 --no-h2d}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${PARITY:-}" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
        --timeout-method thread > gpurun_out/sweep_pytest.log 2>&1; rc=$?
    echo "pytest rc=$rc"; tail -2 gpurun_out/sweep_pytest.log
    if [ $rc -ne 0 ]; then exit $rc; fi
fi
for i in $(seq 1 "$REPS"); do
    for v in $VALUES; do
        log=gpurun_out/sweep_${VAR}_${v}_$i.log
        if [ "$VAR" = B ]; then
            timeout -k 10 600 python bench.py $ARGS --batch "$v" > "$log" 2>&1; rc=$?
        else
            env "$VAR=$v" timeout -k 10 600 python bench.py $ARGS > "$log" 2>&1; rc=$?
        fi
        echo "$VAR=$v rep=$i rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step_median": [0-9.]*' "$log" | tr '\n' ' ')"
        grep -o '"stages_ms_per_batch": {[^}]*}' "$log"
        if [ $rc -ne 0 ]; then exit $rc; fi
    done
done
