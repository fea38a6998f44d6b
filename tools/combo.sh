#!/bin/bash
# Bench once per configuration line of $COMBOS ("label|ENV=v ENV2=w|extra bench args", one per line),
# REPS times interleaved; prints value, median step and stage times per run. Stops at the first failure.
#   COMBOS=$'base||\nfused256|DOFS_FUSED_EXTRA=160|\nb128|DOFS_SLOTS=2|--batch 128' bash tools/combo.sh
set -u
REPS=${REPS:-1}
ARGS=${BENCH_ARGS:---cpu-frames 0 --no-h2d --steps 8 --warmup 2}
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in $(seq 1 "$REPS"); do
    while IFS='|' read -r label envs extra; do
        [ -z "$label" ] && continue
        log=gpurun_out/combo_${label}_$i.log
        env $envs timeout -k 10 600 python bench.py $ARGS $extra > "$log" 2>&1; rc=$?
        echo "$label rep=$i rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step_median": [0-9.]*' "$log" | tr '\n' ' ')"
        grep -o '"stages_ms_per_batch": {[^}]*}' "$log"
        if [ $rc -ne 0 ]; then tail -5 "$log"; exit $rc; fi
    done <<< "$COMBOS"
done
