#!/bin/bash
# One GPU session at HEAD: parity suite + bench + kernel-trace stats (tools/gpu_check.sh), then the
# per-kernel PMC passes (tools/pmc_round.sh). Stops at the first step that faults or times out.
set -u
ROCPROF=1 bash tools/gpu_check.sh || exit $?
bash tools/pmc_round.sh
