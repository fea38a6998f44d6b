"""GPU: the batch path is deterministic across repetitions while its workspaces are reused and re-laid out —
the fixed-job split of test_gpu_bench_config.py (three simulated ranks, chunks of 8 and 6 frames through
frames.Pipelined) run again and again on one keep_events context, with a larger batch in between that
re-lays out the workspaces, must give the same records every time (tools/stress_determinism.py is the
longer form). Round 5: a 24-byte replay record let stale neighbour bytes reach a reader about once in fifty
runs; that form failed this check, the 32-byte one passes it."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("keep", ["1", "0"])
def test_repeated_batches_give_identical_records(keep):
    # its own process: the tool's context and workspaces are fresh, as bench.py's are. keep "0": a default
    # context, whose stage B reuses stage A's dead arrays and the replay inputs
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "stress_determinism.py"), "8", "-", keep],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "differed 0 of 7" in r.stdout
