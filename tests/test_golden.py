"""Golden fixtures: the oracle must reproduce them (regression pin), and so must the HIP path (gpu)."""
import numpy as np
import pytest

from golden_io import load, names
from oracle import binding as ob
from parity import EVENT_FIELDS, check_solution_close


def _b(a):
    return np.ascontiguousarray(a).tobytes()


@pytest.mark.parametrize("name", names())
def test_oracle_reproduces_golden(name):
    g = load(name)
    o = ob.segment(g["flow"], *g["calib"], params=g["prm"], mode=0, events=True)
    assert _b(o.blurred) == _b(g["blurred"])
    assert _b(o.events) == _b(g["events"])
    assert _b(o.snapshots) == _b(g["snapshots"])
    for s, m in zip(o.snapshots, g["members"]):
        assert np.array_equal(o.members(s), m)
    assert np.array_equal(o.labels, g["labels"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", names())
def test_gpu_reproduces_golden(gpu, name):
    g = load(name)
    r = gpu.segment(g["flow"], *g["calib"], params=g["prm"])
    ev = gpu.events(0)
    assert _b(r.blurred) == _b(g["blurred"])
    for k in EVENT_FIELDS:
        assert _b(ev[k]) == _b(g["events"][k]), k
    assert len(r.snapshots) == len(g["snapshots"])
    for k in ("slot", "event", "size", "bbox", "move"):
        assert _b(r.snapshots[k]) == _b(g["snapshots"][k]), k
    for a, b, m in zip(r.snapshots, g["snapshots"], g["members"]):
        assert np.array_equal(r.members(a), m)
        check_solution_close(a["sol"], b["sol"])
        assert abs(a["score"] - b["score"]) <= 1e-6
    assert np.array_equal(r.labels, g["labels"])
