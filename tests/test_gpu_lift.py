"""GPU: the exported lifting entry points (dofs_lift, dofs_lift_batch, dofs_intersect_batch) against the
reference's own known answers (cpp/tests/test_liftig_3d.cpp) and against the CPU oracle.

Tolerances: the reference KAT's own 0.1 (test_liftig_3d.cpp:214-226); against the oracle, the stated
float tolerance of the lifting path (tests/parity.py::check_solution_close: 1e-3 px + 1e-5 relative
on corners, 1e-6 on errors / orientation) — the device atan2 / sin / cos (double) may differ from
glibc by an ulp. get_intersect has no transcendental, so it is compared bit for bit."""
import numpy as np
import pytest

from denseopticalflowsegmentation3d_amd.abi import solution_dict
from oracle import binding as ob
from parity import check_solution_close
from test_oracle_kat import KAT_BOX, KAT_DIR, KAT_INV, KAT_MAT, KAT_UP, _check_kat

pytestmark = pytest.mark.gpu


def test_get_bottom_variants_kat_gpu(gpu):
    """test_liftig_3d.cpp:179-227 through dofs_lift (cls 2, the test's matrices)."""
    _check_kat(gpu.lift(KAT_DIR, KAT_BOX, KAT_MAT, KAT_INV, KAT_UP, 2))


def test_get_bottom_variants_kat_gpu_batch(gpu):
    """The same KAT through dofs_lift_batch (inv_upper of class 2 in slot 2 of the 3-matrix array)."""
    up27 = np.zeros((3, 3, 3), np.float32)
    up27[2] = KAT_UP
    out = gpu.lift_batch([KAT_DIR], [KAT_BOX], [2], KAT_MAT, KAT_INV, up27)
    _check_kat(solution_dict(out[0]))


def _random_boxes(n, seed):
    rng = np.random.default_rng(seed)
    x0 = rng.integers(0, 1700, n)
    y0 = rng.integers(40, 900, n)
    boxes = np.stack([x0, y0, x0 + rng.integers(5, 400, n), y0 + rng.integers(5, 180, n)], 1).astype(np.int32)
    dirs = (rng.normal(size=(n, 2)) * 3).astype(np.float32)
    cls = rng.integers(0, 3, n).astype(np.int32)
    return dirs, boxes, cls


def test_lift_batch_matches_oracle(gpu, calib):
    persp, inv, up = calib
    dirs, boxes, cls = _random_boxes(200, 17)
    got = gpu.lift_batch(dirs, boxes, cls, persp, inv, up)
    nvalid = 0
    for i in range(len(dirs)):
        o = solution_dict(ob.lift(dirs[i], boxes[i], persp, inv, up[cls[i]], int(cls[i])))
        g = got[i]
        if not o["valid"]:
            assert not g["valid"], i
            continue
        nvalid += 1
        check_solution_close(o, g)
    assert nvalid > 50  # the sample exercises the full back-projection, not only rejections


def test_lift_single_matches_oracle(gpu, calib):
    persp, inv, up = calib
    dirs, boxes, cls = _random_boxes(20, 3)
    for i in range(len(dirs)):
        c = int(cls[i])
        o = solution_dict(ob.lift(dirs[i], boxes[i], persp, inv, up[c], c))
        g = gpu.lift(dirs[i], boxes[i], persp, inv, up[c], c)
        assert o["valid"] == g["valid"]
        if o["valid"]:
            check_solution_close(o, g)


def test_intersect_device_reference_cases(gpu):
    """test_liftig_3d.cpp:69-78 (≈(2.4, 2.4), tol 1e-2) and :80-89 (parallel lines -> NaN)."""
    r = gpu.intersect_batch([[1, 1], [4, 4], [1, 8], [2, 4], [1, 1], [1, 2], [3, 3], [3, 4]])
    assert abs(r[0, 0] - 2.4) < 1e-2 and abs(r[0, 1] - 2.4) < 1e-2
    assert np.isnan(r[1]).all()


def test_intersect_device_bit_exact(gpu):
    rng = np.random.default_rng(4)
    pts = (rng.normal(size=(500, 4, 2)) * 50).astype(np.float32)
    pts[:50, 3] = pts[:50, 2] + (pts[:50, 1] - pts[:50, 0])  # parallel pairs
    got = gpu.intersect_batch(pts)
    exp = np.stack([ob.intersect(*p) for p in pts])
    assert got.tobytes() == exp.tobytes()
