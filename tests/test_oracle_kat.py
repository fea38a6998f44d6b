"""The oracle (and the product's host helpers) against the reference's own gtest known answers
(cpp/tests/test_liftig_3d.cpp). These are the only reference-provided vectors for this path."""
import math

import numpy as np
import pytest

from oracle import binding as ob
from oracle import ref_py as rp

# test_liftig_3d.cpp:183-185 (matrix literals) and :188-205 (expected Solution)
KAT_MAT = np.array([20.1377838, -13.4744920, 402.174272, 5.11635077, 800.335022, -62251.3321,
                    0.000393565444, 0.0397205947, 1.0], np.float32).reshape(3, 3)
KAT_INV = np.array([0.202212552, 0.00181942728, 31.9370859, -0.00182975914, 0.00123437589, 77.5774258,
                    -6.90475148e-06, -4.97462083e-05, 1.0], np.float32).reshape(3, 3)
KAT_UP = np.array([0.203701900, 0.00169508037, 32.3672674, 0.0, 0.00146371164, 29.6614710, 0.0,
                   -5.01704822e-05, 1.0], np.float32).reshape(3, 3)
KAT_DIR = (2.5470946, 1.9316475)
KAT_BOX = (375, 92, 576, 286)
EXP_PS_BEV = [(327.809749190909, 13476.772230116465), (1398.2414179174136, 2769.3562851313454),
              (2204.8576245955073, 2935.1653236816246), (647.3324083001849, 13473.77576520306)]
EXP_LOWER = [(385.305, 286.0), (375.0, 269.47327), (555.45557, 270.2111), (576.0, 286.92706)]
EXP_UPPER = [(385.305, 99.43571), (375.0, 92.75792), (555.45557, 92.0), (576.0, 98.69487)]
EXP_W, EXP_H, EXP_ORIENT = 0.5987518562843858, 0.7156805292391223, -1.6261444189491607
TOL = 1e-1  # the reference test's tolerance (:214-226)


def test_intersection_exists():  # :69-78
    r = ob.intersect([1, 1], [4, 4], [1, 8], [2, 4])
    assert abs(r[0] - 2.4) < 1e-2 and abs(r[1] - 2.4) < 1e-2


def test_intersection_parallel_is_nan():  # :80-89
    r = ob.intersect([1, 1], [1, 2], [3, 3], [3, 4])
    assert np.isnan(r).all()


def _check_kat(sol):
    assert sol["cls"] == 2
    for k, exp in (("ps_bev", EXP_PS_BEV), ("lower_face", EXP_LOWER), ("upper_face", EXP_UPPER)):
        got = np.asarray(sol[k], np.float64).reshape(4, 2)
        assert np.all(np.abs(got - np.asarray(exp)) < TOL), (k, got)
    assert abs(sol["w_error"] - EXP_W) < TOL
    assert abs(sol["h_error"] - EXP_H) < TOL
    assert abs(sol["orient"] - EXP_ORIENT) < TOL


def test_get_bottom_variants_kat_oracle():  # :179-227
    from denseopticalflowsegmentation3d_amd.abi import solution_dict
    _check_kat(solution_dict(ob.lift(KAT_DIR, KAT_BOX, KAT_MAT, KAT_INV, KAT_UP, 2)))


def test_get_bottom_variants_kat_python_restatement():
    s = rp.get_bottom_variants((np.float32(KAT_DIR[0]), np.float32(KAT_DIR[1])), KAT_BOX, KAT_MAT, KAT_INV,
                               KAT_UP, 2)
    _check_kat({k: (np.asarray(v, np.float64) if isinstance(v, list) else v) for k, v in s.items()})


def test_oracle_and_python_lifting_bit_exact():
    rng = np.random.default_rng(5)
    persp, inv, up = ob.calib()
    for _ in range(200):
        x0, y0 = int(rng.integers(0, 500)), int(rng.integers(40, 300))
        box = (x0, y0, x0 + int(rng.integers(5, 140)), y0 + int(rng.integers(5, 60)))
        d = rng.normal(size=2).astype(np.float32) * 3
        cls = int(rng.integers(0, 3))
        a = ob.lift(d, box, persp, inv, up[cls], cls)
        b = rp.get_bottom_variants((d[0], d[1]), box, persp, inv, up[cls], cls)
        assert a.valid == b["valid"]
        if not b["valid"]:
            continue
        assert a.w_error == b["w_error"] or (math.isnan(a.w_error) and math.isnan(b["w_error"]))
        assert a.h_error == b["h_error"] or (math.isnan(a.h_error) and math.isnan(b["h_error"]))
        assert a.orient == b["orient"]
        got = np.array(a.lower_face, np.float32).ravel()
        exp = np.array(b["lower_face"], np.float32).ravel()
        assert got.tobytes() == exp.tobytes()


def test_calibration_matches_kat_literals():
    """get_mat / get_mat_upper(2) restated (cv::getPerspectiveTransform) vs the literals the reference
    test hard-codes (:183-185, printed to 9 significant digits). The exact 0 / -0 entries of the
    upper-face homography pin the LU back-substitution order."""
    persp, inv, up = ob.calib()
    for got, exp in ((persp, KAT_MAT), (inv, KAT_INV), (up[2], KAT_UP)):
        assert np.allclose(got, exp, rtol=2e-7, atol=0), (got, exp)
    assert up[2][1][0] == 0.0 and up[2][2][0] == 0.0


def test_product_host_helpers_match_oracle():
    """dofs_calib / dofs_intersect (host code of the product library) == oracle, bit-exact."""
    from denseopticalflowsegmentation3d_amd import runtime
    p1, i1, u1 = runtime.calib()
    p0, i0, u0 = ob.calib()
    assert p1.tobytes() == p0.tobytes() and i1.tobytes() == i0.tobytes() and u1.tobytes() == u0.tobytes()
    rng = np.random.default_rng(0)
    for _ in range(100):
        pts = rng.normal(size=(4, 2)).astype(np.float32) * 50
        assert runtime.intersect(*pts).tobytes() == ob.intersect(*pts).tobytes()


def test_gaussian_kernel():
    k = ob.gaussian_kernel(3.0)
    assert len(k) == 25  # cvRound(3*4*2+1)|1 for float input
    assert np.array_equal(k, k[::-1])
    assert abs(float(k.astype(np.float64).sum()) - 1.0) < 1e-6
    assert np.array_equal(np.array(rp.gaussian_kernel(25, 3.0), np.float32), k)
