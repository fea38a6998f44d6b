"""The rest of the reference's public boundary, vs the oracle:

- get_upper_face (lifting_3d.hpp:21-22, lifting_3d.cpp:290-348), get_upper_face_simple (:23-24, :261-288)
  and get_obj_size (:25, :524-528): dofs_upper_face / dofs_upper_face_simple / dofs_obj_size (host) and
  dofs_upper_face_batch (device). Float-only arithmetic: bit-exact on both.
- Forest::get_segment_best_score (graph.hpp:96, graph.cpp:386-389): segment_scores[root] is written for
  EVERY scored candidate before the convexity / threshold tests (graph.cpp:326) — the root's last scored
  score — and stays 0.0 elsewhere (:139). dofs_segment_scores.
- Forest::get_bounding_box after the loop (graph.hpp:103, graph.cpp:446-452): merge clears the non-root
  side (:208), so only the final roots keep a box. dofs_final_roots.

The oracle's faithful mode keeps the reference's own containers (segment_scores vector, bboxes vectors); the
product runs on the host emulator (CPU) and on the GPU. Scores recomputed on the GPU go through the device
atan2/sin/cos, so they are compared within 1e-9 (the lifting tolerance of tests/parity.py is 1e-6)."""
import numpy as np
import pytest

from oracle import binding as ob
from parity import params

GRID = [(1, 1, 0, 1), (5, 1, 0, 1), (9, 13, 2, 3), (24, 32, 0, 20), (30, 40, 3, 30), (90, 160, 0, 500)]


def _faces(n, seed):
    rng = np.random.default_rng(seed)
    boxes, lfs = [], []
    for i in range(n):
        x0, y0 = rng.integers(0, 600), rng.integers(0, 300)
        boxes.append([x0, y0, x0 + rng.integers(1, 300), y0 + rng.integers(1, 200)])
        if i % 10 == 0:  # degenerate: parallel sides (get_intersect's NaN branch)
            lfs.append([[0, 0], [0, 10], [10, 10], [10, 0]])
        else:
            lfs.append(rng.normal(size=(4, 2)) * 80 + [x0 + 100, y0 + 100])
    return np.array(boxes, np.int32), np.array(lfs, np.float32)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("simple", [False, True])
def test_upper_face_host(simple):
    from denseopticalflowsegmentation3d_amd import runtime
    boxes, lfs = _faces(300, 3 + simple)
    for b, lf in zip(boxes, lfs):
        assert np.array_equal(_bits(runtime.upper_face(b, lf, simple)), _bits(ob.upper_face(b, lf, simple)))
    # the KAT's face (test_liftig_3d.cpp:179-227, cls 2) stays finite through both forms
    lf = np.array([[330.1, 245.3], [302.7, 219.9], [352.2, 210.4], [378.5, 234.8]], np.float32)
    assert np.isfinite(runtime.upper_face([290, 150, 390, 250], lf, simple)).all()


def test_obj_size():
    from denseopticalflowsegmentation3d_amd import runtime
    for c in range(3):
        assert runtime.obj_size(c) == ob.obj_size(c)
    assert runtime.obj_size(2) == (370.0, 180.0)  # lifting_3d.cpp:526
    with pytest.raises(ValueError):
        runtime.obj_size(3)


def test_oracle_scores_modes_agree(calib):
    """The faithful mode (the reference's segment_scores vector) and the fast mode give the same
    scores and final boxes; scores differ from the snapshot (best) scores on some slot."""
    persp, inv, up = calib
    differs = False
    for H, W, seed, ms in GRID[2:]:
        flow = ob.synth_flow(H, W, seed)
        a = ob.segment(flow, persp, inv, up, params=params(ms, 8), mode=1, forest=True)
        b = ob.segment(flow, persp, inv, up, params=params(ms, 8), mode=0, forest=True)
        assert a.scores.tobytes() == b.scores.tobytes() and np.array_equal(a.boxes, b.boxes)
        roots = np.nonzero(a.boxes[:, 0] >= 0)[0]
        assert len(roots) == 1 and a.boxes[roots[0]].tolist() == [0, 0, W - 1, H - 1]
        for s in a.snapshots:
            assert a.scores[s["slot"]] != 0.0  # a snapshot slot was scored at least once
            differs |= a.scores[s["slot"]] != s["score"]
    assert differs  # the last scored candidate is not always the best


def _final_from_oracle(o):
    roots = np.nonzero(o.boxes[:, 0] >= 0)[0]
    return np.column_stack([roots, o.boxes[roots]]).astype(np.int32)


def _check_grid(ctx, calib, H, W, seed, ms, tol):
    persp, inv, up = calib
    flow = ob.synth_flow(H, W, seed)
    o = ob.segment(flow, persp, inv, up, params=params(ms, 8), mode=1, forest=True)
    ctx.segment(flow, persp, inv, up, params=params(ms, 8))
    got = ctx.segment_scores(0)
    assert np.array_equal(got == 0.0, o.scores == 0.0)
    assert np.allclose(got, o.scores, rtol=0, atol=tol)
    assert np.array_equal(ctx.final_roots(0), _final_from_oracle(o))


def _check_graph(ctx, calib, H, W, seed, ms, tol):
    from test_graph_api import _variants
    persp, inv, up = calib
    rng = np.random.default_rng(seed)
    blurred, cases = _variants(ob.synth_flow(H, W, seed), rng)
    for name, edges in cases:
        o = ob.segment_graph(blurred, edges["start"], edges["end"], edges["weight"], persp, inv, up,
                             params=params(ms, 8), mode=1, forest=True)
        ctx.segment_graph(blurred, edges, persp, inv, up, params=params(ms, 8))
        got = ctx.segment_scores(0)
        assert np.array_equal(got == 0.0, o.scores == 0.0), name
        assert np.allclose(got, o.scores, rtol=0, atol=tol), name
        assert np.array_equal(ctx.final_roots(0), _final_from_oracle(o)), name


@pytest.mark.parametrize("H,W,seed,ms", GRID)
def test_emu_grid(emu, calib, H, W, seed, ms):
    _check_grid(emu, calib, H, W, seed, ms, 0.0)


@pytest.mark.parametrize("H,W,seed,ms", [(9, 13, 1, 3), (24, 32, 2, 20), (40, 50, 5, 30)])
def test_emu_graph(emu, calib, H, W, seed, ms):
    _check_graph(emu, calib, H, W, seed, ms, 0.0)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed,ms", GRID + [(360, 640, 1, 500), (1080, 1920, 2, 500)])
def test_gpu_grid(gpu, calib, H, W, seed, ms):
    _check_grid(gpu, calib, H, W, seed, ms, 1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed,ms", [(9, 13, 1, 3), (24, 32, 2, 20), (90, 160, 5, 300)])
def test_gpu_graph(gpu, calib, H, W, seed, ms):
    _check_graph(gpu, calib, H, W, seed, ms, 1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("simple", [False, True])
def test_gpu_upper_face_batch(gpu, simple):
    boxes, lfs = _faces(500, 11 + simple)
    got = gpu.upper_face_batch(boxes, lfs, simple)
    want = np.stack([ob.upper_face(b, lf, simple) for b, lf in zip(boxes, lfs)])
    assert np.array_equal(_bits(got), _bits(want))
