"""Overlay: plot_best_segments_simple + draw_cube (cpp/src/draw.cpp:85-160).

CPU: the device line walk (closed-form Bresenham, dofs_overlay.h, run on the host by the test
emulator) against the oracle's iterative LineIterator/clipLine restatement on random, clipped and
degenerate lines; the whole overlay step of the product (emulator) against the oracle's literal
restatement. GPU: the HIP overlay (host and device-batch entry points, in place) against the oracle
restatement applied to the GPU's own snapshots — bit-exact (uint8 output).
Parity against OpenCV itself is unpinned (OpenCV absent; see oracle/overlay.cpp)."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import binding as ob
from parity import params

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def emu_lines(emu):
    L = C.CDLL(os.path.join(ROOT, "tests", "emu", "_build", "libdofs_emu.so"))
    L.emu_line_mask.argtypes = [C.c_int32, C.c_int32, C.c_float, C.c_float, C.c_float, C.c_float,
                                C.POINTER(C.c_uint8)]
    return L


def _emu_mask(L, H, W, a, b):
    m = np.zeros((H, W), np.uint8)
    L.emu_line_mask(H, W, float(a[0]), float(a[1]), float(b[0]), float(b[1]), m.ctypes.data_as(C.POINTER(C.c_uint8)))
    return m


def _lines(rng, H, W, n):
    out = []
    for _ in range(n):
        k = rng.integers(0, 4)
        if k == 0:    # inside
            a, b = rng.uniform([0, 0], [W, H], size=(2, 2))
        elif k == 1:  # ends well outside (clipLine)
            a, b = rng.uniform([-2 * W, -2 * H], [3 * W, 3 * H], size=(2, 2))
        elif k == 2:  # exact .5 ends (round half to even), short segments
            a = rng.integers(-3, max(W, H) + 3, 2) + 0.5
            b = a + rng.integers(-4, 5, 2)
        else:         # axis-aligned and 45 degree
            a = rng.integers(0, [W, H])
            d = rng.integers(-40, 41)
            b = a + [(d, 0), (0, d), (d, d), (d, -d)][rng.integers(0, 4)]
        out.append((np.asarray(a, np.float32), np.asarray(b, np.float32)))
    return out


def test_line_walk_matches_line_iterator(emu_lines):
    rng = np.random.default_rng(7)
    for H, W in [(1, 1), (5, 9), (37, 61), (120, 90)]:
        for a, b in _lines(rng, H, W, 300):
            assert np.array_equal(_emu_mask(emu_lines, H, W, a, b), ob.line_mask(H, W, a, b)), (H, W, a, b)


@pytest.mark.parametrize("a,b", [((np.nan, 3.0), (10.0, 4.0)), ((1e10, 2.0), (3.0, 4.0)), ((-1e10, -1e10), (1e10, 1e10)),
                                 ((2.5, 2.5), (2.5, 2.5)), ((-0.5, 7.5), (40.5, -0.5)), ((3.0, -5.0), (3.0, 50.0))])
def test_line_walk_degenerate(emu_lines, a, b):
    H, W = 31, 43
    a, b = np.float32(a), np.float32(b)
    assert np.array_equal(_emu_mask(emu_lines, H, W, a, b), ob.line_mask(H, W, a, b))


def _frame(rng, H, W):
    return rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)


@pytest.mark.parametrize("H,W,seed,min_score", [(90, 160, 0, 0.7), (180, 320, 1, 0.7), (180, 320, 2, 0.3)])
def test_emu_overlay_matches_oracle(emu, calib, H, W, seed, min_score):
    prm = params(500, 8)
    prm.overlay_min_score = min_score
    flow = ob.synth_flow(H, W, seed)
    r = emu.segment(flow, *calib, params=prm)
    fr = _frame(np.random.default_rng(seed), H, W)
    got = emu.overlay(fr)
    want = ob.overlay(fr, r.snapshots, r.leaf_order, min_score)
    assert (r.snapshots["score"] > min_score).sum() > 0
    assert np.array_equal(got, want)
    o = ob.segment(flow, *calib, params=prm)  # the oracle end to end (emulator lifting is bit-exact)
    assert np.array_equal(got, ob.overlay(fr, o.snapshots, o.leaf_order, min_score))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,seed", [(90, 160, 0), (360, 640, 3), (1080, 1920, 0)])
def test_gpu_overlay_host(gpu, calib, H, W, seed):
    r = gpu.segment(ob.synth_flow(H, W, seed), *calib, params=params(500, 8))
    fr = _frame(np.random.default_rng(seed), H, W)
    got = gpu.overlay(fr)
    assert np.array_equal(got, ob.overlay(fr, r.snapshots, r.leaf_order, 0.7))
    assert (got != fr).any()


@pytest.mark.gpu
def test_gpu_overlay_batch_in_place(gpu, calib):
    import torch
    B, H, W = 3, 360, 640
    dev = torch.device("cuda", 0)
    flows = np.stack([ob.synth_flow(H, W, s) for s in range(B)])
    frames = np.stack([_frame(np.random.default_rng(10 + s), H, W) for s in range(B)])
    d_flow = torch.from_numpy(flows).to(dev)
    d_fr = torch.from_numpy(frames).to(dev)
    d_out = torch.empty_like(d_fr)
    sh = torch.cuda.current_stream(dev).cuda_stream
    bid = gpu.segment_batch_device(d_flow.data_ptr(), B, H, W, *calib, params=params(500, 8), stream=sh)
    gpu.overlay_batch_device(bid, d_fr.data_ptr(), d_out.data_ptr(), stream=sh)
    out = d_out.cpu().numpy()
    gpu.overlay_batch_device(bid, d_fr.data_ptr(), d_fr.data_ptr(), stream=sh)  # in place, as the reference
    inplace = d_fr.cpu().numpy()
    for f in range(B):
        r = gpu.fetch(f, want_blur=False)
        want = ob.overlay(frames[f], r.snapshots, r.leaf_order, 0.7)
        assert np.array_equal(out[f], want), f
        assert np.array_equal(inplace[f], want), f
