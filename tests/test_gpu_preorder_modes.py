"""GPU: the two forms of the heavy-first preorder (K4) give the same positions.

Batches of at most 8 frames (DOFS_PRE_JUMP, default 8) take the chip-wide form: the LDS KRT's epilogue
writes each block's outside children's jump words and path-top flags, the block tops jump (KJumpTop) and
every merge adds its top's position (KOrdMerge). Larger batches take the per-frame top-down sweep
(k_pre_sweep). Both must give the same preorder, hence the same replay (Forest::merge, graph.cpp:170-218):
every merge event, the snapshots and labels, bit for bit, and equal to the oracle.
"""
import numpy as np
import pytest

from oracle import binding as ob
from parity import EVENT_FIELDS, params

pytestmark = pytest.mark.gpu


def _run(monkeypatch, jump, B, H, W, calib, seed, prm, krt=None):
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    monkeypatch.setenv("DOFS_PRE_JUMP", "8" if jump else "0")
    if krt is not None:
        monkeypatch.setenv("DOFS_KRT_DNC", krt)
    persp, inv, up = calib
    ctx = runtime.Dofs(0, keep_events=True)
    try:
        fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
        runtime.synth_flow_device(fl.data_ptr(), B, H, W, seed)
        ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up, params=prm)
        torch.cuda.synchronize()
        c = ctx.batch_counters(B)
        ev = [ctx.events(f).copy() for f in range(B)]
        res = [ctx.fetch(f, want_blur=False) for f in range(B)]
        return c, ev, res
    finally:
        ctx.close()


@pytest.mark.parametrize("krt", ["1", "0"])  # the DNC KRT (the small-batch default) and the fused sweep
def test_jump_equals_sweep_1080p(monkeypatch, calib, krt):
    B, H, W = 4, 1080, 1920
    prm = params(500, 8)
    cj, ej, rj = _run(monkeypatch, True, B, H, W, calib, 910, prm, krt)
    cs, es, rs = _run(monkeypatch, False, B, H, W, calib, 910, prm, krt)
    assert int(cj[0, 58]) == 0 and int(cs[0, 58]) == 0
    for f in range(B):
        for k in ej[f].dtype.names:
            assert np.array_equal(ej[f][k], es[f][k]), (f, k)
        assert np.array_equal(rj[f].labels, rs[f].labels), f
        assert np.array_equal(rj[f].snapshots["event"], rs[f].snapshots["event"]), f
        assert np.array_equal(rj[f].leaf_order, rs[f].leaf_order), f


def test_jump_matches_oracle(monkeypatch, calib):
    B, H, W = 3, 270, 480
    prm = params(300, 8)
    persp, inv, up = calib
    c, ev, res = _run(monkeypatch, True, B, H, W, calib, 420, prm)
    assert int(c[0, 58]) == 0
    for f in range(B):
        o = ob.segment(ob.synth_flow(H, W, 420 + f), persp, inv, up, params=prm, mode=0, events=True)
        for k in EVENT_FIELDS:
            assert np.asarray(ev[f][k]).tobytes() == np.asarray(o.events[k]).tobytes(), (f, k)
        assert np.array_equal(res[f].labels, o.labels)
        assert np.array_equal(res[f].snapshots["slot"], o.snapshots["slot"])
