"""Snapshot-record capacity of the batch API: an overflow is reported (the full counts from
dofs_batch_records_copy, dofs_batch_fetch and the overlay), never dropped silently, and the labels stay
exact (KPaint works per history slot, not per stored record). Run on the host emulator of the product
pipeline (CPU) and on the GPU."""
import ctypes as C

import numpy as np
import pytest

from denseopticalflowsegmentation3d_amd.frames import RECORD_DTYPE
from oracle import binding as ob
from parity import params

H, W, B, MIN_SIZE, CAP = 90, 160, 2, 20, 2


def _run(ctx, flows, calib, prm, dev_ptr):
    persp, inv, up = calib
    return ctx.segment_batch_device(dev_ptr(flows), B, H, W, persp, inv, up, params=prm, stream=0)


def _check(ctx, calib, dev_alloc, dev_ptr, to_host):
    prm = params(MIN_SIZE, 8)
    persp, inv, up = calib
    oracle = [ob.segment(ob.synth_flow(H, W, s), persp, inv, up, params=prm, mode=0) for s in range(B)]
    assert all(len(o.snapshots) > CAP for o in oracle)  # the case overflows
    flows = dev_alloc(np.stack([ob.synth_flow(H, W, s) for s in range(B)]))
    old = ctx.snapshot_capacity()
    ctx.set_snapshot_capacity(CAP)
    try:
        bid = _run(ctx, flows, calib, prm, dev_ptr)
        blk = dev_alloc(np.zeros(4 * B + B * 4 * RECORD_DTYPE.itemsize, np.uint8))
        # more records per frame than the workspace keeps: refused whatever the data (all ranks alike)
        with pytest.raises(RuntimeError, match=r"\(4\)"):
            ctx.records_copy(dev_ptr(blk), 4, stream=0, batch=bid)
        # up to the capacity: the first records of every frame exist, the counts show the truncation
        ctx.records_copy(dev_ptr(blk), CAP, stream=0, batch=bid)
        h = to_host(blk)
        counts = h[:4 * B].view(np.int32)
        assert list(counts) == [len(o.snapshots) for o in oracle]
        recs = h[4 * B:4 * B + B * CAP * RECORD_DTYPE.itemsize].view(RECORD_DTYPE).reshape(B, CAP)
        for f in range(B):
            assert list(recs[f]["slot"]) == list(oracle[f].snapshots["slot"][:CAP])
            assert list(recs[f]["size"]) == list(oracle[f].snapshots["size"][:CAP])
        for f in range(B):
            r, snaps, labels, leaf, _ = ctx._result(H, W, 64, want_blur=False)
            rc = ctx.lib.dofs_batch_fetch(ctx.ctx, f, C.byref(r))
            assert rc == 4 and r.n_snapshots == len(oracle[f].snapshots)
            assert np.array_equal(labels, oracle[f].labels)  # exact despite the overflow
        ctr = ctx.batch_counters(B)
        assert [int(c) for c in ctr[:, 14]] == [len(o.snapshots) for o in oracle]  # C_OVF per frame
        # a capacity that fits: the same batch copies every record
        ctx.set_snapshot_capacity(64)
        bid = _run(ctx, flows, calib, prm, dev_ptr)
        ctx.records_copy(dev_ptr(blk), 4, stream=0, batch=bid)
        counts = to_host(blk)[:4 * B].view(np.int32)
        assert list(counts) == [len(o.snapshots) for o in oracle]
        assert not ctx.batch_counters(B)[:, 14].any()
    finally:
        ctx.set_snapshot_capacity(old)


def test_capacity_overflow_emulator(emu, calib):
    keep = []

    def alloc(a):
        a = np.ascontiguousarray(a)
        keep.append(a)
        return a
    _check(emu, calib, alloc, lambda a: a.ctypes.data, lambda a: a)


@pytest.mark.gpu
def test_capacity_overflow_gpu(calib):
    import torch
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    ctx = Dofs(0)
    try:
        _check(ctx, calib, lambda a: torch.from_numpy(np.ascontiguousarray(a)).to("cuda:0"),
               lambda t: t.data_ptr(), lambda t: t.cpu().numpy())
    finally:
        ctx.close()


def test_events_refused_without_kept_records(emu, calib):
    """dofs_keep_events (default off): a batch issued without it has no per-merge records, and dofs_events
    says so instead of returning unwritten ones (the emulator follows the HIP backend's rule)."""
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    ctx = Dofs(0, lib=emu.lib)
    try:
        flow = ob.synth_flow(24, 32, 5)
        ctx.segment(flow, *calib)
        with pytest.raises(RuntimeError, match="event records"):
            ctx.events(0)
        ctx.keep_events(True)
        ctx.segment(flow, *calib)
        assert len(ctx.events(0)) == 24 * 32 - 1
    finally:
        ctx.close()
