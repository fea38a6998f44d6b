"""GPU: a batch whose dataflow replay gave up a bounded wait (C_FLOWERR) can never ship results silently
(VERDICT r4 #1). dofs_debug_flow_giveup makes the next batches report a give-up; then every accessor of
the batch fails with DOFS_ERR_INVALID_RESULT — the records copy after writing every count as DOFS_RECORDS_INVALID
(so a collective gather still moves equal blocks and the receivers see the invalid frames), the fetch, the
final roots, the segment scores and the events — and FrameParallel.collect raises after its gather. The
next batch without the knob is valid again. The same holds for a replay record whose union-find root lies
outside its frame (dofs_debug_bad_root): the scoring refuses it instead of using it as an index
into its slot arrays, and every accessor reports the batch invalid."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B, H, W, PER = 3, 180, 320, 8


def test_giveup_fails_every_accessor(calib):
    import torch

    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.frames import FrameParallel, decode_records, records_nbytes
    ctx = runtime.Dofs(0, keep_events=True)
    lib = ctx.lib
    lib.dofs_debug_flow_giveup.argtypes = [C.c_int]
    lib.dofs_debug_flow_giveup.restype = C.c_int
    fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
    runtime.synth_flow_device(fl.data_ptr(), B, H, W, 55)
    torch.cuda.synchronize()
    blk = torch.zeros(records_nbytes(B, PER), dtype=torch.uint8, device="cuda")
    try:
        lib.dofs_debug_flow_giveup(1)
        bid = ctx.segment_batch_device(fl.data_ptr(), B, H, W, *calib)
        lib.dofs_debug_flow_giveup(0)
        rc = ctx.records_copy(blk.data_ptr(), PER, batch=bid, check=False)
        assert rc == 6, rc  # DOFS_ERR_INVALID_RESULT
        torch.cuda.synchronize()
        counts = blk[:4 * B].cpu().numpy().view(np.int32)
        assert (counts == -1).all(), counts
        with pytest.raises(RuntimeError, match="gather|replay|DOFS_RECORDS_INVALID"):
            decode_records(blk.cpu().numpy(), B, PER)
        with pytest.raises(RuntimeError, match="gave up a bounded wait"):
            ctx.fetch(0, want_blur=False)
        with pytest.raises(RuntimeError, match="gave up a bounded wait"):
            ctx.final_roots(0)
        with pytest.raises(RuntimeError, match="gave up a bounded wait"):
            ctx.segment_scores(0)
        with pytest.raises(RuntimeError, match="gave up a bounded wait"):
            ctx.events(0)
        fp = FrameParallel(ctx, 1, PER)
        lib.dofs_debug_flow_giveup(1)
        bid = fp.submit(fl, *calib)
        lib.dofs_debug_flow_giveup(0)
        with pytest.raises(RuntimeError, match="gave up a bounded wait"):
            fp.collect(bid)
        # the next batch is valid again
        bid = fp.submit(fl, *calib)
        g = fp.collect(bid)
        torch.cuda.synchronize()
        recs = decode_records(g.cpu().numpy(), B, PER)
        assert len(recs) == B and all(len(r) >= 0 for r in recs)
        assert ctx.fetch(0, want_blur=False).labels.shape == (H * W,)
    finally:
        lib.dofs_debug_flow_giveup(0)
        ctx.close()


def test_out_of_range_root_is_refused(calib):
    """An out-of-range root in a scoring candidate's replay record (injected after the replay) must not become an
    out-of-range atomic in KLift / KSlotEvent: the device refuses it, and every accessor of the batch fails with
    DOFS_ERR_INVALID_RESULT naming it; the context keeps working (no device fault), and the next batch is valid."""
    import torch

    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.frames import FrameParallel, decode_records, records_nbytes
    ctx = runtime.Dofs(0)
    lib = ctx.lib
    lib.dofs_debug_bad_root.argtypes = [C.c_int]
    lib.dofs_debug_bad_root.restype = C.c_int
    fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
    runtime.synth_flow_device(fl.data_ptr(), B, H, W, 56)
    torch.cuda.synchronize()
    blk = torch.zeros(records_nbytes(B, PER), dtype=torch.uint8, device="cuda")
    try:
        lib.dofs_debug_bad_root(1)
        bid = ctx.segment_batch_device(fl.data_ptr(), B, H, W, *calib)
        lib.dofs_debug_bad_root(0)
        rc = ctx.records_copy(blk.data_ptr(), PER, batch=bid, check=False)
        assert rc == 6, (rc, ctx.last_error())  # DOFS_ERR_INVALID_RESULT
        assert "outside its frame" in ctx.last_error()
        torch.cuda.synchronize()
        assert (blk[:4 * B].cpu().numpy().view(np.int32) == -1).all()
        for call in (lambda: ctx.fetch(0, want_blur=False), lambda: ctx.final_roots(0),
                     lambda: ctx.segment_scores(0)):
            with pytest.raises(RuntimeError, match="outside its frame"):
                call()
        fp = FrameParallel(ctx, 1, PER)
        bid = fp.submit(fl, *calib)
        g = fp.collect(bid)
        torch.cuda.synchronize()
        assert len(decode_records(g.cpu().numpy(), B, PER)) == B
        assert ctx.fetch(0, want_blur=False).labels.shape == (H * W,)
    finally:
        lib.dofs_debug_bad_root(0)
        ctx.close()
