"""GPU: the two KRT modes agree merge for merge.

The top-down global-depth KRT (DOFS_KRT_DNC=1, chip-wide: small batches and config 5's single 4K
frame) must give the same Kruskal reconstruction tree as the per-frame sweep (DOFS_KRT_DNC=0, the
large-batch default), hence the same merge events (root, rank, mean bits, bbox — graph.cpp:170-218),
path counters and labels. Round 3 found a cross-wave race in `k_dnc_compress` that lost an L-root in
about one of six first batches of a fresh context; it is caught here by fresh contexts and distinct
inputs per batch (a later batch on the same input would re-read the previous batch's sizes and hide
it). Both modes are checked against the oracle at a small size as well.

The race is also forced deterministically: with the wave-skew knob (dofs_debug_dnc_skew) the odd waves
of every k_dnc_compress workgroup sleep before reading their slot's maximum, so the even waves reach the
slot-table clear first in every iteration — exactly the interleaving that lost L-roots before the
barrier between read and clear existed. The DNC KRT must still equal the sweep merge for merge.
"""
import numpy as np
import pytest

from oracle import binding as ob
from parity import EVENT_FIELDS, params

pytestmark = pytest.mark.gpu

CTXS, BATCHES = 4, 3


def _run(monkeypatch, mode, B, H, W, calib, seeds, prm=None, skew=0):
    import ctypes as C

    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    monkeypatch.setenv("DOFS_KRT_DNC", mode)
    persp, inv, up = calib
    ctx = runtime.Dofs(0, keep_events=True)
    ctx.lib.dofs_debug_dnc_skew.argtypes = [C.c_int]
    assert ctx.lib.dofs_debug_dnc_skew(skew) == 0
    fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
    out = []
    try:
        for s in seeds:
            runtime.synth_flow_device(fl.data_ptr(), B, H, W, s)
            torch.cuda.synchronize()
            ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up, params=prm)
            torch.cuda.synchronize()
            c = ctx.batch_counters(B)
            ev = [ctx.events(f).copy() for f in range(B)]
            lab = ctx.fetch(B - 1, want_blur=False).labels.copy()
            out.append((c, ev, lab))
    finally:
        ctx.lib.dofs_debug_dnc_skew(0)
        ctx.close()
    return out


@pytest.mark.parametrize("B", [8])
def test_dnc_matches_sweep_fresh_contexts_1080p(monkeypatch, calib, B):
    H, W = 1080, 1920
    for k in range(CTXS):
        seeds = [1000 * k + B * b for b in range(BATCHES)]
        dnc = _run(monkeypatch, "1", B, H, W, calib, seeds)
        swp = _run(monkeypatch, "0", B, H, W, calib, seeds)
        for b, ((c1, e1, l1), (c0, e0, l0)) in enumerate(zip(dnc, swp)):
            where = f"context {k} batch {b}"
            assert int(c1[0, 58]) == 0, f"{where}: the DNC replay gave up (C_FLOWERR)"
            assert int(c0[0, 58]) == 0, f"{where}: the sweep replay gave up (C_FLOWERR)"
            for f in range(B):
                assert np.array_equal(e1[f], e0[f]), f"{where} frame {f}: merge events differ"
            assert np.array_equal(l1, l0), f"{where}: labels differ"


def test_dnc_matches_oracle_small(monkeypatch, calib):
    H, W, B = 180, 320, 4
    prm = params(300, 8)
    persp, inv, up = calib
    got = _run(monkeypatch, "1", B, H, W, calib, [77], prm=prm)[0]
    c, ev, lab = got
    assert int(c[0, 58]) == 0
    for f in range(B):
        o = ob.segment(ob.synth_flow(H, W, 77 + f), persp, inv, up, params=prm, mode=0, events=True)
        for k in EVENT_FIELDS:
            assert np.asarray(ev[f][k]).tobytes() == np.asarray(o.events[k]).tobytes(), f"frame {f}: event field {k}"
        if f == B - 1:
            assert np.array_equal(lab, o.labels)


def test_dnc_race_forced_by_wave_skew(monkeypatch, calib):
    """The k_dnc_compress interleaving of the round-3 race, forced in every workgroup iteration."""
    H, W, B = 540, 960, 4
    seeds = [5000]
    dnc = _run(monkeypatch, "1", B, H, W, calib, seeds, skew=64)
    swp = _run(monkeypatch, "0", B, H, W, calib, seeds)
    (c1, e1, l1), (c0, e0, l0) = dnc[0], swp[0]
    assert int(c1[0, 58]) == 0 and int(c0[0, 58]) == 0
    for f in range(B):
        assert np.array_equal(e1[f], e0[f]), f"frame {f}: merge events differ under the wave skew"
    assert np.array_equal(l1, l0)


def test_tail_batch_keeps_large_workspace(calib):
    """a small tail batch (<= 8 frames, the DNC KRT's auto range) on a workspace laid out for a
    larger batch runs the sweep in place instead of re-laying the workspace out (no free + re-allocation
    down and back up); its results equal the oracle's."""
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    H, W = 180, 320
    prm = params(300, 8)
    persp, inv, up = calib
    ctx = runtime.Dofs(0, keep_events=True)
    try:
        fl = torch.empty((16, H, W, 2), dtype=torch.float32, device="cuda")
        runtime.synth_flow_device(fl.data_ptr(), 16, H, W, 300)
        sizes = []
        for B in (16, 16, 16, 4, 4, 4, 16):  # every workspace sees the large shape, then a tail batch
            ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up, params=prm)
            torch.cuda.synchronize()
            sizes.append(ctx.workspace_bytes())
            if B == 4:
                c = ctx.batch_counters(B)
                assert int(c[0, 58]) == 0
                for f in (0, 3):
                    o = ob.segment(ob.synth_flow(H, W, 300 + f), persp, inv, up, params=prm, mode=0, events=True)
                    ev = ctx.events(f)
                    for k in EVENT_FIELDS:
                        assert np.asarray(ev[k]).tobytes() == np.asarray(o.events[k]).tobytes(), (f, k)
        assert len(set(sizes)) == 1, sizes  # no workspace was laid out again
    finally:
        ctx.close()


@pytest.mark.parametrize("mode", ["0", "1"])
def test_deep_depth_forms_equal(monkeypatch, calib, mode):
    """The LDS KRT's depths below 32 merges as the register window pass (dofs_debug_krt_deep_wave(1), the
    default) and as union-find depths (0) give the same tree, in both KRT modes. The union-find form leaves the first
    half's last merge without a size in LDS (the top level writes it to SZ), which the second half's
    prefetched labels must then take from SZ — the case this pins."""
    import ctypes as C

    from denseopticalflowsegmentation3d_amd import runtime
    B, H, W = 12, 270, 480
    seeds = [77, 177]
    lib = runtime.load()
    lib.dofs_debug_krt_deep_wave.argtypes = [C.c_int]
    lib.dofs_debug_krt_deep_wave.restype = C.c_int
    old = lib.dofs_debug_krt_deep_wave(1)
    try:
        a = _run(monkeypatch, mode, B, H, W, calib, seeds)
        lib.dofs_debug_krt_deep_wave(0)
        b = _run(monkeypatch, mode, B, H, W, calib, seeds)
    finally:
        lib.dofs_debug_krt_deep_wave(old)
    for (ca, ea, la), (cb, eb, lb) in zip(a, b):
        assert int(ca[0, 58]) == 0 and int(cb[0, 58]) == 0  # C_FLOWERR (the list positions are not ordered)
        assert np.array_equal(la, lb)
        for f in range(B):
            for name in EVENT_FIELDS:
                assert np.array_equal(ea[f][name], eb[f][name]), (f, name)
