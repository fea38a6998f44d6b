"""GPU: the batch MST sort on truncated keys + its fix-up (csrc/dofs_sortfix.h) gives the full-key order.

Kruskal's order is the stable order of the 64-bit weight keys (segment.cpp:68). The batch sort keeps the
top 64 - cut bits and the fix-up re-sorts every run of equal truncated keys holding different weights.
Each cut's per-merge event records (Kruskal order) must equal those of the full 64-bit sort (cut 0),
bit for bit; cut 48 (16-bit keys) makes mixed groups of thousands and drives the merge-sort fallback.
"""
import ctypes as C

import numpy as np
import pytest

from oracle import binding as ob
from parity import params

pytestmark = pytest.mark.gpu

H, W, B = 180, 320, 4
C_SORTFIX = 60  # dofs_common.h: frame 0 fix-up counters (groups sorted locally, fallback flag)


def _run(gpu, calib, flows, cut):
    import torch
    lib = gpu.lib
    lib.dofs_debug_sort_cut.argtypes = [C.c_int]
    lib.dofs_debug_sort_cut.restype = C.c_int
    old = lib.dofs_debug_sort_cut(cut)
    try:
        sh = torch.cuda.current_stream().cuda_stream
        gpu.segment_batch_device(flows.data_ptr(), B, H, W, *calib, params=params(300, 8), stream=sh)
        torch.cuda.synchronize()
        ev = [gpu.events(f).copy() for f in range(B)]
        labels = [gpu.fetch(f, want_blur=False).labels for f in range(B)]
        ctr = gpu.batch_counters(B)[0, C_SORTFIX:C_SORTFIX + 2].copy()
    finally:
        lib.dofs_debug_sort_cut(old)
    return ev, labels, ctr


def test_truncated_sort_matches_full(gpu, calib):
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    flows = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda:0")
    runtime.synth_flow_device(flows.data_ptr(), B, H, W, seed0=70, stream=torch.cuda.current_stream().cuda_stream)
    ev0, lab0, ctr0 = _run(gpu, calib, flows, 0)
    assert ctr0.tolist() == [0, 0]  # no fix-up after the full sort
    for f in range(B):  # the full sort is the oracle's order
        o = ob.segment(ob.synth_flow(H, W, 70 + f), *calib, params=params(300, 8), mode=0)
        assert np.array_equal(lab0[f], o.labels)
    seen = {}
    for cut in (24, 32, 40, 48):
        ev, lab, ctr = _run(gpu, calib, flows, cut)
        seen[cut] = ctr.tolist()
        for f in range(B):  # field by field (the records' padding bytes are not written)
            for name in ev0[f].dtype.names:
                assert np.array_equal(ev[f][name], ev0[f][name]), (cut, f, name)
            assert np.array_equal(lab[f], lab0[f]), (cut, f)
    assert seen[24][0] > 0 and seen[24][1] == 0  # mixed groups sorted by the local pass, no fallback
    assert seen[32][0] > seen[24][0]
    assert seen[48][1] == 1  # 16-bit keys: mixed groups longer than kFixScan, the fallback merge sort
