"""GPU: the replay's constant-key chunks change nothing but speed.

The long-path loop skips the rank/root key update for a 64-step chunk when no step's light child
reaches the carried rank (union by rank leaves the key as it is: graph.cpp:177-182, 210-213).
dofs_debug_replay_keyfast(0) runs every chunk with the key update; on the same seeded 1080p batch the
two modes' merge events (root, rank, size, mean bits, bbox) and labels must be identical. Parity of the
default mode against the oracle is covered by every other GPU test.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B, H, W = 4, 1080, 1920


def _run(gpu, calib, fl, keyfast):
    import torch
    lib = gpu.lib
    lib.dofs_debug_replay_keyfast.argtypes = [C.c_int]
    lib.dofs_debug_replay_keyfast.restype = C.c_int
    old = lib.dofs_debug_replay_keyfast(keyfast)
    try:
        gpu.segment_batch_device(fl.data_ptr(), B, H, W, *calib)
        torch.cuda.synchronize()
        c = gpu.batch_counters(B)
        ev = [gpu.events(f).view(np.uint8).copy() for f in range(B)]
        lab = gpu.fetch(B - 1, want_blur=False).labels
    finally:
        lib.dofs_debug_replay_keyfast(old)
    return int(c[0, 58]), ev, lab


def test_constant_key_chunks_change_nothing(gpu, calib):
    import torch

    from denseopticalflowsegmentation3d_amd import runtime
    fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
    runtime.synth_flow_device(fl.data_ptr(), B, H, W, 500)
    torch.cuda.synchronize()
    ea, eva, la = _run(gpu, calib, fl, 1)
    eb, evb, lb = _run(gpu, calib, fl, 0)
    assert ea == 0 and eb == 0  # C_FLOWERR
    for f in range(B):
        assert eva[f].tobytes() == evb[f].tobytes(), f"frame {f}: merge events differ"
    assert np.array_equal(la, lb)
