"""MST sort fix-up anatomy (csrc/dofs_sortfix.h) on one synthetic batch: the group statistics of the
batch-wide key order (from the full-sort run's Kruskal-order event weights) and, per cut, the fix-up
counters (mixed pairs, groups, fallback flag) and the k_sortfix time.
usage: python tools/sortfix_stats.py [B] [H] [W]
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
H = int(sys.argv[2]) if len(sys.argv) > 2 else 1080
W = int(sys.argv[3]) if len(sys.argv) > 3 else 1920
ctx = runtime.Dofs(0, keep_events=True)
L = ctx.lib
L.dofs_debug_sort_cut.argtypes = [C.c_int]
L.dofs_debug_sort_cut.restype = C.c_int
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)


def run(cut, reps=3):
    L.dofs_debug_sort_cut(cut)
    ctx.probe("k_sortfix")
    for _ in range(reps):
        ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
    torch.cuda.synchronize()
    ms, n = ctx.probe_read()
    c = ctx.batch_counters(B)[0, 60:62].tolist()
    return ms / max(n, 1), c


run(0, 1)
keys = None if os.environ.get("NOSTAT") else np.concatenate([ctx.events(f)["weight"].view(np.uint64) for f in range(B)])
for cut in ((16, 24, 32) if keys is not None else ()):
    frame = np.repeat(np.arange(B), len(keys) // B)
    k = keys[np.lexsort((frame, keys))]  # the batch order: key, then emission (frame-major)
    t = k >> np.uint64(cut)
    brk = np.flatnonzero(t[1:] != t[:-1]) + 1
    starts = np.concatenate([[0], brk])
    ends = np.concatenate([brk, [len(t)]])
    mixed = np.flatnonzero((t[1:] == t[:-1]) & (k[1:] != k[:-1])) + 1
    gid = np.searchsorted(starts, mixed, side="right") - 1
    g = np.unique(gid)
    sz = ends[g] - starts[g]
    print(f"cut {cut}: {len(mixed)} mixed pairs in {len(g)} groups; group sizes max {sz.max() if len(sz) else 0} "
          f"p99 {int(np.percentile(sz, 99)) if len(sz) else 0}; >64: {(sz > 64).sum()}, >4096: {(sz > 4096).sum()}")
for cut in [int(c) for c in os.environ.get("CUTS", "0,16,24,32").split(",")]:
    ms, c = run(cut)
    print(f"cut {cut}: k_sortfix {ms:.3f} ms/batch, counters (groups sorted, fallback) {c}")
L.dofs_debug_sort_cut(24)
ctx.close()
