"""Diagnosis of the MST sort fix-up on one small batch: the batch order after the fix-up must be a
permutation of the full sort's pairs and sorted by (key, value). usage: python tools/sortfix_diag.py [cut]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

cut = int(sys.argv[1]) if len(sys.argv) > 1 else 24
fix = int(sys.argv[2]) if len(sys.argv) > 2 else 1
B, H, W = 4, 180, 320
ctx = runtime.Dofs(0, keep_events=True)
L = ctx.lib
L.dofs_debug_sort_cut.argtypes = [C.c_int]
L.dofs_debug_sort_dump.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
L.dofs_debug_sort_fix.argtypes = [C.c_int]
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 70)
prm = runtime.default_params()
prm.neighbor = int(os.environ.get("NB", "8"))
prm.min_size = 300
n = B * (H * W - 1) * (2 if prm.neighbor == 8 else 1)  # (upper bound: the MST has H W - 1 edges)
out, evs = {}, {}
cuts = [int(c) for c in os.environ.get("CUTS", str(cut)).split(",")]
runs = [(0, 1)] + [(c, fix) for c in cuts] * int(os.environ.get("REPS", "1"))
for r, (c, f) in enumerate(runs):
    k = torch.zeros(n, dtype=torch.int64, device="cuda")
    v = torch.zeros(n, dtype=torch.int32, device="cuda")
    L.dofs_debug_sort_cut(c)
    L.dofs_debug_sort_fix(f)
    L.dofs_debug_sort_dump(k.data_ptr(), v.data_ptr(), n)
    ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up, params=prm)
    torch.cuda.synchronize()
    print("cut", c, "fix", f, "batch ok", ctx.batch_counters(B)[0, 60:62].tolist(), flush=True)
    out[c] = (k.cpu().numpy().view(np.uint64), v.cpu().numpy().view(np.uint32))
    ev = [ctx.events(fr).tobytes() for fr in range(B)]
    if r == 0:
        evs[0] = ev
    else:
        k0_, v0_ = out[0]
        same = bool(np.array_equal(out[c][0], k0_) and np.array_equal(out[c][1], v0_))
        print(f"run {r} cut {c}: order == full sort {same}; events equal per frame", [a == b for a, b in zip(ev, evs[0])],
              flush=True)
k0, v0 = out[0]
k1, v1 = out[cuts[-1]]
print("full sort ordered:", bool(np.all((k0[1:] > k0[:-1]) | ((k0[1:] == k0[:-1]) & (v0[1:] > v0[:-1])))))
print("same multiset:", bool(np.array_equal(np.sort(v1), np.sort(v0))))
bad = np.flatnonzero((k1 != k0) | (v1 != v0))
print("positions differing from the full sort:", len(bad), bad[:10].tolist())
for i in bad[:5]:
    lo, hi = max(i - 3, 0), i + 4
    print(i, [hex(x) for x in k1[lo:hi]], v1[lo:hi].tolist(), "| full", [hex(x) for x in k0[lo:hi]], v0[lo:hi].tolist())
if not fix:  # the fix-up's logic on the truncated order, on the host (tools/sortfix_sim)
    key, val = k1.copy(), v1.copy()
    T = key >> np.uint64(cut)
    head = np.ones(n, bool)
    head[1:] = T[1:] != T[:-1]
    starts = np.flatnonzero(head)
    ends = np.append(starts[1:], n)
    for s0, e0 in zip(starts, ends):
        if e0 - s0 > 1 and len(np.unique(key[s0:e0])) > 1:
            o = np.lexsort((val[s0:e0], key[s0:e0]))
            key[s0:e0], val[s0:e0] = key[s0:e0][o], val[s0:e0][o]
    print("host fix-up of the truncated order == full sort:", bool(np.array_equal(key, k0) and np.array_equal(val, v0)))
