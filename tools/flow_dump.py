"""Diagnosis of a dataflow replay that gave up (C_FLOWERR): runs synthetic 1080p batches in a fresh context
and, for the first batch with the error, lists the paths left incomplete and what each waits on.
usage: DOFS_KRT_DNC=1 python tools/flow_dump.py B [batches]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 1
H, W = 1080, 1920
ctx = runtime.Dofs(0, keep_events=True)  # the graph arrays stay readable after the batch
L = ctx.lib
L.dofs_debug_ws_ptrs.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.POINTER(C.c_longlong)]
path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = C.CDLL(path)
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]


def d2h(ptr, off_bytes, n_bytes, dtype):
    a = np.empty(n_bytes // np.dtype(dtype).itemsize, dtype)
    assert hip.hipMemcpy(a.ctypes.data, ptr + off_bytes, n_bytes, 2) == 0
    return a


persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)
torch.cuda.synchronize()
for b in range(NB):
    ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
    torch.cuda.synchronize()
    c = ctx.batch_counters(B)
    print(f"batch {b}: flowerr {int(c[0, 58])}", flush=True)
    if not c[0, 58]:
        continue
    ptrs = (C.c_ulonglong * 18)()
    dims = (C.c_longlong * 3)()
    assert L.dofs_debug_ws_ptrs(ctx.ctx, ptrs, dims) == 0
    cur_p, ptop_p, ll_p, in_p, ready_p, ord_p, lite_p, ctr_p, rv_p, pre_p, ctl_p, bw_p = [int(x) for x in ptrs][:12]
    Bd, N, NL = int(dims[0]), int(dims[1]), int(dims[2])
    ctl = d2h(ctl_p, 0, 4 * 8 * 64, np.int32)
    qh, qt = int(ctl[2 * 64]), int(ctl[3 * 64])
    print(f"ctl: long_next {ctl[0]} short_next {ctl[64]} qhead {qh} qtail {qt} err {ctl[4 * 64]} "
          f"ldone {ctl[5 * 64]} nl {ctl[7 * 64]} nt {ctl[7 * 64 + 1]} ns {ctl[7 * 64 + 2]} nlpool {ctl[7 * 64 + 4]}")
    if qt > 0:
        slots = d2h(bw_p, 0, 8 * min(qt + 8, Bd * N), np.uint64)
        print("queue slots (epoch, task):", [(int(v >> np.uint64(32)), int(v & np.uint64(0xFFFFFFFF))) for v in slots][-12:])
    cur = d2h(cur_p, 0, 4 * Bd * N, np.int32).reshape(Bd, N)
    ptop = d2h(ptop_p, 0, 4 * Bd * N, np.int32).reshape(Bd, N)
    shown = 0
    for f in range(Bd):
        npaths = int(c[f, 0])
        ready = d2h(ready_p, 32 * f * NL, 32 * NL - 24, np.int32)[::8]  # state words: one per 32-byte record
        # a path is complete once its top's state word says so (a completed path leaves its cursor as it was)
        inc = np.flatnonzero(ready[ptop[f, :npaths]] != 0x7FFFFFF0)  # kFlowDone (dofs_dataflow.h)
        if len(inc) == 0:
            continue
        print(f"frame {f}: {len(inc)} incomplete paths of {npaths}; long {int(c[f, 7])} rootl {int(c[f, 59])}")
        tops = {int(t): j for j, t in enumerate(ptop[f, :npaths])}
        for j in inc[:6]:
            q, top = int(cur[f, j]), int(ptop[f, j])
            rec = d2h(in_p, 16 * (f * NL + q), 16, np.uint8)  # StepIn (16 B): hs = size(h) | flags << 26, lt, wb
            hs = int(rec[0:4].view(np.uint32)[0])
            meta = hs >> 26
            lb = q + 2 * (hs & ((1 << 26) - 1)) if meta & 4 else int(rec[4:8].view(np.int32)[0])
            line = f"  path {j}: top {top} cursor {q} len {q - top + 1} meta {meta}"
            if meta & 4:
                st = int(d2h(ready_p, 32 * (f * NL + lb), 4, np.int32)[0])
                x = int(d2h(ord_p, 4 * (f * NL + lb), 4, np.int32)[0])
                lite = int(d2h(lite_p, f * NL + x, 1, np.uint8)[0])
                jj = tops.get(lb, -1)
                line += (f" | light child at {lb}: state {st:#x} node {x} lite {lite} path {jj}"
                         f" (its cursor {int(cur[f, jj]) if jj >= 0 else None})")
            print(line)
        shown += 1
        if shown >= 4:
            break
    break
ctx.close()
