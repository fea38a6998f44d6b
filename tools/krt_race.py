"""Which stage differs when the DNC KRT's first batch goes wrong: runs one synthetic 1080p batch with
DOFS_KRT_DNC=1 in a fresh context, then the same batch with the sweep (DOFS_KRT_DNC=0) in a second
context, and compares the KRT outputs (final children lu / lv, node sizes, children sizes, heavy side)
and the preorder outputs (pre, ord, path-top flags, leaf scan) frame by frame.
usage: python tools/krt_race.py B [tries]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H, W = 1080, 1920
path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln) if False else None
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)
torch.cuda.synchronize()
path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
hip = C.CDLL(path)
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]


def grab(ctx):
    L = ctx.lib
    L.dofs_debug_ws_ptrs.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.POINTER(C.c_longlong)]
    ptrs = (C.c_ulonglong * 18)()
    dims = (C.c_longlong * 3)()
    assert L.dofs_debug_ws_ptrs(ctx.ctx, ptrs, dims) == 0
    Bd, N, NL = int(dims[0]), int(dims[1]), int(dims[2])
    M = N - 1
    spec = {"lu": (12, 4 * Bd * M, np.int32), "lv": (13, 4 * Bd * M, np.int32), "SZ": (14, 4 * Bd * NL, np.int32),
            "hls": (15, 8 * Bd * M, np.uint64), "hlB": (16, Bd * M, np.uint8), "pre": (9, 4 * Bd * NL, np.int32),
            "ord": (5, 4 * Bd * NL, np.int32), "lite": (6, Bd * NL, np.uint8), "lscan": (17, 4 * Bd * NL, np.int32)}
    out = {}
    for k, (i, nb, dt) in spec.items():
        a = np.empty(nb // np.dtype(dt).itemsize, dt)
        assert hip.hipMemcpy(a.ctypes.data, C.c_void_p(int(ptrs[i])), nb, 2) == 0
        out[k] = a
    c = ctx.batch_counters(B)
    return out, c, (Bd, N, NL)


os.environ["DOFS_KRT_DNC"] = "1"
ctx = runtime.Dofs(0, keep_events=True)  # the graph arrays stay readable after the batch
ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
torch.cuda.synchronize()
a, ca, dims = grab(ctx)
print("dnc: flowerr", int(ca[0, 58]), flush=True)
ctx.close()
os.environ["DOFS_KRT_DNC"] = "0"
ctx = runtime.Dofs(0, keep_events=True)  # the graph arrays stay readable after the batch
ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
torch.cuda.synchronize()
b, cb, _ = grab(ctx)
ctx.close()
Bd, N, NL = dims
M = N - 1
for k in a:
    n = len(a[k]) // Bd
    x, y = a[k].reshape(Bd, n), b[k].reshape(Bd, n)
    if k in ("lite", "pre"):  # a leaf's flag and position are never written (never read either)
        x, y = x[:, N:], y[:, N:]
    bad = [(f, int((x[f] != y[f]).sum()), int(np.flatnonzero(x[f] != y[f])[0])) for f in range(Bd) if (x[f] != y[f]).any()]
    print(k, "differs in frames (frame, count, first index):", bad[:6])
# the first differing node sizes of the first differing frame, with their children and the children's sizes
sa, sb = a["SZ"].reshape(Bd, NL), b["SZ"].reshape(Bd, NL)
lu, lv = a["lu"].reshape(Bd, M), a["lv"].reshape(Bd, M)
for f in range(Bd):
    idx = np.flatnonzero(sa[f] != sb[f])
    if len(idx) == 0:
        continue
    print(f"frame {f}: node sizes differ at merges {[int(i - N) for i in idx[:24]]}")
    for x in idx[:6]:
        j = int(x - N)
        ca, cb2 = int(lu[f, j]), int(lv[f, j])
        print(f"  merge {j} (block {j // 4096}, offset {j % 4096}): size dnc {int(sa[f, x])} sweep {int(sb[f, x])}; children "
              f"{ca} (size {int(sa[f, ca])}/{int(sb[f, ca])}) {cb2} (size {int(sa[f, cb2])}/{int(sb[f, cb2])})")
    break
