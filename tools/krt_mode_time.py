"""Per-batch wall time of synthetic 1080p batches, each synchronised, for the KRT mode in DOFS_KRT_DNC
(unset: auto). usage: python tools/krt_mode_time.py B [batches]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 4
H, W = 1080, 1920
ctx = runtime.Dofs(0)
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)
torch.cuda.synchronize()
ts = []
prof = bool(os.environ.get("PROF"))
for b in range(NB):
    if prof:
        ctx.profile(True)
    t0 = time.perf_counter()
    ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
    ctx.fetch(0, want_blur=False)
    torch.cuda.synchronize()
    ts.append(round((time.perf_counter() - t0) * 1e3, 2))
    st = ""
    if prof:
        ms, nb = ctx.profile_read()
        ctx.profile(False)
        st = " " + " ".join(f"{k}={v:.1f}" for k, v in ms.items())
    c = ctx.batch_counters(B)
    import ctypes as C
    ctx.lib.dofs_debug_flow_stats.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
    fs = (C.c_ulonglong * 16)()
    ctx.lib.dofs_debug_flow_stats(ctx.ctx, fs, 16)
    flow = f" flowerr={int(c[0, 58])} short_done={(fs[1] - fs[0]) / 1e5:.1f} long_last={(fs[2] - fs[0]) / 1e5:.1f} exit={(fs[3] - fs[0]) / 1e5:.1f}"
    print(f"B={B} mode={os.environ.get('DOFS_KRT_DNC', 'auto')} batch {b}: {ts[-1]} ms{st}{flow}", flush=True)
ctx.close()
