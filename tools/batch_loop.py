"""Measurement helper: K synthetic 1080p batches of B frames through one context, nothing else (no checks, no
timing of its own) — the program to run under `rocprofv3 --kernel-trace --stats` with a measurement library
(DOFS_LIB=.../_build/measure/libdofs_hip.so, DOFS_SKIPMASK, DOFS_SERIAL=1) for per-kernel times.
usage: python tools/batch_loop.py [B] [K]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 112
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
H, W = 1080, 1920
ctx = runtime.Dofs(0)
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)
torch.cuda.synchronize()
ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)  # (first batch: allocation)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / K
print(f"batches {K} of {B}: {ms:.2f} ms per batch, {B * H * W / ms / 1e3:.1f} Mpixels/s")
ctx.close()
