"""The two KRT modes on one synthetic 1080p batch (DOFS_KRT_DNC=1 top-down global depths, =0 sweep):
per-frame events, path counters and the replay's error flag must agree. usage: python tools/krt_dnc_check.py B"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
H, W = int(os.environ.get("H", 1080)), int(os.environ.get("W", 1920))
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)
torch.cuda.synchronize()
res = {}
for mode in ("1", "0"):
    os.environ["DOFS_KRT_DNC"] = mode
    ctx = runtime.Dofs(0, keep_events=True)
    ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
    torch.cuda.synchronize()
    c = ctx.batch_counters(B)
    ev = {f: ctx.events(f).copy() for f in (0, B // 2, B - 1)}
    res[mode] = (c, ev)
    print(f"mode {mode}: flowerr {int(c[0, 58])} paths {int(c[:, 0].sum())} long {int(c[:, 7].sum())} "
          f"short {int(c[:, 6].sum())} tiny {int(c[:, 15].sum())}", flush=True)
    ctx.close()
c1, e1 = res["1"]
c0, e0 = res["0"]
for f in e1:
    same = all(np.array_equal(e1[f][n], e0[f][n]) for n in e1[f].dtype.names)
    print(f"frame {f}: events equal {same}")
print("path counters equal", bool(np.array_equal(c1[:, [0, 6, 7, 15]], c0[:, [0, 6, 7, 15]])))
