"""Per-frame pipeline counters of one synthetic 1080p batch (dofs_batch_counters; dofs_common.h Counter).

Heavy paths: tiny (<= kTinyPath merges, round 0's first replay list), short (the rest of the
per-lane list) and long (the wave-per-path replay); tiny + short + long = paths.
usage: python tools/counters.py [B]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

C_PATHS, C_CAND, C_SHORT, C_LONG, C_TINY, C_ACT = 0, 1, 6, 7, 15, 16
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H, W = 1080, 1920
ctx = runtime.Dofs(0)
persp, inv, up = runtime.calib()
fl = torch.empty((B, H, W, 2), dtype=torch.float32, device="cuda")
runtime.synth_flow_device(fl.data_ptr(), B, H, W, 0)
ctx.segment_batch_device(fl.data_ptr(), B, H, W, persp, inv, up)
c = ctx.batch_counters(B)
print("paths", c[:, C_PATHS].tolist())
print("tiny", c[:, C_TINY].tolist())
print("short", c[:, C_SHORT].tolist())
print("long", c[:, C_LONG].tolist())
print("tiny+short+long == paths", bool(((c[:, C_TINY] + c[:, C_SHORT] + c[:, C_LONG]) == c[:, C_PATHS]).all()))
print("cand", c[:, C_CAND].tolist())
print("borůvka rounds", (c[:, C_ACT:C_ACT + 24] != 0).sum(1).tolist())
ctx.close()
