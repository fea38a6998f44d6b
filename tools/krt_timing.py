"""KRT phase anatomy from a measurement build (-DDOFS_KRT_TIMING, exports dofs_debug_krt_timing):
runs batches of synthetic 1080p frames and prints the wall time per phase, summed over workgroups and
per 4096-merge block. usage: DOFS_LIB=denseopticalflowsegmentation3d_amd/_build/krt/libdofs_hip.so python tools/krt_timing.py [B] [batches]
(the measurement build: make -C denseopticalflowsegmentation3d_amd/csrc krt)"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 96
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 3
H, W = 1080, 1920
ctx = runtime.Dofs(0)
L = ctx.lib
L.dofs_debug_krt_timing.argtypes = [C.POINTER(C.c_double), C.c_int]
persp, inv, up = runtime.calib()
dev = torch.device("cuda", 0)
flows = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
sh = torch.cuda.current_stream(dev).cuda_stream
runtime.synth_flow_device(flows.data_ptr(), B, H, W, 0, stream=sh)
ctx.segment_batch_device(flows.data_ptr(), B, H, W, persp, inv, up, stream=sh)
torch.cuda.synchronize()
out = (C.c_double * 20)()
L.dofs_debug_krt_timing(out, 20)
for _ in range(NB):
    ctx.segment_batch_device(flows.data_ptr(), B, H, W, persp, inv, up, stream=sh)
torch.cuda.synchronize()
ctx.records_device()
L.dofs_debug_krt_timing(out, 20)
blocks = NB * B * ((H * W - 1 + 4095) // 4096)
names = ["sweep A finds", "sweep B root hash", "sweep C R-half unions + sizes", "sweep D stores", "sweep C L-half unions + top level", "top level",
         "deep block 1", "deep block 2", "parent epilogue", "deep depths S>=256", "deep depths S<256",
         "LDS worker wait"]
res = {n: {"total_ms": round(out[i] / 1e3, 2), "us_per_block": round(out[i] / blocks, 2)}
       for i, n in enumerate(names)}
hops = {"phase A find rounds (slowest thread) per sweep block": round(out[12] * 100 / max(out[13] * 100, 1), 2)}
# the preorder sweep (k_pre_sweep, one workgroup per frame, the same 4096-merge blocks)
pre_names = {14: "pre: tops' pushed positions (load, LDS)", 15: "pre: positions + pushes (issue)",
             16: "pre: store drain (block barrier)"}
res.update({n: {"total_ms": round(out[i] / 1e3, 2), "us_per_block": round(out[i] / blocks, 2)}
            for i, n in pre_names.items()})
print(json.dumps({"B": B, "batches": NB, "blocks": blocks, "phases": res, "sweep": hops}, indent=1))
