"""Anatomy of the dataflow replay launch (dofs_dataflow.h, FlowStat): runs batches of synthetic 1080p
frames serially (DOFS_SERIAL=1 recommended) and prints the last launch's timeline and task counts.
usage: DOFS_SERIAL=1 python tools/flow_stats.py [B] [batches]"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 96
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 2
H, W = int(os.environ.get("H", 1080)), int(os.environ.get("W", 1920))
ctx = runtime.Dofs(0, lib=os.environ.get("DOFS_LIB") or None)  # DOFS_LIB: another build, for A/B
L = ctx.lib
L.dofs_debug_flow_stats.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
persp, inv, up = runtime.calib()
dev = torch.device("cuda", 0)
flows = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
sh = torch.cuda.current_stream(dev).cuda_stream
runtime.synth_flow_device(flows.data_ptr(), B, H, W, 0, stream=sh)
names = ["t0", "t_short_done", "t_long_last", "t_exit", "long_runs", "long_parks", "long_chunks", "pushes", "injects",
         "long_done", "long_ticks", "short_rounds", "short_ticks", "long_steps", "t_root", "root_parks", "root_steps", "root_chunks", "p_steps", "p_tail", "p_next", "kfast_chunks", "restarts", "p_cwait", "p_hwait"]
for b in range(NB):
    ctx.segment_batch_device(flows.data_ptr(), B, H, W, persp, inv, up, stream=sh)
    torch.cuda.synchronize()
    out = (C.c_ulonglong * 28)()
    L.dofs_debug_flow_stats(ctx.ctx, out, 28)
    v = {n: int(out[i]) for i, n in enumerate(names)}
    t0 = v["t0"]
    res = {"ms_last_short_worker_done": (v["t_short_done"] - t0) / 1e5, "ms_last_long_done": (v["t_long_last"] - t0) / 1e5,
           "ms_last_exit": (v["t_exit"] - t0) / 1e5, "ms_last_root_done": (v["t_root"] - t0) / 1e5, "wave_ms_in_long": v["long_ticks"] / 1e5,
           "wave_ms_in_short": v["short_ticks"] / 1e5,
           "prof_ms": {k: v[k] / 1e5 for k in ("p_steps", "p_tail", "p_next", "p_cwait", "p_hwait")}}
    res.update({k: v[k] for k in ("long_runs", "long_parks", "long_chunks", "pushes", "injects", "long_done",
                                  "short_rounds", "long_steps", "root_parks", "root_steps", "root_chunks", "kfast_chunks",
                                  "restarts")})
    print(json.dumps(res), flush=True)
ctr = ctx.batch_counters(B)
print(json.dumps({"paths": int(ctr[:, 0].sum()), "long": int(ctr[:, 7].sum()), "short": int(ctr[:, 6].sum()),
                  "tiny": int(ctr[:, 15].sum()), "long_merges": int(ctr[:, 57].sum()), "flow_err": int(ctr[0, 58])}))
ctx.close()
