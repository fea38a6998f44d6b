"""The replay's critical path of one frame: tools/critical_path.cpp over the frame's merge stream.

The merges come from the product library's per-merge events (a context with keep_events) on the GPU, or from
the test-only host emulator (--emu, CPU). Prints one JSON line per cost model: the KRT height (every step 1,
no wake-ups), and the dataflow replay's modelled time with the measured per-step costs of long paths
(c_long: p_steps / long steps, profiles/r04/anatomy) and assumed costs of short-path steps and wake-ups.

Usage: python tools/critical_path.py [--H 2160 --W 3840 --seed 1 --emu --long-path 256 ...]
"""
import argparse
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BIN = os.path.join(ROOT, "tools", "_build", "critical_path")


def build():
    src = os.path.join(ROOT, "tools", "critical_path.cpp")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < os.path.getmtime(src):
        os.makedirs(os.path.dirname(BIN), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-o", BIN, src], check=True)


def merges(H, W, seed, emu):
    from denseopticalflowsegmentation3d_amd import runtime
    lib = os.path.join(ROOT, "tests", "emu", "_build", "libdofs_emu.so") if emu else None
    ctx = runtime.Dofs(0, lib=lib, keep_events=True)
    try:
        persp, inv, up = runtime.calib()
        if emu:  # the emulator's "device" is the host: its synthetic field fills a host buffer
            flow = np.empty((H, W, 2), np.float32)
            runtime.synth_flow_device(flow.ctypes.data, 1, H, W, seed, lib=ctx.lib)
            ctx.segment(flow, persp, inv, up)
        else:
            import torch
            fl = torch.empty((1, H, W, 2), dtype=torch.float32, device="cuda")
            runtime.synth_flow_device(fl.data_ptr(), 1, H, W, seed)
            torch.cuda.synchronize()
            ctx.segment_batch_device(fl.data_ptr(), 1, H, W, persp, inv, up)
            torch.cuda.synchronize()
        ev = ctx.events(0)
        return np.ascontiguousarray(np.stack([ev["start"], ev["end"]], 1).astype(np.int32))
    finally:
        ctx.close()


def run(pairs, N, cl, cs, cw, lp):
    blob = np.int64(N).tobytes() + pairs.tobytes()
    r = subprocess.run([BIN, str(cl), str(cs), str(cw), str(lp)], input=blob, capture_output=True, check=True)
    return json.loads(r.stdout)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--emu", action="store_true")
    ap.add_argument("--c-long", type=float, default=21.5, help="ns per long-path step (profiles/r04/anatomy)")
    ap.add_argument("--c-short", type=float, default=1000.0, help="ns per short-path step (one lane, assumed)")
    ap.add_argument("--c-wake", type=float, default=5000.0, help="ns per wake-up of a parked path (assumed)")
    ap.add_argument("--long-path", default="256,64,16")
    a = ap.parse_args()
    build()
    pairs = merges(a.H, a.W, a.seed, a.emu)
    N = a.H * a.W
    out = {"frame": f"{a.W}x{a.H} seed {a.seed}", "unit": run(pairs, N, 1, 1, 0, 256)}
    for lp in (int(x) for x in a.long_path.split(",")):
        out[f"model_long_path_{lp}"] = run(pairs, N, a.c_long, a.c_short, a.c_wake, lp)
        out[f"model_long_path_{lp}_nowake"] = run(pairs, N, a.c_long, a.c_short, 0, lp)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
