"""Determinism stress of the batch path on the GPU (no oracle): the fixed-job split of
tests/test_gpu_bench_config.py (180x320, three simulated ranks, chunks of 8 and 6 frames through
frames.Pipelined over one keep_events context), repeated; between repetitions a larger batch re-lays out the
workspaces (as the GPU suite's earlier tests do). Every repetition's gathered records must equal the first's
byte for byte. Prints one line per repetition and the number that differed.
usage: python tools/stress_determinism.py [reps] [lib] [keep]   (keep 0: a default context, whose stage B reuses
stage A's dead arrays; 1, the default: keep_events, whose layout keeps the graph)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402
from denseopticalflowsegmentation3d_amd.abi import default_params  # noqa: E402
from denseopticalflowsegmentation3d_amd.frames import FrameParallel, Pipelined, decode_records, job_plan  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
LIB = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] not in ("", "-") else None
KEEP = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
H, W, F, WORLD, BATCH, PER = 180, 320, 40, 3, 8, 64
ctx = runtime.Dofs(0, lib=LIB, keep_events=KEEP)
persp, inv, up = runtime.calib()
prm = default_params()
prm.min_size = 300
dev = torch.device("cuda", 0)
sh = torch.cuda.current_stream(dev).cuda_stream
big = torch.empty((12, 540, 960, 2), dtype=torch.float32, device=dev)
runtime.synth_flow_device(big.data_ptr(), 12, 540, 960, 7, stream=sh)


def one():
    out = []
    for rank in range(WORLD):
        mine, chunks = job_plan(F, rank, WORLD, BATCH)
        flows = torch.empty((max(len(mine), 1), H, W, 2), dtype=torch.float32, device=dev)
        runtime.synth_flow_device(flows.data_ptr(), max(len(mine), 1), H, W, seed0=mine.start, stream=sh)
        blocks = {}
        pipe = Pipelined(FrameParallel(ctx, 1, PER), persp, inv, up, params=prm, stream=sh,
                         sink=lambda bid, g: blocks.__setitem__(bid, g.cpu().numpy()))
        ids = pipe.run_chunks(flows, chunks)
        pipe.flush()
        torch.cuda.synchronize()
        for (_, n), b in zip(chunks, ids):  # the valid records of each frame (the rest of a block is padding)
            buf = blocks[b]
            counts = buf[:4 * n].view(np.int32)
            recs = decode_records(buf, n, PER)
            out.append([(int(counts[f]), recs[f][:int(counts[f])].tobytes()) for f in range(n)])
    return out


ref = None
bad = 0
for r in range(REPS):
    if r % 2 == 1:  # re-lay out the workspaces with a larger shape in between
        ctx.segment_batch_device(big.data_ptr(), 12, 540, 960, persp, inv, up, stream=sh)
        torch.cuda.synchronize()
    got = one()
    if ref is None:
        ref = got
        print(f"rep {r}: reference", flush=True)
        continue
    diff = [i for i, (a, b) in enumerate(zip(ref, got)) if a != b]
    bad += 1 if diff else 0
    print(f"rep {r}: {'differs in chunks ' + str(diff) if diff else 'equal'}", flush=True)
ctx.close()
print(f"differed {bad} of {REPS - 1}")
sys.exit(1 if bad else 0)
