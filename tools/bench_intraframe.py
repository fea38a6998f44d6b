"""BASELINE config 5: one 3840x2160 synthetic frame tiled across N GPUs by row bands (intra-frame
shard of the MST stage, denseopticalflowsegmentation3d_amd/bands.py), beside the same frame on one GPU.

  python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 tools/bench_intraframe.py
Prints one JSON line on rank 0 (frames/s and Mpix/s of the sharded path, and of the 1-GPU path).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402
from denseopticalflowsegmentation3d_amd.abi import default_params  # noqa: E402
from denseopticalflowsegmentation3d_amd.bands import IntraFrame, band_bounds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl" if world > 1 else "gloo", rank=rank, world_size=world,
                            init_method=None if world > 1 else "tcp://127.0.0.1:29581")
    H, W = a.height, a.width
    ctx = runtime.Dofs(local)
    persp, inv, up = runtime.calib()
    prm = default_params()
    sh = torch.cuda.current_stream().cuda_stream
    full = torch.empty((1, H, W, 2), dtype=torch.float32, device="cuda")
    runtime.synth_flow_device(full.data_ptr(), 1, H, W, seed0=0, stream=sh)
    r0, r1 = band_bounds(H, world, rank)
    band = full[0, r0:r1].contiguous()
    rec = torch.empty(4 + 64 * 88, dtype=torch.uint8, device="cuda")
    shard = IntraFrame(ctx, world, rank, prm)

    def step():
        bid = shard.step(band, H, W, persp, inv, up, stream=sh)
        if rank == 0:
            ctx.records_copy(rec.data_ptr(), 64, stream=sh, batch=bid)

    def timed(fn, n):
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        return (time.perf_counter() - t0) / n

    for _ in range(a.warmup):
        step()
    t_shard = timed(step, a.steps)
    t_one = None
    if rank == 0:  # the same frame through the single-GPU path
        def one():
            ctx.segment_batch_device(full.data_ptr(), 1, H, W, persp, inv, up, params=prm, stream=sh)
            ctx.records_copy(rec.data_ptr(), 64, stream=sh)
        for _ in range(a.warmup):
            one()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            one()
        torch.cuda.synchronize()
        t_one = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"config": f"{W}x{H} synthetic, row bands over {world} GPU(s), MST sharded",
                          "frames_per_sec": round(1 / t_shard, 3), "mpix_per_sec": round(H * W / t_shard / 1e6, 3),
                          "ms_per_frame": round(t_shard * 1e3, 3), "one_gpu_ms_per_frame": round(t_one * 1e3, 3),
                          "n_gpus": world}), flush=True)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
