"""BASELINE config 5: one 3840x2160 synthetic frame tiled across N GPUs by row bands (intra-frame
shard of the MST stage, denseopticalflowsegmentation3d_amd/bands.py), beside the same frame on one GPU.

  python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 tools/bench_intraframe.py
Prints one JSON line on rank 0 (frames/s and Mpix/s of the sharded path, and of the 1-GPU path).

  python tools/bench_intraframe.py --model 4
One GPU: the expected N-GPU time of the sharded path from measured parts — the slowest band's
minimum spanning forest (dofs_band_msf_device, each band timed alone), the gather of band forests and
flow rows over xGMI (bytes / link bandwidth), and rank 0's masked whole-frame path
(dofs_segment_masked_device) with its stage times — next to the single-GPU path. The ceiling is
rank 0's part: the KRT sweep and the replay chains are sequential in merge order and do not shard.
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


def model(a):
    """Projected N-GPU time of the row-band path from single-GPU measurements of its parts."""
    from denseopticalflowsegmentation3d_amd.bands import add_cut_edges, blur_radius, halo_bounds, split_gain_ms
    H, W, n = a.height, a.width, a.model
    ctx = runtime.Dofs(0)
    persp, inv, up = runtime.calib()
    prm = default_params()
    sh = torch.cuda.current_stream().cuda_stream
    full = torch.empty((1, H, W, 2), dtype=torch.float32, device="cuda")
    runtime.synth_flow_device(full.data_ptr(), 1, H, W, seed0=0, stream=sh)
    R = blur_radius(prm)
    bounds = [band_bounds(H, n, r) for r in range(n)]
    masks = [torch.zeros((b1 - b0, W), dtype=torch.uint8, device="cuda") for b0, b1 in bounds]

    def timeit(fn, reps):
        for _ in range(a.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    band_ms = []
    for (b0, b1), m in zip(bounds, masks):
        h0, h1 = halo_bounds(H, b0, b1, R)
        rows = full[0, h0:h1].contiguous()
        band_ms.append(1e3 * timeit(lambda: ctx.band_msf_device(rows.data_ptr(), h0, h1 - h0, H, W, b0, b1,
                                                               m.data_ptr(), params=prm, stream=sh), a.steps))
    allowed = torch.cat(masks)
    add_cut_edges(allowed, bounds, prm.neighbor == 8)
    rec = torch.empty(4 + 64 * 96, dtype=torch.uint8, device="cuda")

    def masked():
        ctx.segment_masked_device(full.data_ptr(), H, W, allowed.data_ptr(), persp, inv, up, params=prm, stream=sh)
        ctx.records_copy(rec.data_ptr(), 64, stream=sh)

    def one():
        ctx.segment_batch_device(full.data_ptr(), 1, H, W, persp, inv, up, params=prm, stream=sh)
        ctx.records_copy(rec.data_ptr(), 64, stream=sh)

    t_masked = 1e3 * timeit(masked, a.steps)
    t_one = 1e3 * timeit(one, a.steps)
    ctx.profile(True)
    masked()
    torch.cuda.synchronize()
    ms, nb = ctx.profile_read()
    ctx.profile(False)
    per_band = max(b1 - b0 for b0, b1 in bounds)
    gather_bytes = (n - 1) * per_band * W * (1 + 8)  # edge-bit mask + flow rows of every other band
    t_gather = 1e3 * gather_bytes / (a.xgmi_gbs * 1e9)
    t_n = max(band_ms) + t_gather + t_masked
    # the policy IntraFrame(split="auto") takes for this shape (the frame resident on rank 0, as here): the
    # split only where its cost model says it saves time, else the frame on rank 0 alone (= one GPU)
    split = split_gain_ms(H, W, n, a.xgmi_gbs, resident=True) > 0
    t_pol = t_n if split else t_one
    # the single-frame latency floor: the replay's dependency chain (profiles/r05/critical_path_4k_emu.json:
    # 1,536,516 merges at 4K, seed 1) at the measured 21.5 ns per long-path step — no split shortens it
    floor = 1536516 * 21.5e-6 if (H, W) == (2160, 3840) else None
    print(json.dumps({"config": f"{W}x{H} synthetic, {n} row bands, projected from one GPU",
                      "band_msf_ms": [round(x, 3) for x in band_ms], "gather_ms_est": round(t_gather, 3),
                      "gather_bytes": gather_bytes, "xgmi_gbs_assumed": a.xgmi_gbs,
                      "rank0_masked_ms": round(t_masked, 3),
                      "rank0_stage_ms": {k: round(v / max(nb, 1), 3) for k, v in ms.items()},
                      "split_model_gain_ms": round(split_gain_ms(H, W, n, a.xgmi_gbs, resident=True), 3),
                      "policy": "split" if split else "replica (rank 0 alone)",
                      "projected_ms_per_frame_split": round(t_n, 3), "projected_speedup_split": round(t_one / t_n, 3),
                      "projected_ms_per_frame": round(t_pol, 3), "one_gpu_ms_per_frame": round(t_one, 3),
                      "projected_speedup": round(t_one / t_pol, 3),
                      "latency_floor_ms": round(floor, 1) if floor else None,
                      "latency_floor": "the replay's dependency chain, 1,536,516 merges x 21.5 ns (one 4K frame)"}),
          flush=True)
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", type=int, default=0, help="one GPU: project the N-band sharded time (N = value)")
    ap.add_argument("--xgmi-gbs", type=float, default=64.0, help="assumed gather bandwidth to rank 0 (GB/s)")
    ap.add_argument("--split", default="auto", help="row-band split: auto (IntraFrame's cost model), 1 or 0")
    a = ap.parse_args()
    if a.model:
        return model(a)
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
    rec = torch.empty(4 + 64 * 96, dtype=torch.uint8, device="cuda")
    shard = IntraFrame(ctx, world, rank, prm, split=a.split if a.split == "auto" else a.split == "1",
                       xgmi_gbs=a.xgmi_gbs)

    def step():  # (the frame is resident on every rank here: rank 0 passes it, so "auto" may skip the split)
        bid = shard.step(band, H, W, persp, inv, up, stream=sh, frame=full[0] if rank == 0 else None)
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
                          "split": bool(shard.did_split),
                          "frames_per_sec": round(1 / t_shard, 3), "mpix_per_sec": round(H * W / t_shard / 1e6, 3),
                          "ms_per_frame": round(t_shard * 1e3, 3), "one_gpu_ms_per_frame": round(t_one * 1e3, 3),
                          "n_gpus": world}), flush=True)
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
