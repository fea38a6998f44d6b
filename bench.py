"""Benchmark: Mpixels/s of segment + lifting_3d on synthetic 1080p flow fields (BASELINE.json metric).

One step = one batch of `--batch` synthetic 1920x1080 flow fields per GPU pushed through the whole
HIP path (blur → MST → Kruskal replay → per-merge filters + 3D lifting → snapshots → labels), then
the fixed-size 3D-box records of every frame gathered to all ranks (RCCL all_gather over xGMI when
N > 1). Inputs are generated on device before timing (resident in HBM); frames are independent, so
ranks shard frames with no data-path collective besides the box gather ("scaling": "weak").

Usage: python bench.py [--gpus N --steps K --warmup W --batch B]
       (N > 1 under torch.distributed.run, one process per GPU)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime  # noqa: E402
from denseopticalflowsegmentation3d_amd.abi import default_params  # noqa: E402
from denseopticalflowsegmentation3d_amd.frames import FrameParallel  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
GATHER_PER_FRAME = 64  # box records per frame in the gathered block
DEEP_BLOCK = int(os.environ.get("DOFS_DEEP_S", "4096"))  # KRT depths with block size <= this run in LDS (k_dnc_deep), the rest globally

# Algorithmic (compulsory) bytes of the probed kernels:
#   k_boruvka_min, per pixel of a frame still active in that Borůvka pass:
#     pass 0: its component label (4 B) and blurred flow (8 B) read once, its kept incident-minimum
#             candidate (weight 8 B + index 4 B) written once = 24 B (neighbours' words are other
#             pixels' own reads; the per-component minima are LDS-aggregated per tile);
#     pass 1: its label (4 B) and kept candidate (12 B) read once = 16 B.
#   k_dnc_compress (DOFS_KRT_DNC=1 only), per L edge of a depth: own label 4 B, parent 4 B, size 4 B,
#     component size RMW 8 B, max rank RMW 8 B.
KERNEL_BYTES = {"k_boruvka_min": (24, 16), "KDncCompress": 28, "k_dnc_compress": 28}
ROOF_KERNEL = "k_boruvka_min"
ROUND_FLAG = 16  # counters: C_ACT + r = Borůvka round r found a cross-component edge


def boruvka_min_bytes(counters, N):
    """Algorithmic bytes per batch of k_boruvka_min and its launches: round r >= 1 runs pass 0 for
    frames whose round r - 1 found an edge and pass 1 for frames whose round r found one
    (dofs_pipeline.h boruvka())."""
    R = min(ceil_log2(N) + 2, 40 - 1)
    act = counters[:, ROUND_FLAG:ROUND_FLAG + R] != 0
    b0, b1 = KERNEL_BYTES["k_boruvka_min"]
    return int(act[:, 0:R - 1].sum()) * N * b0 + int(act[:, 1:R].sum()) * N * b1, 2 * (R - 1)


def ceil_log2(n):
    k = 0
    while (1 << k) < n:
        k += 1
    return k


def dnc_L_edges(M):
    """L edges (lanes doing work) of every global KRT depth launch: block size S > DEEP_BLOCK."""
    out = []
    S = 1 << ceil_log2(M)
    while S > DEEP_BLOCK:
        h, n = S // 2, 0
        for s0 in range(0, M, S):
            if s0 + h < M:
                n += h
        out.append(n)
        S //= 2
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=96, help="frames per GPU per step")
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--cpu-frames", type=int, default=1, help="frames of the CPU baseline sample (0 = skip)")
    ap.add_argument("--no-stages", action="store_true", help="skip the per-stage event timing pass")
    ap.add_argument("--probe", default=ROOF_KERNEL, help="kernel timed with device events for the roofline")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r01", "pmc_summary.json"),
                    help="PMC summary JSON (tools/pmc_summary.py) for roofline.traffic")
    return ap.parse_args()


def cpu_baseline(H, W, frames):
    """Reference-faithful CPU restatement (oracle mode 1: std::multiset / std::set structures, -O2,
    one thread) on a bounded sample of the same workload."""
    from oracle import binding as ob
    persp, inv, up = ob.calib()
    total = 0.0
    for s in range(frames):
        flow = ob.synth_flow(H, W, s)
        t0 = time.perf_counter()
        ob.segment(flow, persp, inv, up, mode=1)
        total += time.perf_counter() - t0
    return {"value": round(frames * H * W / total / 1e6, 4), "unit": "Mpixels/sec", "cores": 1, "kind": "port",
            "sample": f"{frames} synthetic {W}x{H} frame(s) (seed 0..{frames - 1}), faithful mode "
                      f"(std::multiset edge sort + std::set unions + set-copy snapshots), g++ -O2, "
                      f"{total:.1f} s"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B, H, W = a.batch, a.height, a.width
    N = H * W

    ctx = runtime.Dofs(local)
    persp, inv, up = runtime.calib()
    prm = default_params()
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    flows = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    runtime.synth_flow_device(flows.data_ptr(), B, H, W, seed0=rank * B, stream=sh)
    fp = FrameParallel(ctx, world, GATHER_PER_FRAME)
    pending = []
    lag = ctx.batch_slots() - 1

    # one step = submit a batch, then gather the records of the batch submitted `lag` steps before
    # (the context overlaps earlier batches' replay stages with this batch's graph stage); flush()
    # gathers the rest.
    def step():
        pending.append(fp.submit(flows, persp, inv, up, params=prm, stream=sh))
        if len(pending) > lag:
            fp.collect(pending.pop(0), stream=sh)

    def flush():
        while pending:
            fp.collect(pending.pop(0), stream=sh)

    for _ in range(a.warmup):
        step()
    flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ctx.probe(a.probe)
    ctx.probe_read()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        step()
    flush()
    e1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms_ev = e0.elapsed_time(e1)
    probe_ms, probe_n = ctx.probe_read()
    ctx.probe(None)
    t = torch.tensor([max(wall, ms_ev / 1e3)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    frames = world * B * a.steps
    value = frames * N / elapsed / 1e6

    # roofline of the probed kernel: algorithmic bytes of its launches in the timed region over their
    # device-event time (events recorded on the stream the kernel runs on)
    roof = None
    probe = None
    if probe_n and a.probe not in KERNEL_BYTES:  # a kernel without a roofline model: its time only
        probe = {"kernel": a.probe, "ms_per_batch": round(probe_ms / a.steps, 3),
                 "launches_per_batch": probe_n / a.steps}
    elif probe_n:
        if a.probe == "k_boruvka_min":
            alg_batch, launches_per_batch = boruvka_min_bytes(ctx.batch_counters(B), N)
        else:
            per_launch = [n * B * KERNEL_BYTES[a.probe] for n in dnc_L_edges(N - 1)]
            launches_per_batch, alg_batch = len(per_launch), sum(per_launch)
        assert launches_per_batch and probe_n == launches_per_batch * a.steps, (probe_n, launches_per_batch)
        alg = alg_batch * a.steps
        achieved = alg / (probe_ms / 1e3) / 1e9
        traffic = None
        if a.pmc and os.path.exists(a.pmc):
            pm = json.load(open(a.pmc))
            if pm.get("kernel") == a.probe and pm.get("batch") == B:
                traffic = pm["hbm_bytes_per_launch"]
        roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
                "kernel": a.probe, "launches": probe_n, "avg_launch_us": round(probe_ms / probe_n * 1e3, 2),
                "alg_bytes_per_launch": round(alg / probe_n),
                "alg_bytes_per_unit": ("24 (pass 0) / 16 (pass 1) per active pixel" if a.probe == "k_boruvka_min"
                                       else KERNEL_BYTES[a.probe]),
                "path_input_roofline_frac": None}

    # per-stage device-event timing of extra profiled batches (not part of the timed region)
    stages = None
    if not a.no_stages:
        ctx.profile(True)
        for _ in range(max(2, a.steps // 2)):
            step()
        flush()
        torch.cuda.synchronize()
        ms, nb = ctx.profile_read()
        ctx.profile(False)
        stages = {k: round(v / nb, 3) for k, v in ms.items()}
    if roof is not None:  # the north star's whole-path figure: 8 B/px input read over the wall time
        roof["path_input_roofline_frac"] = round(B * a.steps * N * 8 / elapsed / 1e9 / HBM_PEAK_GBS, 8)

    if rank == 0:
        res = ctx.fetch(0, want_blur=False)
        out = {
            "metric": "Mpixels/sec segment+lifting_3d @1080p",
            "value": round(value, 3),
            "unit": "Mpixels/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+f64",
            "data": "synthetic (on-device splitmix64 flow fields, DESIGN.md §Synthetic input)",
            "config": {"workload": f"{W}x{H} synthetic flow, full segment + lifting_3d (BASELINE config 3 shape)",
                       "frames_per_gpu_per_step": B, "frames_per_sec": round(frames / elapsed, 3),
                       "parallelism": f"frame-parallel x{world}", "snapshots_frame0": int(len(res.snapshots)),
                       "candidates_frame0": int(res.stats["n_candidates"])},
            "roofline": roof,
            "stages_ms_per_batch": stages,
            "cpu_baseline": None,
        }
        if probe is not None:
            out["probe"] = probe
        if world == 1 and a.cpu_frames > 0:
            out["cpu_baseline"] = cpu_baseline(H, W, a.cpu_frames)
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
