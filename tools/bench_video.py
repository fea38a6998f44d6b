"""Throughput of the stages around the path at 1080p, one GPU:
  flow     dofs_farneback_batch_device on B frame pairs (Mpixels/s of flow output)
  overlay  dofs_overlay_batch_device on one segmented batch of B frames
  clip     dofs_video_clip_device: main1's loop (gray -> Farneback -> segment -> overlay) over a
           device-resident clip of n frames (frames/s over n - 1 pairs)
Synthetic clip (video.synth_clip upscaled to 1080p); inputs resident in HBM before timing; device
events on the caller's stream. Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from denseopticalflowsegmentation3d_amd import runtime, video  # noqa: E402
from denseopticalflowsegmentation3d_amd.abi import default_params  # noqa: E402


def timed(fn, reps, stream):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--frames", type=int, default=65, help="clip length (pairs = frames - 1)")
    ap.add_argument("--batch", type=int, default=16, help="pairs per chunk")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    H, W, n, B = a.height, a.width, a.frames, a.batch
    N = H * W
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    ctx = runtime.Dofs(0)
    persp, inv, up = runtime.calib()
    prm = default_params()
    clip = torch.from_numpy(video.synth_clip(n, H, W)).to(dev)
    gray = torch.empty((n, H, W), dtype=torch.uint8, device=dev)
    runtime.bgr_to_gray_device(clip.data_ptr(), n * N, gray.data_ptr(), stream=sh)
    flow = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    out = {"config": {"H": H, "W": W, "frames": n, "batch": B, "data": "synthetic clip (video.synth_clip)"}}

    def fb():
        ctx.farneback_batch_device(gray.data_ptr(), gray[1:].data_ptr(), B, H, W, flow.data_ptr(), stream=sh)
    fb()
    ms = timed(fb, a.reps, stream)
    out["flow"] = {"ms_per_batch": round(ms, 3), "Mpixels_per_s": round(B * N / ms / 1e3, 1)}

    bid = ctx.segment_batch_device(flow.data_ptr(), B, H, W, persp, inv, up, params=prm, stream=sh)
    ov = torch.empty((B, H, W, 3), dtype=torch.uint8, device=dev)

    def ovl():
        ctx.overlay_batch_device(bid, clip[1:].data_ptr(), ov.data_ptr(), stream=sh)
    ovl()
    ms = timed(ovl, a.reps, stream)
    out["overlay"] = {"ms_per_batch": round(ms, 3), "Mpixels_per_s": round(B * N / ms / 1e3, 1),
                      "GB_per_s_alg": round(B * N * 18 / ms / 1e6, 1)}

    ovc = torch.empty((n - 1, H, W, 3), dtype=torch.uint8, device=dev)
    cnt = torch.empty((n - 1,), dtype=torch.int32, device=dev)

    def clipfn():
        ctx.video_clip_device(clip.data_ptr(), n, H, W, persp, inv, up, batch=B, d_overlay=ovc.data_ptr(),
                              d_counts=cnt.data_ptr(), params=prm, stream=sh)
    clipfn()
    t0 = time.perf_counter()
    ms = timed(clipfn, a.reps, stream)
    out["clip"] = {"ms_per_clip": round(ms, 3), "frames_per_s": round((n - 1) / ms * 1e3, 2),
                   "Mpixels_per_s": round((n - 1) * N / ms / 1e3, 1),
                   "wall_s": round(time.perf_counter() - t0, 3),
                   "snapshots_last": int(cnt[-1].item())}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
