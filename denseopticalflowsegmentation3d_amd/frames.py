"""Frame-parallel execution over the GPUs of one node (BASELINE config 4).

Frame pairs are independent (segment.cpp:209-269 carries only prev_frame), so ranks shard frames
with no data-path collective; the only exchange is one gather of fixed-size 3D-box records
(dofs_box_record) per batch — RCCL all_gather over xGMI under the "nccl" backend, gloo in the
CPU tests.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .abi import DofsBoxRecord

RECORD_DTYPE = DofsBoxRecord.np_dtype()


def frame_shard(total: int, rank: int, world: int) -> range:
    """Contiguous block of frames owned by `rank` (block size ceil(total / world))."""
    per = -(-total // world)
    lo = min(total, rank * per)
    return range(lo, min(total, lo + per))


def records_nbytes(frames: int, per_frame: int) -> int:
    """Layout written by dofs_batch_records_copy: int32 counts[frames], then frames × per_frame records."""
    return 4 * frames + frames * per_frame * RECORD_DTYPE.itemsize


def decode_records(buf: np.ndarray, frames: int, per_frame: int) -> list[np.ndarray]:
    """Per-frame arrays of valid box records from one rank's block."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    counts = buf[:4 * frames].view(np.int32)
    recs = buf[4 * frames:records_nbytes(frames, per_frame)].view(RECORD_DTYPE).reshape(frames, per_frame)
    return [recs[f, :min(int(counts[f]), per_frame)].copy() for f in range(frames)]


def gather_records(block: torch.Tensor, world: int) -> torch.Tensor:
    """All ranks' record blocks, rank-major (one collective)."""
    if world == 1:
        return block
    out = torch.empty(world * block.numel(), dtype=block.dtype, device=block.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, block)
    else:
        parts = list(out.chunk(world))
        dist.all_gather(parts, block)
        out = torch.cat(parts)
    return out


def decode_gathered(gathered: np.ndarray, world: int, frames_per_rank: int, per_frame: int) -> list[np.ndarray]:
    n = records_nbytes(frames_per_rank, per_frame)
    out: list[np.ndarray] = []
    for r in range(world):
        out.extend(decode_records(gathered[r * n:(r + 1) * n], frames_per_rank, per_frame))
    return out


class FrameParallel:
    """One rank's share of a frame-parallel job: segment device-resident batches, then gather the
    fixed-size box records of every frame to every rank.

    `submit` only enqueues; `collect(batch)` gathers a batch's records. Collecting batch k after
    submitting batch k + slots - 1 (ctx.batch_slots()) lets the context overlap k's replay stage
    with the following batches' graph stages."""

    def __init__(self, ctx, world: int = 1, per_frame: int = 64):
        self.ctx, self.world, self.per_frame = ctx, world, per_frame
        self.block = None
        self.frames = {}

    def submit(self, flows: torch.Tensor, persp, inv, inv_upper, params=None, stream: int | None = None) -> int:
        B, H, W = flows.shape[:3]
        bid = self.ctx.segment_batch_device(flows.data_ptr(), B, H, W, persp, inv, inv_upper, params=params,
                                            stream=stream)
        keep = self.ctx.batch_slots() if hasattr(self.ctx, "batch_slots") else 2
        self.frames = {k: v for k, v in self.frames.items() if k > bid - keep}
        self.frames[bid] = (B, flows.device)
        return bid

    def collect(self, bid: int, stream: int | None = None) -> torch.Tensor:
        B, device = self.frames[bid]
        nb = records_nbytes(B, self.per_frame)
        if self.block is None or self.block.numel() != nb:
            self.block = torch.empty(nb, dtype=torch.uint8, device=device)
        self.ctx.records_copy(self.block.data_ptr(), self.per_frame, stream=stream, batch=bid)
        return gather_records(self.block, self.world)

    def step(self, flows: torch.Tensor, persp, inv, inv_upper, params=None, stream: int | None = None):
        return self.collect(self.submit(flows, persp, inv, inv_upper, params, stream), stream)
