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
RECORDS_INVALID = -1  # include/dofs.h DOFS_RECORDS_INVALID: the frame's batch failed (its results are invalid)
DOFS_ERR_INVALID_RESULT = 6  # include/dofs.h: the block was written with RECORDS_INVALID counts


def frame_shard(total: int, rank: int, world: int) -> range:
    """Contiguous block of frames owned by `rank` (block size ceil(total / world))."""
    per = -(-total // world)
    lo = min(total, rank * per)
    return range(lo, min(total, lo + per))


def job_plan(total: int, rank: int, world: int, batch: int) -> tuple[range, list[tuple[int, int]]]:
    """A fixed job of `total` frames over `world` ranks (BASELINE config 4): this rank's frames and the
    chunks (start, n) every rank runs — ceil(total / world) frame positions in batches of at most `batch`,
    the same on every rank, so each collective gather moves equal blocks. A rank with fewer real frames
    fills its positions by cycling its own frames (`batch_view`); those are not counted as work."""
    if total < 1 or world < 1 or batch < 1 or not 0 <= rank < world:
        raise ValueError("job_plan: total, world and batch must be >= 1 and 0 <= rank < world")
    per_rank = -(-total // world)
    return frame_shard(total, rank, world), [(s, min(batch, per_rank - s)) for s in range(0, per_rank, batch)]


def batch_view(flows: torch.Tensor, start: int, n: int) -> torch.Tensor:
    """Frames [start, start + n) of a rank's resident frames, positions past the last one cycling through
    its frames (a rank without frames of its own holds one placeholder frame). Always n frames."""
    L = flows.shape[0]
    if L < 1:
        raise ValueError("batch_view: a rank needs at least one (placeholder) frame")
    if start + n <= L:
        part = flows[start:start + n]
    else:
        ids = torch.arange(start, start + n, device=flows.device)
        part = flows[torch.where(ids < L, ids, ids % L)]
    assert part.shape[0] == n
    return part


def records_nbytes(frames: int, per_frame: int) -> int:
    """Layout written by dofs_batch_records_copy: int32 counts[frames], then frames × per_frame records."""
    return 4 * frames + frames * per_frame * RECORD_DTYPE.itemsize


def decode_records(buf: np.ndarray, frames: int, per_frame: int) -> list[np.ndarray]:
    """Per-frame arrays of valid box records from one rank's block. A block whose counts are
    RECORDS_INVALID (its rank's batch failed) raises instead of decoding."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    counts = buf[:4 * frames].view(np.int32)
    if (counts == RECORDS_INVALID).any():
        raise RuntimeError("gathered box records of a batch whose replay gave up (DOFS_RECORDS_INVALID)")
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
        self.checked = 0  # batches collected whose replay completed (records_copy checks each)

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
        # every batch collected is checked: a batch whose results are invalid (a replay give-up or a refused
        # record) fails here, after the gather, which the other ranks are in — its block carries RECORDS_INVALID
        # counts, so the receivers see it too. Any other error leaves the block undefined: it is not sent.
        rc = self.ctx.records_copy(self.block.data_ptr(), self.per_frame, stream=stream, batch=bid, check=False)
        if rc not in (0, DOFS_ERR_INVALID_RESULT):
            raise RuntimeError(f"dofs_batch_records_copy failed ({rc}): {self.ctx.last_error()}")
        out = gather_records(self.block, self.world)
        self.checked += 1
        if rc:
            raise RuntimeError(f"batch {bid}: dofs_batch_records_copy failed ({rc}): {self.ctx.last_error()}")
        return out

    def step(self, flows: torch.Tensor, persp, inv, inv_upper, params=None, stream: int | None = None):
        return self.collect(self.submit(flows, persp, inv, inv_upper, params, stream), stream)


class Pipelined:
    """The caller's side of the two-stage batch pipeline (bench.py's timed loop and config 4's job): each
    batch is submitted, and batch k's records are gathered right after batch k + slots - 1 is submitted,
    so batch k's replay stage overlaps the graph stage of the batches after it. `sink(bid, gathered)`,
    if given, sees every gathered block (a device tensor reused by the next gather: copy what you keep)
    while the batch's results are still readable on the context."""

    def __init__(self, fp: FrameParallel, persp, inv, inv_upper, params=None, stream: int | None = None, sink=None):
        self.fp, self.args, self.params, self.stream, self.sink = fp, (persp, inv, inv_upper), params, stream, sink
        slots = fp.ctx.batch_slots() if hasattr(fp.ctx, "batch_slots") else 2
        self.lag = slots - 1
        self.pending: list[int] = []

    def _collect(self):
        bid = self.pending.pop(0)
        g = self.fp.collect(bid, stream=self.stream)
        if self.sink is not None:
            self.sink(bid, g)

    def submit(self, flows: torch.Tensor) -> int:
        bid = self.fp.submit(flows, *self.args, params=self.params, stream=self.stream)
        self.pending.append(bid)
        if len(self.pending) > self.lag:
            self._collect()
        return bid

    def flush(self):
        while self.pending:
            self._collect()

    def run_chunks(self, flows: torch.Tensor, chunks) -> list[int]:
        """Submit every chunk (start, n) of this rank's resident frames (batch_view); returns the batch ids."""
        return [self.submit(batch_view(flows, s, n)) for s, n in chunks]
