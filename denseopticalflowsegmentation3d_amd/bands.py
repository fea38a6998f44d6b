"""Intra-frame sharding of one large frame across GPUs (BASELINE config 5).

The frame is split into contiguous row bands, one per rank. Each rank exchanges the blur halo with
its neighbours (point-to-point over RCCL/xGMI; gloo in the CPU tests), computes its band's minimum
spanning forest on its GPU (`dofs_band_msf_device`), and rank 0 gathers the band forests and flow
rows. Under the strict (weight, emission index) order the global MST — exactly the edges Kruskal
accepts in `segment_graph` (graph.cpp:519-531) — lies inside the union of the band forests and
the band-crossing edges (cycle property: an edge a band's forest drops is the heaviest edge of a
cycle inside that band), so rank 0's MST search over that edge set (`dofs_segment_masked_device`)
gives exactly the single-GPU result. The order-dependent replay and scoring then run on rank 0
(replica-only beyond the MST: the merge order is inherently sequential).

Whether the split pays is decided per frame shape (`split_gain_ms`, `IntraFrame(split="auto")`): it removes
only part of rank 0's MST stage and adds the slowest band's forest and the gather of the band forests to
rank 0. On MI355X at 3840x2160 it costs more than it saves, so "auto" runs the frame on rank 0
alone there ("replica": the ranks hand rank 0 their flow rows, or nothing when the frame is already resident
on rank 0) — a 4-GPU run of config 5 is never slower than one GPU. The single-frame latency floor is the
replay's dependency chain (1.54 M merges at 4K, about 33 ms at 21.5 ns a step), which no split shortens.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .abi import default_params

# edge bits of the per-pixel masks (k: 0 left, 1 up, 2 up-left, 3 down-left; graph.cpp:66-90)
UP, UP_LEFT, DOWN_LEFT = 2, 4, 8


def blur_radius(params=None) -> int:
    """Rows of halo the separable blur needs on each side (ksize = cvRound(8 sigma + 1) | 1)."""
    sigma = (params or default_params()).blur_sigma
    taps = int(round(sigma * 8 + 1)) | 1
    return taps // 2


def band_bounds(H: int, world: int, rank: int) -> tuple[int, int]:
    per = -(-H // world)
    r0 = min(H, rank * per)
    return r0, min(H, r0 + per)


def halo_bounds(H: int, r0: int, r1: int, radius: int) -> tuple[int, int]:
    return max(0, r0 - radius), min(H, r1 + radius)


def add_cut_edges(allowed: torch.Tensor, bounds: list[tuple[int, int]], nbr8: bool = True) -> None:
    """Allow every edge crossing a band boundary (uint8 H x W edge-bit mask, in place)."""
    for r0, _ in bounds[1:]:
        if r0 <= 0 or r0 >= allowed.shape[0]:
            continue
        allowed[r0, :] |= UP
        if nbr8:
            allowed[r0, 1:] |= UP_LEFT
            allowed[r0 - 1, 1:] |= DOWN_LEFT


# Cost model of the split on MI355X, per pixel, from one-GPU measurements of its parts at 3840x2160
# (tools/bench_intraframe.py --model 4, profiles/r05/intraframe_model.json): a band's minimum spanning forest
# 1.28 ms for 3840 x 540 px; rank 0's masked whole-frame path 53.93 ms against 54.86 ms unmasked (the MST work
# the band forests remove); per pixel of every other band, an edge-bit mask byte and a flow row (8 B) gathered.
BAND_MSF_NS_PER_PX = 0.62
MST_SAVED_NS_PER_PX = 0.11
GATHER_BYTES_PER_PX = 9


def split_gain_ms(H: int, W: int, world: int, xgmi_gbs: float = 64.0, resident: bool = True) -> float:
    """Projected ms the row-band split saves one H x W frame over running it on rank 0 alone (negative: it
    costs). resident: the frame's flow is already on rank 0 (else the unsplit path gathers the flow rows
    too, 8 of the split's 9 bytes per pixel, and only the mask byte is extra)."""
    if world < 2:
        return 0.0
    per = -(-H // world) * W
    others = per * (world - 1)
    extra_bytes = (GATHER_BYTES_PER_PX if resident else GATHER_BYTES_PER_PX - 8) * others
    return (MST_SAVED_NS_PER_PX * H * W - BAND_MSF_NS_PER_PX * per) * 1e-6 - extra_bytes / (xgmi_gbs * 1e9) * 1e3


class IntraFrame:
    """One rank's share of an intra-frame sharded frame (one process per GPU).

    split: True — row bands (band forests on every rank, the masked MST on rank 0); False — rank 0 runs the
    frame alone (replica); "auto" — the split only where split_gain_ms says it saves time."""

    def __init__(self, ctx, world: int, rank: int, params=None, split="auto", xgmi_gbs: float = 64.0):
        self.ctx, self.world, self.rank = ctx, world, rank
        self.params = params or default_params()
        self.radius = blur_radius(self.params)
        self.split, self.xgmi_gbs = split, xgmi_gbs

    def splits(self, H: int, W: int, resident: bool = False) -> bool:
        if self.split == "auto":
            return split_gain_ms(H, W, self.world, self.xgmi_gbs, resident) > 0
        return bool(self.split)

    def halo_rows(self, band: torch.Tensor, H: int) -> tuple[torch.Tensor, int]:
        """Flow rows [h0, h1) around this rank's band, from the neighbours' bands (P2P exchange)."""
        world, rank, R = self.world, self.rank, self.radius
        r0, r1 = band_bounds(H, world, rank)
        h0, h1 = halo_bounds(H, r0, r1, R)
        ops, above, below = [], None, None
        # a neighbour band can be thinner than the halo: take rows from as many ranks as needed
        parts_above, parts_below = [], []
        for src in range(world):
            if src == rank:
                continue
            s0, s1 = band_bounds(H, world, src)
            a0, a1 = max(s0, h0), min(s1, r0)  # rows of src this rank needs above its band
            b0, b1 = max(s0, r1), min(s1, h1)  # rows of src this rank needs below
            for lo, hi, dst_list in ((a0, a1, parts_above), (b0, b1, parts_below)):
                if lo < hi:
                    buf = torch.empty((hi - lo,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
                    ops.append(dist.P2POp(dist.irecv, buf, src))
                    dst_list.append((lo, buf))
            # rows of this rank that src needs
            t0, t1 = halo_bounds(H, s0, s1, R)
            for lo, hi in ((max(r0, t0), min(r1, s0)), (max(r0, s1), min(r1, t1))):
                if lo < hi:
                    ops.append(dist.P2POp(dist.isend, band[lo - r0:hi - r0].contiguous(), src))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        above = [b for _, b in sorted(parts_above, key=lambda t: t[0])]
        below = [b for _, b in sorted(parts_below, key=lambda t: t[0])]
        return torch.cat(above + [band] + below), h0

    def step(self, band: torch.Tensor, H: int, W: int, persp, inv, inv_upper, stream: int | None = None,
             frame: torch.Tensor | None = None):
        """band: this rank's flow rows (r1 - r0, W, 2), float32 on the rank's device; frame (rank 0, optional):
        the whole (H, W, 2) flow already resident there. Returns rank 0's batch id (results in rank 0's
        context), None on the other ranks. Every rank must pass the same H, W and whether rank 0 has `frame`
        (the split decision is taken from them on every rank alike)."""
        world, rank = self.world, self.rank
        bounds = [band_bounds(H, world, r) for r in range(world)]
        r0, r1 = bounds[rank]
        self.did_split = self.splits(H, W, resident=frame is not None)
        if not self.did_split:
            return self._replica(band, H, W, persp, inv, inv_upper, stream, frame, bounds)
        rows, h0 = self.halo_rows(band.contiguous(), H)
        mask = torch.zeros((max(r1 - r0, 0), W), dtype=torch.uint8, device=band.device)
        if r1 > r0:
            self.ctx.band_msf_device(rows.data_ptr(), h0, rows.shape[0], H, W, r0, r1, mask.data_ptr(),
                                     params=self.params, stream=stream)
        # gather the band forests and flow rows to rank 0 (fixed-size, padded to the widest band)
        per = max(b1 - b0 for b0, b1 in bounds)
        pm = torch.zeros((per, W), dtype=torch.uint8, device=band.device)
        pf = torch.zeros((per, W, 2), dtype=torch.float32, device=band.device)
        pm[:r1 - r0] = mask
        pf[:r1 - r0] = band
        gm = [torch.empty_like(pm) for _ in range(world)] if rank == 0 else None
        gf = [torch.empty_like(pf) for _ in range(world)] if rank == 0 else None
        dist.gather(pm, gm, dst=0)
        dist.gather(pf, gf, dst=0)
        if rank != 0:
            return None
        allowed = torch.cat([gm[r][:b1 - b0] for r, (b0, b1) in enumerate(bounds)])
        flow = torch.cat([gf[r][:b1 - b0] for r, (b0, b1) in enumerate(bounds)]).contiguous()
        add_cut_edges(allowed, bounds, self.params.neighbor == 8)
        self.flow, self.allowed = flow, allowed  # kept alive until the batch is read
        return self.ctx.segment_masked_device(flow.data_ptr(), H, W, allowed.data_ptr(), persp, inv, inv_upper,
                                              params=self.params, stream=stream)

    def _replica(self, band, H, W, persp, inv, inv_upper, stream, frame, bounds):
        """The frame on rank 0 alone: its flow rows gathered there unless already resident (`frame`)."""
        world, rank = self.world, self.rank
        if frame is None:
            r0, r1 = bounds[rank]
            per = max(b1 - b0 for b0, b1 in bounds)
            pf = torch.zeros((per, W, 2), dtype=torch.float32, device=band.device)
            pf[:r1 - r0] = band
            gf = [torch.empty_like(pf) for _ in range(world)] if rank == 0 else None
            dist.gather(pf, gf, dst=0)
            if rank == 0:
                frame = torch.cat([gf[r][:b1 - b0] for r, (b0, b1) in enumerate(bounds)])
        if rank != 0:
            return None
        self.flow, self.allowed = frame.contiguous(), None  # kept alive until the batch is read
        return self.ctx.segment_batch_device(self.flow.data_ptr(), 1, H, W, persp, inv, inv_upper,
                                             params=self.params, stream=stream)
