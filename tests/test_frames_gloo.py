"""N > 1 path on the CPU: frame sharding and the box-record gather with torch.distributed (gloo,
world size 2), using record blocks laid out exactly as dofs_batch_records_copy writes them."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from conftest import locked_make

from denseopticalflowsegmentation3d_amd.frames import (RECORD_DTYPE, decode_gathered, frame_shard, gather_records,
                                                        records_nbytes)

B, PER = 3, 4


def fake_block(rank):
    counts = np.array([1 + (rank + f) % PER for f in range(B)], np.int32)
    recs = np.zeros((B, PER), RECORD_DTYPE)
    for f in range(B):
        for k in range(counts[f]):
            recs[f, k]["frame"] = rank * B + f
            recs[f, k]["slot"] = 1000 * rank + 10 * f + k
            recs[f, k]["score"] = 0.5 + 0.01 * k
    return np.concatenate([counts.view(np.uint8), recs.view(np.uint8).ravel()])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    blk = torch.from_numpy(fake_block(rank))
    assert blk.numel() == records_nbytes(B, PER)
    g = gather_records(blk, world).numpy()
    frames = decode_gathered(g, world, B, PER)
    q.put((rank, [(int(r["frame"]), int(r["slot"])) for fr in frames for r in fr]))
    dist.destroy_process_group()


def test_frame_shard_covers_all():
    for total in (1, 7, 512):
        for world in (1, 2, 4, 8):
            got = [f for r in range(world) for f in frame_shard(total, r, world)]
            assert got == list(range(total))


def test_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = []
    for r in range(2):
        blk = fake_block(r)
        counts = blk[:4 * B].view(np.int32)
        for f in range(B):
            expect += [(r * B + f, 1000 * r + 10 * f + k) for k in range(counts[f])]
    assert res[0] == expect and res[1] == expect


# ---- the real batch path on every rank: host emulator of the product pipeline (tests/emu) -------------
EH, EW, EB, EPER, EMIN = 61, 47, 2, 16, 40


def _emu_worker(rank, world, port, q, per=16, cap=0):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from denseopticalflowsegmentation3d_amd.abi import default_params
    from denseopticalflowsegmentation3d_amd.frames import FrameParallel
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    from oracle import binding as ob
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = Dofs(0, lib=EMU)
        if cap:
            ctx.set_snapshot_capacity(cap)
        persp, inv, up = ob.calib()
        prm = default_params()
        prm.min_size = EMIN
        mine = frame_shard(world * EB, rank, world)
        flows = torch.from_numpy(np.stack([ob.synth_flow(EH, EW, s) for s in mine]))
        fp = FrameParallel(ctx, world, per)
        g = fp.step(flows, persp, inv, up, params=prm).numpy()
        if rank == 0:
            n = records_nbytes(EB, per)
            counts = [int(c) for r in range(world) for c in g[r * n:r * n + 4 * EB].view(np.int32)]
            frames = decode_gathered(g, world, EB, per)
            q.put(([f.tobytes() for f in frames], counts))
        ctx.close()
    finally:
        dist.destroy_process_group()


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "_build", "libdofs_emu.so")


def _run_emu_world2(per, cap):
    locked_make(os.path.join(ROOT, "tests", "emu"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() + 7 * per) % 500
    ps = [ctx.Process(target=_emu_worker, args=(r, 2, port, q, per, cap)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def _check_emu(got, calib, per):
    from oracle import binding as ob
    from parity import check_records, params
    persp, inv, up = calib
    frames, counts = got
    assert len(frames) == 2 * EB
    nsnap, truncated = 0, 0
    for gf, raw in enumerate(frames):
        recs = np.frombuffer(raw, RECORD_DTYPE)
        o = ob.segment(ob.synth_flow(EH, EW, gf), persp, inv, up, params=params(EMIN, 8), mode=0)
        s = o.snapshots
        assert counts[gf] == len(s)  # the full count, also when the records were truncated
        truncated += len(s) > per
        s = s[:per]
        assert len(recs) == len(s)
        # frame index within the rank's batch; every field of the record bit-exact (emulator: same libm)
        nsnap += check_records(recs, s, gf % EB, exact=True)
    assert nsnap > 0
    return truncated


def test_gather_real_pipeline_world2(calib):
    """Each gloo rank segments its frames through the product pipeline (host emulator, same kernel
    bodies) and the gathered box records equal the oracle's snapshots of every frame, in frame order —
    slot, size, class, move, score and the 3D box faces, bit for bit."""
    assert _check_emu(_run_emu_world2(EPER, 0), calib, EPER) == 0


def test_gather_one_rank_overflows_world2(calib):
    """Snapshot capacity 6 on both ranks: rank 0's second frame has 7 snapshots (its records overflow the
    capacity), rank 1's frames fit. Neither rank fails or skips the collective (the record copy never
    depends on the data); the gathered counts show the truncated frame and its first 6 records are exact."""
    assert _check_emu(_run_emu_world2(6, 6), calib, 6) == 1
