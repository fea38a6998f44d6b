"""N > 1 path on the CPU: frame sharding and the box-record gather with torch.distributed (gloo,
world size 2), using record blocks laid out exactly as dofs_batch_records_copy writes them."""
import os

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

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
