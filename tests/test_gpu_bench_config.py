"""GPU: the configuration bench.py measures, checked against the CPU oracle.

bench.py's step drives `frames.Pipelined` over `FrameParallel`: 1920x1080 batches, three workspaces in
turn, batch k's records gathered right after batch k + 2 is submitted, `k_krt_fused` running one
sequential sweep per frame of the batch side by side. Here the same driver runs the benchmarked
configuration itself: four consecutive batches of B = 112 distinct 1080p fields (every workspace is
reused, 112 concurrent sweeps, the MST sort's fix-up at its full cross-frame group count), and sampled
frames of every batch — first, middle, last and one seeded random position — are compared with the
oracle, in the context's default mode (no per-merge event records, dofs_keep_events off: the replay stores
only the records the results read, as bench.py runs it): the gathered box records (slot, size, cls, frame,
move exact; score and the 3D faces within the
stated tolerance, parity.check_records) and, through dofs_batch_fetch_id while the batch is still
readable, the label map and snapshots.

The second test runs config 4's fixed-job split (`frames.job_plan` + `batch_view`, as bench.py
--frames does) for a job of F = 40 frames over three simulated ranks in batches of 8, so chunks are
ragged and the last rank pads; every real frame's gathered records are checked against the oracle.
(Frames are independent — segment.cpp:209-269 — and new_merge's snapshot rule is graph.cpp:348-356.)
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import binding as ob
from parity import check_records

pytestmark = pytest.mark.gpu

PER = 64  # records per frame in the gathered block (bench.py GATHER_PER_FRAME)


def _oracle_many(calib, H, W, seeds, prm=None):
    """Oracle results for several seeds; the oracle's ctypes calls release the GIL, so threads overlap."""
    persp, inv, up = calib

    def one(seed):
        return ob.segment(ob.synth_flow(H, W, seed), persp, inv, up, params=prm, mode=0)
    with ThreadPoolExecutor(max_workers=8) as ex:
        return dict(zip(seeds, ex.map(one, seeds)))


def _check_records(recs, count, o, frame):
    snaps = o.snapshots
    assert int(count) == len(snaps), (int(count), len(snaps))
    check_records(recs, snaps, frame)


def test_bench_configuration_1080p(calib):
    import torch

    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.abi import default_params
    from denseopticalflowsegmentation3d_amd.frames import FrameParallel, Pipelined, decode_records

    H, W, B, NB = 1080, 1920, 112, 4  # bench.py's defaults: B = 112 frames per batch, 1080p
    persp, inv, up = calib
    prm = default_params()
    dev = torch.device("cuda", 0)
    sh = torch.cuda.current_stream(dev).cuda_stream
    rng = np.random.default_rng(4)
    samples = {b: sorted({0, B // 2, B - 1, int(rng.integers(1, B - 1))}) for b in range(NB)}
    seeds = {b: [1000 + b * B + f for f in range(B)] for b in range(NB)}
    want = [seeds[b][f] for b in range(NB) for f in samples[b]]
    oracle = _oracle_many(calib, H, W, want)  # before the GPU work: the CPU is free while it runs

    # its own context (3 workspaces x 112 frames hold ~206 GB of HBM), closed at the end so the
    # session's shared context and later tests get the memory back
    gpu = runtime.Dofs(0)
    flows = []
    for b in range(NB):  # distinct fields per batch, each resident in HBM (as bench.py's input)
        t = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
        runtime.synth_flow_device(t.data_ptr(), B, H, W, seed0=seeds[b][0], stream=sh)
        flows.append(t)

    got = {}
    order = []

    def sink(bid, gathered):  # called while batch `bid` is still readable (before its workspace is reused)
        rec = decode_records(gathered.cpu().numpy(), B, PER)
        buf = gathered.cpu().numpy()
        b = len(order)
        order.append(bid)
        res = {f: gpu.fetch(f, want_blur=False, batch=bid) for f in samples[b]}
        got[bid] = (rec, buf[:4 * B].view(np.int32).copy(), res)

    try:
        assert gpu.batch_slots() == 3
        pipe = Pipelined(FrameParallel(gpu, 1, PER), persp, inv, up, params=prm, stream=sh, sink=sink)
        ids = [pipe.submit(flows[b]) for b in range(NB)]
        pipe.flush()
        torch.cuda.synchronize()
        counters = gpu.batch_counters(B)
        assert not counters[0, 58], "C_FLOWERR: the dataflow replay gave up a bounded wait"
    finally:
        gpu.close()
        del flows
        torch.cuda.empty_cache()
    assert sorted(got) == ids
    for b, bid in enumerate(ids):
        rec, counts, res = got[bid]
        assert all(int(c) > 0 for c in counts), "every 1080p synthetic frame has snapshots"
        for f in samples[b]:
            o = oracle[seeds[b][f]]
            _check_records(rec[f], counts[f], o, f)
            g = res[f]
            assert np.array_equal(g.labels, o.labels), (b, f)
            assert np.array_equal(g.snapshots["slot"], o.snapshots["slot"]), (b, f)
            assert np.array_equal(g.snapshots["event"], o.snapshots["event"]), (b, f)
            assert np.array_equal(g.snapshots["bbox"], o.snapshots["bbox"]), (b, f)


def test_fixed_job_split_ragged(gpu, calib):
    import torch

    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.abi import default_params
    from denseopticalflowsegmentation3d_amd.frames import FrameParallel, Pipelined, decode_records, job_plan

    H, W, F, WORLD, BATCH = 180, 320, 40, 3, 8
    persp, inv, up = calib
    prm = default_params()
    prm.min_size = 300
    dev = torch.device("cuda", 0)
    sh = torch.cuda.current_stream(dev).cuda_stream
    oracle = _oracle_many(calib, H, W, list(range(F)), prm)
    seen = set()
    for rank in range(WORLD):  # each simulated rank's share, run as bench.py --frames runs it
        mine, chunks = job_plan(F, rank, WORLD, BATCH)
        assert chunks == [(0, 8), (8, 6)]  # ceil(40 / 3) = 14 positions per rank, the same chunks on all
        flows = torch.empty((max(len(mine), 1), H, W, 2), dtype=torch.float32, device=dev)
        runtime.synth_flow_device(flows.data_ptr(), max(len(mine), 1), H, W, seed0=mine.start, stream=sh)
        blocks = {}
        pipe = Pipelined(FrameParallel(gpu, 1, PER), persp, inv, up, params=prm, stream=sh,
                         sink=lambda bid, g: blocks.__setitem__(bid, g.cpu().numpy()))
        ids = pipe.run_chunks(flows, chunks)
        pipe.flush()
        torch.cuda.synchronize()
        for (s, n), bid in zip(chunks, ids):
            buf = blocks[bid]
            assert buf.size == 4 * n + n * PER * 96  # every chunk has exactly n frames (equal blocks)
            recs = decode_records(buf, n, PER)
            counts = buf[:4 * n].view(np.int32)
            for f in range(n):
                pos = s + f
                # positions past the rank's frames cycle through its own frames (padding)
                seed = mine.start + (pos if pos < len(mine) else pos % len(mine))
                _check_records(recs[f], counts[f], oracle[seed], f)
                if pos < len(mine):
                    seen.add(seed)
    assert seen == set(range(F))  # every frame of the job ran exactly where job_plan put it
    assert job_plan(9, 6, 8, 4)[0] == range(9, 9)  # F = 9 on 8 ranks: rank 6 owns no frame (placeholder)
