"""Intra-frame sharding (BASELINE config 5) on the CPU: row bands over world-size 2 and 3 gloo ranks,
halo exchange, per-band minimum spanning forests, gather to rank 0 and the masked MST search — run
through the test-only host emulator of the product pipeline (tests/emu), and compared with the
oracle's single-frame result (bit-exact, lifting included)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from conftest import locked_make

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "_build", "libdofs_emu.so")
H, W, SEED, MIN_SIZE = 61, 47, 3, 40


def _worker(rank, world, port, q, split=True):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from denseopticalflowsegmentation3d_amd.bands import IntraFrame, band_bounds
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    from oracle import binding as ob
    from parity import params
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = Dofs(0, lib=EMU, keep_events=True)
        persp, inv, up = ob.calib()
        flow = torch.from_numpy(ob.synth_flow(H, W, SEED))
        r0, r1 = band_bounds(H, world, rank)
        sh = IntraFrame(ctx, world, rank, params(MIN_SIZE, 8), split=split)
        bid = sh.step(flow[r0:r1].contiguous(), H, W, persp, inv, up)
        assert sh.did_split == (split is True)  # ("auto" takes the replica path on a frame this small)
        if rank == 0:
            g = ctx.fetch(0)
            ev = ctx.events(0)
            allowed = int(np.unpackbits(sh.allowed.numpy()[..., None], axis=-1).sum()) if sh.did_split else -1
            q.put((bid, g.labels, g.snapshots, g.leaf_order, g.blurred, g.stats, ev, allowed))
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,split", [(2, True), (3, True), (2, "auto"), (3, False)])
def test_intraframe_matches_single_frame(world, split, calib):
    locked_make(os.path.join(ROOT, "tests", "emu"))
    from oracle import binding as ob
    from parity import check_exact, params
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + 4 * world + (split is True) + 2 * (split == "auto") + os.getpid() % 500
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, split)) for r in range(world)]
    for p in ps:
        p.start()
    bid, labels, snaps, leaf, blurred, stats, ev, allowed = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    persp, inv, up = calib
    o = ob.segment(ob.synth_flow(H, W, SEED), persp, inv, up, params=params(MIN_SIZE, 8), mode=0, events=True)

    class G:
        pass
    g = G()
    g.labels, g.snapshots, g.blurred, g.stats, g.leaf_order = labels, snaps, blurred, stats, leaf
    g.members = lambda s: np.sort(leaf[s["seg_begin"]:s["seg_begin"] + s["size"]])
    check_exact(o, g, ev, lift_exact=True)
    if split is True:
        total = 4 * H * W - 3 * W - 3 * H + 2
        assert H * W - 1 <= allowed < total  # the band forests pruned the edge set, and kept the MST


def test_split_policy():
    """The split cost model (bands.split_gain_ms): at 3840x2160 on 4 GPUs the band forests and their gather
    cost more than the MST work they remove, so "auto" runs the frame on rank 0 alone (config 5 never slower
    than one GPU); with a very fast link and many GPUs the model's sign follows its terms."""
    from denseopticalflowsegmentation3d_amd.bands import split_gain_ms
    assert split_gain_ms(2160, 3840, 4) < 0 and split_gain_ms(2160, 3840, 4, resident=False) < 0
    assert split_gain_ms(2160, 3840, 1) == 0.0
    g8 = split_gain_ms(2160, 3840, 8, xgmi_gbs=1e9, resident=False)
    g2 = split_gain_ms(2160, 3840, 2, xgmi_gbs=1e9, resident=False)
    assert g8 > g2
