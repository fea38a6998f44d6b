"""GPU: the C-ABI RCCL gather of box records (include/dofs_rccl.h, libdofs_rccl.so) on a one-rank
communicator (ncclCommInitAll over device 0): the gathered block equals dofs_batch_records_copy's block
byte for byte (ncclGather to root 0 and ncclAllGather), and decodes to the oracle's snapshots (3D box
faces, move and score included). Multi-rank
runs need one process per GPU; the exchange is the same collective with equal blocks per rank."""
import numpy as np
import pytest

from oracle import binding as ob
from parity import check_records, params

pytestmark = pytest.mark.gpu

H, W, B, PER = 90, 160, 4, 64


def test_gather_records_one_rank(gpu, calib):
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.frames import decode_records

    persp, inv, up = calib
    prm = params(300, 8)
    dev = torch.device("cuda", 0)
    sh = torch.cuda.current_stream(dev).cuda_stream
    flows = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    runtime.synth_flow_device(flows.data_ptr(), B, H, W, seed0=7, stream=sh)
    gpu.segment_batch_device(flows.data_ptr(), B, H, W, persp, inv, up, params=prm, stream=sh)
    (comm,) = runtime.Comm.local([0])
    try:
        assert comm.rank() == (0, 1)
        nb = comm.block_bytes(B, PER)
        ref = torch.zeros(nb, dtype=torch.uint8, device=dev)
        got = torch.full((nb,), 0xAB, dtype=torch.uint8, device=dev)
        got_all = torch.full((nb,), 0xCD, dtype=torch.uint8, device=dev)
        gpu.records_copy(ref.data_ptr(), PER, stream=sh)
        comm.gather_records(gpu, PER, got.data_ptr(), root=0, stream=sh)
        comm.gather_records(gpu, PER, got_all.data_ptr(), root=-1, stream=sh)
        torch.cuda.synchronize()
        r = ref.cpu().numpy()
        assert np.array_equal(got.cpu().numpy(), r) and np.array_equal(got_all.cpu().numpy(), r)
    finally:
        comm.close()
    per_frame = decode_records(r, B, PER)
    for f in range(B):
        o = ob.segment(ob.synth_flow(H, W, 7 + f), persp, inv, up, params=prm, mode=0)
        recs = per_frame[f]
        assert len(recs) == len(o.snapshots)
        check_records(recs, o.snapshots, f)  # slot/size/cls/move exact, score and 3D faces within tolerance
