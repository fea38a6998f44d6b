"""GPU: the device-resident batch API (dofs_segment_batch_device) and its two-stage pipeline.

Consecutive batches overlap on the context's two streams and alternate between two workspaces;
the caller may overwrite its input buffer in stream order right after a call. Every frame's box
records and labels must still equal the CPU oracle's snapshots for that frame's seeded input.
"""
import numpy as np
import pytest

from oracle import binding as ob
from parity import params

pytestmark = pytest.mark.gpu

H, W, B, PER = 180, 320, 3, 256


def _oracle(calib, seed, prm):
    persp, inv, up = calib
    return ob.segment(ob.synth_flow(H, W, seed), persp, inv, up, params=prm, mode=0)


def _check_records(recs, counts, o, frame):
    snaps = o.snapshots
    assert int(counts) == len(snaps)
    r = recs[:len(snaps)]
    assert np.array_equal(r["slot"], snaps["slot"])
    assert np.array_equal(r["size"], snaps["size"])
    assert np.array_equal(r["frame"], np.full(len(snaps), frame, np.int32))
    assert np.array_equal(r["cls"], snaps["sol"]["cls"])
    assert np.allclose(r["score"], snaps["score"].astype(np.float32), rtol=0, atol=1e-6)


def test_pipelined_batches_match_oracle(gpu, calib):
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.frames import decode_records, records_nbytes

    persp, inv, up = calib
    prm = params(300, 8)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream
    flows = torch.empty((B, H, W, 2), dtype=torch.float32, device=dev)
    nb = records_nbytes(B, PER)
    blocks = [torch.empty(nb, dtype=torch.uint8, device=dev) for _ in range(3)]

    # three batches through ONE input buffer, regenerated in stream order after each call
    ids = []
    for b in range(3):
        runtime.synth_flow_device(flows.data_ptr(), B, H, W, seed0=b * B, stream=sh)
        ids.append(gpu.segment_batch_device(flows.data_ptr(), B, H, W, persp, inv, up, params=prm, stream=sh))
        if b >= 1:  # results of the previous batch while this one runs
            gpu.records_copy(blocks[b - 1].data_ptr(), PER, stream=sh, batch=ids[b - 1])
    gpu.records_copy(blocks[2].data_ptr(), PER, stream=sh, batch=ids[2])
    assert ids == [ids[0], ids[0] + 1, ids[0] + 2]
    torch.cuda.synchronize()

    for b in range(3):
        per_frame = decode_records(blocks[b].cpu().numpy(), B, PER)
        buf = blocks[b].cpu().numpy()
        counts = buf[:4 * B].view(np.int32)
        for f in range(B):
            o = _oracle(calib, b * B + f, prm)
            _check_records(per_frame[f], counts[f], o, f)
            if b == 2:  # the last batch is also readable through dofs_batch_fetch
                g = gpu.fetch(f, want_blur=False)
                assert np.array_equal(g.labels, o.labels)
                assert np.array_equal(g.snapshots["slot"], o.snapshots["slot"])

    with pytest.raises(RuntimeError):  # only the last (three) batches stay readable
        gpu.records_copy(blocks[0].data_ptr(), PER, stream=sh, batch=ids[0] - 1)


def test_batch_records_device_pointers(gpu, calib):
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    from denseopticalflowsegmentation3d_amd.abi import DofsBoxRecord

    persp, inv, up = calib
    prm = params(300, 8)
    flows = torch.empty((2, H, W, 2), dtype=torch.float32, device="cuda:0")
    sh = torch.cuda.current_stream().cuda_stream
    runtime.synth_flow_device(flows.data_ptr(), 2, H, W, seed0=40, stream=sh)
    gpu.segment_batch_device(flows.data_ptr(), 2, H, W, persp, inv, up, params=prm, stream=sh)
    rec, cnt, cap = gpu.records_device()
    isz = DofsBoxRecord.np_dtype().itemsize
    raw = np.empty(2 * cap * isz, np.uint8)
    ctr = np.empty(2 * 64, np.int32)
    import ctypes
    # the HIP runtime already mapped into this process (torch's or /opt/rocm's; one soname)
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(path)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    assert hip.hipMemcpy(raw.ctypes.data, rec, raw.nbytes, 2) == 0
    assert hip.hipMemcpy(ctr.ctypes.data, cnt, ctr.nbytes, 2) == 0
    recs = raw.view(DofsBoxRecord.np_dtype()).reshape(2, cap)
    for f in range(2):
        o = _oracle(calib, 40 + f, prm)
        _check_records(recs[f], ctr[64 * f + 4], o, f)


def test_device_synth_matches_oracle():
    """The bench's on-device input generator is the oracle's synthetic spec, bit for bit."""
    import torch
    from denseopticalflowsegmentation3d_amd import runtime
    flows = torch.empty((3, 37, 53, 2), dtype=torch.float32, device="cuda:0")
    runtime.synth_flow_device(flows.data_ptr(), 3, 37, 53, seed0=5, stream=torch.cuda.current_stream().cuda_stream)
    got = flows.cpu().numpy()
    for f in range(3):
        assert got[f].tobytes() == ob.synth_flow(37, 53, 5 + f).tobytes()
