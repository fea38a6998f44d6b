"""Generate the golden fixtures of tests/golden/ with the CPU oracle (oracle/dofs_oracle.cpp).

The reference itself cannot run here (its C++ needs OpenCV + spdlog, absent), so these vectors come
from the oracle — pinned by the reference's lifting KAT and cross-checked against the independent
Python restatement (tests/test_oracle_cross.py). They freeze: blurred flow, the Kruskal merge stream
(start, end, weight, root, size, rank, bbox, mean), the snapshot list with member sets, labels.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from denseopticalflowsegmentation3d_amd.abi import default_params  # noqa: E402
from oracle import binding as ob  # noqa: E402

CASES = {  # name: (H, W, seed, min_size, neighbor, extra)
    "g8x8": (8, 8, 0, 5, 8, None),
    "g17x33": (17, 33, 5, 10, 8, None),
    "g48x64_n4": (48, 64, 7, 50, 4, None),
    "g90x160": (90, 160, 0, 500, 8, None),
    "g40x50_ties": (40, 50, 2, 20, 8, "ties"),
}


def make_flow(H, W, seed, extra):
    f = ob.synth_flow(H, W, seed)
    if extra == "ties":  # integer-valued field: massive exact weight ties
        rng = np.random.default_rng(seed)
        f = (np.round(rng.normal(size=(H, W, 2)) * 2) + 1.0).astype(np.float32)
        f[10:30, 5:35] = [2.0, 1.5]
    return f


def main():
    persp, inv, up = ob.calib()
    for name, (H, W, seed, ms, nbr, extra) in CASES.items():
        f = make_flow(H, W, seed, extra)
        prm = default_params()
        prm.min_size = ms
        prm.neighbor = nbr
        o = ob.segment(f, persp, inv, up, params=prm, mode=0, events=True)
        members = [o.members(s) for s in o.snapshots]
        np.savez_compressed(
            os.path.join(HERE, f"{name}.npz"), flow=f, params=np.array([ms, nbr], np.int32),
            calib=np.concatenate([persp.ravel(), inv.ravel(), up.ravel()]), blurred=o.blurred,
            events=o.events.view(np.uint8).reshape(len(o.events), -1) if len(o.events) else np.zeros((0, 56), np.uint8),
            snapshots=o.snapshots.view(np.uint8).reshape(len(o.snapshots), -1) if len(o.snapshots)
            else np.zeros((0, 208), np.uint8),
            member_off=np.cumsum([0] + [len(m) for m in members]).astype(np.int64),
            members=np.concatenate(members).astype(np.int32) if members else np.zeros(0, np.int32),
            labels=o.labels)
        print(name, len(o.events), "merges", len(o.snapshots), "snapshots")


if __name__ == "__main__":
    main()
