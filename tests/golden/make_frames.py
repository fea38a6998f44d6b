"""Make tests/golden/frames_1052_1053.npz: the reference's own input frame pair (data/frame_1052.png,
data/frame_1053.png — data files of the reference, 640x360 BGR), converted to 8-bit gray with the
COLOR_BGR2GRAY fixed-point rule (oracle/farneback.cpp), plus the oracle's Farneback flow digest
(SHA-256 of the float32 bytes) so later rounds detect any change of the restatement.

Run in the build container (needs /root/reference and PIL): python tests/golden/make_frames.py
"""
import hashlib
import os
import sys

import numpy as np
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import binding as ob  # noqa: E402

REF = "/root/reference/data"


def load_bgr(name):
    rgb = np.array(Image.open(os.path.join(REF, name)).convert("RGB"))
    return np.ascontiguousarray(rgb[:, :, ::-1])


def main():
    g1 = ob.bgr_to_gray(load_bgr("frame_1052.png"))
    g2 = ob.bgr_to_gray(load_bgr("frame_1053.png"))
    flow = ob.farneback(g1, g2)
    digest = hashlib.sha256(flow.tobytes()).hexdigest()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "frames_1052_1053.npz")
    np.savez_compressed(out, prev=g1, next=g2, flow_sha256=np.array(digest),
                        flow_abs_mean=np.array(np.abs(flow).mean(dtype=np.float64)))
    print(out, g1.shape, digest)


if __name__ == "__main__":
    main()
