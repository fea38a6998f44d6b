"""CPU: the product pipeline's algorithm (kernel bodies + orchestration, run sequentially by the
test-only host emulator) vs the oracle. Bit-exact everywhere (same libm on both sides)."""
import numpy as np
import pytest

from oracle import binding as ob
from parity import check_exact, params, run_both

CASES = [
    (1, 1, 0, 1, 8), (1, 7, 0, 1, 8), (5, 1, 0, 1, 8), (2, 2, 0, 1, 8), (8, 8, 0, 5, 8),
    (9, 13, 2, 3, 8), (24, 32, 0, 20, 8), (17, 33, 5, 10, 8), (30, 40, 3, 30, 8),
    (64, 48, 7, 50, 4), (90, 160, 0, 500, 8), (180, 320, 1, 500, 8),
]


@pytest.mark.parametrize("H,W,seed,min_size,nbr", CASES)
def test_emu_synthetic(emu, calib, H, W, seed, min_size, nbr):
    o, g, ev = run_both(emu, ob.synth_flow(H, W, seed), calib, params(min_size, nbr))
    check_exact(o, g, ev, lift_exact=True)


@pytest.mark.parametrize("kind", ["zeros", "const", "normal", "ints"])
def test_emu_adversarial(emu, calib, kind):
    rng = np.random.default_rng(1)
    H, W = 70, 90
    flow = {"zeros": np.zeros((H, W, 2)), "const": np.full((H, W, 2), 1.5),
            "normal": rng.normal(size=(H, W, 2)),
            "ints": np.round(rng.normal(size=(H, W, 2)) * 4) + 2.0}[kind].astype(np.float32)
    o, g, ev = run_both(emu, flow, calib, params(50, 8))
    check_exact(o, g, ev, lift_exact=True)


# heavy-path lists: tiny paths (<= kTinyPath merges) are listed from the back of the
# short-path buffer and the others from its front; fields dominated by tiny paths (all-tie and
# striped fields at small N) must stay exact and every path must land in exactly one list
C_PATHS, C_SHORT, C_LONG, C_TINY = 0, 6, 7, 15


@pytest.mark.parametrize("kind,H,W", [("zeros", 3, 5), ("zeros", 16, 16), ("stripes", 12, 20),
                                      ("checker", 9, 11), ("normal", 40, 64)])
def test_emu_path_lists(emu, calib, kind, H, W):
    rng = np.random.default_rng(7)
    yy, xx = np.mgrid[0:H, 0:W]
    flow = {"zeros": np.zeros((H, W, 2)),
            "stripes": np.stack([(xx % 3).astype(float), np.zeros((H, W))], -1),
            "checker": np.stack([((xx + yy) % 2) * 2.0, ((xx // 2 + yy) % 3) * 1.0], -1),
            "normal": rng.normal(size=(H, W, 2))}[kind].astype(np.float32)
    o, g, ev = run_both(emu, flow, calib, params(2, 8))
    check_exact(o, g, ev, lift_exact=True)
    c = emu.batch_counters(1)[0]
    assert c[C_TINY] + c[C_SHORT] + c[C_LONG] == c[C_PATHS], c[:16]
    if H * W > 1:
        assert c[C_PATHS] > 0
