"""GPU parity: the HIP path through the C-ABI vs the CPU oracle on the same seeded inputs."""
import numpy as np
import pytest

from oracle import binding as ob
from parity import check_exact, params, run_both

pytestmark = pytest.mark.gpu

CASES = [  # (H, W, seed, min_size, neighbor)
    (1, 1, 0, 1, 8), (1, 7, 0, 1, 8), (5, 1, 0, 1, 8), (2, 2, 0, 1, 8), (8, 8, 0, 5, 8),
    (9, 13, 2, 3, 8), (24, 32, 0, 20, 8), (17, 33, 5, 10, 8), (30, 40, 3, 30, 8),
    (64, 48, 7, 50, 4), (90, 160, 0, 500, 8), (180, 320, 1, 500, 8), (360, 640, 0, 500, 8),
    (257, 255, 11, 300, 8),
]


@pytest.mark.parametrize("H,W,seed,min_size,nbr", CASES)
def test_synthetic_parity(gpu, calib, H, W, seed, min_size, nbr):
    flow = ob.synth_flow(H, W, seed)
    o, g, ev = run_both(gpu, flow, calib, params(min_size, nbr))
    check_exact(o, g, ev, lift_exact=False)


@pytest.mark.parametrize("kind", ["zeros", "const", "normal", "ints"])
@pytest.mark.parametrize("H,W", [(70, 90), (72, 96)])  # (72 x 96: W % 4 == 0, the record path and its tiled round 0)
def test_adversarial_parity(gpu, calib, kind, H, W):
    rng = np.random.default_rng(1)
    flow = {"zeros": np.zeros((H, W, 2)), "const": np.full((H, W, 2), 1.5),
            "normal": rng.normal(size=(H, W, 2)),
            "ints": np.round(rng.normal(size=(H, W, 2)) * 4) + 2.0}[kind].astype(np.float32)
    o, g, ev = run_both(gpu, flow, calib, params(50, 8))
    check_exact(o, g, ev, lift_exact=False)


@pytest.mark.parametrize("H,W,seed", [(720, 1280, 3), (1080, 1920, 0)])
def test_full_size_parity(gpu, calib, H, W, seed):
    """BASELINE configs 2/3 shapes: every merge event, snapshot and label bit-exact vs the oracle."""
    flow = ob.synth_flow(H, W, seed)
    o, g, ev = run_both(gpu, flow, calib, params(500, 8))
    check_exact(o, g, ev, lift_exact=False)
