"""Host-side helpers of bench.py (no GPU): the roofline byte model must run on a counters array shaped
like dofs_batch_counters' output, and every helper the timed path calls must exist."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_boruvka_min_bytes():
    b = load_bench()
    N = 1920 * 1080
    R = min(b.ceil_log2(N) + 2, 39)
    assert R == 23
    c = np.zeros((4, 64), np.int32)
    c[:, b.ROUND_FLAG:b.ROUND_FLAG + 5] = 1  # rounds 0..4 found edges
    alg, launches = b.boruvka_min_bytes(c, N)
    b0, b1 = b.KERNEL_BYTES["k_boruvka_min"]
    assert launches == 2 * (R - 1)
    # pass 0 of rounds 1..5 (round r-1 active), pass 1 of rounds 1..4 (round r active)
    assert alg == 4 * N * (5 * b0 + 4 * b1)


def test_dnc_L_edges():
    b = load_bench()
    assert b.dnc_L_edges(b.DEEP_BLOCK) == []
    e = b.dnc_L_edges(4 * b.DEEP_BLOCK)
    assert e == [2 * b.DEEP_BLOCK, 2 * b.DEEP_BLOCK]
