"""Host-side helpers of bench.py (no GPU): the roofline byte model on arrays shaped like the library's
counter and tile-census outputs, and the multi-GPU launcher's refusal to under-report."""
import importlib.util
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_boruvka_min_units():
    b = load_bench()
    N = 1920 * 1080
    R = b.boruvka_rounds(N)
    assert R == 23
    c = np.zeros((2, 64), np.int32)
    c[:, b.ROUND_FLAG:b.ROUND_FLAG + 5] = 1  # rounds 0..4 found edges, round 5 none
    t = np.zeros((2, 40), np.int32)
    t[0, 5] = N          # frame 0: every tile found done in round 5
    t[1, 2] = N // 2     # frame 1: half in round 2, half in round 5
    t[1, 5] = N - N // 2
    p0, p1, launches = b.boruvka_min_units(t, c, N)
    assert launches == 2 * (R - 1)
    # a tile done at round m: pass 0 of rounds 1..m, pass 1 of rounds 1..m-1
    assert p0 == N * 5 + (N // 2) * 2 + (N - N // 2) * 5
    assert p1 == N * 4 + (N // 2) * 1 + (N - N // 2) * 4
    # never found done: every launch that ran for the frame (pass 0 of rounds 1..5, pass 1 of 1..4)
    t2 = np.zeros((1, 40), np.int32)
    t2[0, 0] = N
    assert b.boruvka_min_units(t2, c[:1], N)[:2] == (5 * N, 4 * N)


def test_launcher_refuses_missing_gpus():
    """--gpus 8 with fewer devices must fail (rc != 0), never report fewer GPUs."""
    import torch
    if torch.cuda.device_count() >= 8:
        return
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--cpu-frames", "0"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "device" in r.stderr


def test_world_size_mismatch_fails():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--cpu-frames", "0"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
