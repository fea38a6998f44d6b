"""Host-side frame helpers for the optical-flow stage (SURVEY.md §8(f) #1 and BASELINE configs 1 / 3).

The reference reads a frame pair with cv::imread and converts it with cvtColor(BGR2GRAY)
(cpp/src/segment.cpp:90-98); the pair it ships (data/frame_1052.png, frame_1053.png, 640x360) is
kept here as a gray fixture (tests/golden/frames_1052_1053.npz, made by tests/golden/make_frames.py).
Config 3 asks for a 1920x1080 real pair: the reference has none, so the shipped pair is upscaled x3
with `upscale` (bilinear, pixel centres aligned, rounded to 8 bits) — a fixed, documented input,
not a claim about what a 1080p camera would see.
"""
from __future__ import annotations

import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FRAMES = os.path.join(ROOT, "tests", "golden", "frames_1052_1053.npz")


def load_gray_pair(path: str = FRAMES) -> tuple[np.ndarray, np.ndarray]:
    """The reference's frame pair as 8-bit gray (prev, next)."""
    z = np.load(path, allow_pickle=False)
    return z["prev"].copy(), z["next"].copy()


def upscale(gray: np.ndarray, factor: int) -> np.ndarray:
    """Bilinear upscale by an integer factor (source sample at (d + 0.5) / factor - 0.5, clamped)."""
    g = gray.astype(np.float64)
    H, W = g.shape

    def axis(n):
        s = (np.arange(n * factor) + 0.5) / factor - 0.5
        s = np.clip(s, 0, n - 1)
        i0 = np.floor(s).astype(np.int64)
        i1 = np.minimum(i0 + 1, n - 1)
        return i0, i1, s - i0

    y0, y1, fy = axis(H)
    x0, x1, fx = axis(W)
    top = g[y0][:, x0] * (1 - fx) + g[y0][:, x1] * fx
    bot = g[y1][:, x0] * (1 - fx) + g[y1][:, x1] * fx
    out = top * (1 - fy)[:, None] + bot * fy[:, None]
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def config3_pair() -> tuple[np.ndarray, np.ndarray]:
    """BASELINE config 3 input: the shipped pair upscaled x3 to 1920x1080."""
    a, b = load_gray_pair()
    return upscale(a, 3), upscale(b, 3)


def synth_clip(n: int, H: int = 360, W: int = 640, seed: int = 0) -> np.ndarray:
    """A BGR test clip (n x H x W x 3 uint8): the reference's frame 1052 (resized to H x W by
    `upscale` / subsampling) as a static background, plus two textured boxes moving (+4, +1) and
    (-3, +2) pixels per frame — the kind of scene main1 (segment.cpp:174-275) processes."""
    bg, _ = load_gray_pair()
    if (H, W) != bg.shape:
        f = max(1, -(-H // bg.shape[0]))
        big = upscale(bg, f) if f > 1 else bg
        ys = (np.arange(H) * big.shape[0]) // H
        xs = (np.arange(W) * big.shape[1]) // W
        bg = big[ys][:, xs]
    rng = np.random.default_rng(seed)
    tex = [rng.integers(0, 256, size=(H // 5, W // 6), dtype=np.uint8) for _ in range(2)]
    starts = [(W // 8, H // 3), (W // 2, H // 6)]
    vel = [(4, 1), (-3, 2)]
    out = np.empty((n, H, W, 3), np.uint8)
    for k in range(n):
        g = bg.astype(np.int32).copy()
        for t, (x0, y0), (vx, vy) in zip(tex, starts, vel):
            x, y = x0 + vx * k, y0 + vy * k
            h, w = t.shape
            ys, xs = slice(max(y, 0), min(y + h, H)), slice(max(x, 0), min(x + w, W))
            g[ys, xs] = t[ys.start - y:ys.stop - y, xs.start - x:xs.stop - x]
        out[k, :, :, 0] = np.clip(g + 7, 0, 255)
        out[k, :, :, 1] = g
        out[k, :, :, 2] = np.clip(g - 11, 0, 255)
    return out
