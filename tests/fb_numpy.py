"""Independent numpy restatement of the Farneback oracle (oracle/farneback.cpp) — TEST INFRASTRUCTURE.

Written separately from the C oracle (same published algorithm, OpenCV 4.x optflowgf.cpp and the
imgproc filters it calls, scalar operation order, float32 / float64 exactly where OpenCV uses them)
so that tests/test_farneback.py can catch transcription slips in either. Vectorised across the
independent axis of every step; the running sums of the box filter keep their sequential order.
"""
from __future__ import annotations

import math

import numpy as np

f32 = np.float32


def cv_round(v: float) -> int:
    return int(np.rint(v))  # round half to even, like lrint


def gauss_kernel(n: int, sigma: float) -> np.ndarray:
    if sigma <= 0 and n == 3:
        return np.array([0.25, 0.5, 0.25], f32)
    sx = sigma if sigma > 0 else n * 0.15 + 0.35
    scale2 = -0.125 / (sx * sx)
    n2 = (n - 1) // 2
    v = [math.exp(float(x * x) * scale2) for x in range(1 - n, 0, 2)]
    s = 0.0
    for t in v:
        s += t
    mul = 1.0 / (s * 2.0 + 1.0)
    s2 = 0.0
    for i in range(n2):
        v[i] = v[i] * mul
        s2 += v[i]
    v.append(1.0 - s2 * 2.0)
    k = np.zeros(n, f32)
    for i in range(n2 + 1):
        k[i] = k[n - 1 - i] = f32(v[i])
    return k


def _refl(idx: np.ndarray, n: int) -> np.ndarray:
    idx = np.abs(idx)
    return np.where(idx >= n, 2 * n - idx - 2, idx)


def blur(img: np.ndarray, ks: int, sigma: float) -> np.ndarray:
    k = gauss_kernel(ks, sigma)
    H, W = img.shape
    r = ks // 2
    xs = np.arange(W)
    if ks == 3:
        t = img * k[1] + (img[:, _refl(xs - 1, W)] + img[:, _refl(xs + 1, W)]) * k[0]
    else:
        t = k[0] * img[:, _refl(xs - r, W)]
        for i in range(1, ks):
            t = t + k[i] * img[:, _refl(xs - r + i, W)]
    ys = np.arange(H)
    if ks == 3:
        out = (t[_refl(ys - 1, H)] + t[_refl(ys + 1, H)]) * k[0] + t * k[1] + f32(0)
    else:
        out = k[r] * t + f32(0)
        for j in range(1, r + 1):
            out = out + k[r + j] * (t[_refl(ys + j, H)] + t[_refl(ys - j, H)])
    return out.astype(f32)


def resize(img: np.ndarray, dh: int, dw: int) -> np.ndarray:
    sh, sw = img.shape[:2]
    if (sh, sw) == (dh, dw):
        return img.copy()
    if sw == 2 * dw and sh == 2 * dh:
        a, b = img[0::2, 0::2], img[0::2, 1::2]
        c, d = img[1::2, 0::2], img[1::2, 1::2]
        return ((a + b) + (c + d)) * f32(0.25)
    sx_scale, sy_scale = sw / dw, sh / dh
    xofs = np.zeros(dw, np.int64)
    ax = np.zeros((dw, 2), f32)
    one_term = np.zeros(dw, bool)
    xmin, xmax = 0, dw
    for dx in range(dw):
        fx = f32((dx + 0.5) * sx_scale - 0.5)
        sx = int(math.floor(fx))
        fx = f32(fx - f32(sx))
        if sx < 0:
            xmin = dx + 1
            fx, sx = f32(0), 0
        if sx + 1 >= sw:
            xmax = min(xmax, dx)
            if sx >= sw - 1:
                fx, sx = f32(0), sw - 1
        xofs[dx] = sx
        ax[dx] = (f32(1) - fx, fx)
    one_term[:xmin] = True
    one_term[xmax:] = True
    nxt = np.minimum(xofs + 1, sw - 1)
    exp = (slice(None),) + ((None,) if img.ndim == 3 else ())
    a0, a1 = ax[:, 0][exp], ax[:, 1][exp]
    ot = one_term[exp]
    out = np.zeros((dh, dw) + img.shape[2:], f32)
    for dy in range(dh):
        fy = f32((dy + 0.5) * sy_scale - 0.5)
        sy = int(math.floor(fy))
        fy = f32(fy - f32(sy))
        rows = []
        for k in range(2):
            S = img[min(max(sy + k, 0), sh - 1)]
            rows.append(np.where(ot, S[xofs] * a0, S[xofs] * a0 + S[nxt] * a1))
        out[dy] = rows[0] * (f32(1) - fy) + rows[1] * fy
    return out


def poly_consts(n: int, sigma: float):
    if sigma < 1.1920929e-07:
        sigma = n * 0.3
    xs = list(range(-n, n + 1))
    g = [f32(math.exp(-x * x / (2 * sigma * sigma))) for x in xs]
    s = 0.0
    for v in g:
        s += float(v)
    s = 1.0 / s
    g = [f32(float(v) * s) for v in g]
    xg = [f32(f32(x) * v) for x, v in zip(xs, g)]
    xxg = [f32(f32(x * x) * v) for x, v in zip(xs, g)]
    G = np.zeros((6, 6))
    for iy, y in enumerate(xs):
        for ix, x in enumerate(xs):
            p = f32(g[iy] * g[ix])
            G[0, 0] += float(p)
            G[1, 1] += float(f32(f32(p * f32(x)) * f32(x)))
            G[3, 3] += float(f32(f32(f32(f32(p * f32(x)) * f32(x)) * f32(x)) * f32(x)))
            G[5, 5] += float(f32(f32(f32(f32(p * f32(x)) * f32(x)) * f32(y)) * f32(y)))
    G[2, 2] = G[0, 3] = G[0, 4] = G[3, 0] = G[4, 0] = G[1, 1]
    G[4, 4] = G[3, 3]
    G[3, 4] = G[4, 3] = G[5, 5]
    L = G.copy()
    m = 6
    for i in range(m):
        for j in range(i):
            s = L[i, j]
            for k in range(j):
                s -= L[i, k] * L[j, k]
            L[i, j] = s * L[j, j]
        s = L[i, i]
        for k in range(i):
            s -= L[i, k] * L[i, k]
        L[i, i] = 1.0 / math.sqrt(s)
    X = np.eye(m)
    for i in range(m):
        for j in range(m):
            s = X[i, j]
            for k in range(i):
                s -= L[i, k] * X[k, j]
            X[i, j] = s * L[i, i]
    for i in range(m - 1, -1, -1):
        for j in range(m):
            s = X[i, j]
            for k in range(m - 1, i, -1):
                s -= L[k, i] * X[k, j]
            X[i, j] = s * L[i, i]
    return (np.array(g, f32), np.array(xg, f32), np.array(xxg, f32),
            np.array([X[1, 1], X[0, 3], X[3, 3], X[5, 5]]))


def poly_exp(img: np.ndarray, n: int, sigma: float) -> np.ndarray:
    g, xg, xxg, ig = poly_consts(n, sigma)
    g, xg, xxg = g[n:], xg[n:], xxg[n:]  # index 0..n
    H, W = img.shape
    out = np.zeros((H, W, 5), f32)
    for y in range(H):
        r0 = img[y] * g[0]
        r1 = np.zeros(W, f32)
        r2 = np.zeros(W, f32)
        for k in range(1, n + 1):
            a = img[max(y - k, 0)]
            b = img[min(y + k, H - 1)]
            p = a + b
            r0 = r0 + g[k] * p
            r1 = r1 + xg[k] * (b - a)
            r2 = r2 + xxg[k] * p
        pad = lambda r: np.concatenate([np.full(n, r[0], f32), r, np.full(n, r[-1], f32)])
        R0, R1, R2 = pad(r0), pad(r1), pad(r2)
        c = slice(n, n + W)
        b1 = (R0[c] * g[0]).astype(np.float64)
        b2 = np.zeros(W)
        b3 = (R1[c] * g[0]).astype(np.float64)
        b4 = np.zeros(W)
        b5 = (R2[c] * g[0]).astype(np.float64)
        b6 = np.zeros(W)
        for k in range(1, n + 1):
            p, m_ = slice(n + k, n + k + W), slice(n - k, n - k + W)
            tg = (R0[p] + R0[m_]).astype(np.float64)
            b1 = b1 + tg * np.float64(g[k])
            b4 = b4 + tg * np.float64(xxg[k])
            b2 = b2 + ((R0[p] - R0[m_]) * xg[k]).astype(np.float64)
            b3 = b3 + ((R1[p] + R1[m_]) * g[k]).astype(np.float64)
            b6 = b6 + ((R1[p] - R1[m_]) * xg[k]).astype(np.float64)
            b5 = b5 + ((R2[p] + R2[m_]) * g[k]).astype(np.float64)
        out[y, :, 1] = (b2 * ig[0]).astype(f32)
        out[y, :, 0] = (b3 * ig[0]).astype(f32)
        out[y, :, 3] = (b1 * ig[1] + b4 * ig[2]).astype(f32)
        out[y, :, 2] = (b1 * ig[1] + b5 * ig[2]).astype(f32)
        out[y, :, 4] = (b6 * ig[3]).astype(f32)
    return out


_BORDER = np.array([0.14, 0.14, 0.4472, 0.4472, 0.4472], f32)


def update_matrices(R0, R1, flow):
    H, W = flow.shape[:2]
    ys, xs = np.mgrid[0:H, 0:W]
    dx, dy = flow[..., 0], flow[..., 1]
    fx = xs.astype(f32) + dx
    fy = ys.astype(f32) + dy
    x1 = np.floor(fx).astype(np.int64)
    y1 = np.floor(fy).astype(np.int64)
    fx = fx - x1.astype(f32)
    fy = fy - y1.astype(f32)
    inside = (x1 >= 0) & (x1 < W - 1) & (y1 >= 0) & (y1 < H - 1)
    xc, yc = np.clip(x1, 0, W - 2), np.clip(y1, 0, H - 2)
    one = f32(1)
    a00, a01 = (one - fx) * (one - fy), fx * (one - fy)
    a10, a11 = (one - fx) * fy, fx * fy
    r = []
    for c in range(5):
        v = a00 * R1[yc, xc, c] + a01 * R1[yc, xc + 1, c] + a10 * R1[yc + 1, xc, c] + a11 * R1[yc + 1, xc + 1, c]
        r.append(v)
    r2, r3, r4, r5, r6 = r
    r4 = np.where(inside, (R0[..., 2] + r4) * f32(0.5), R0[..., 2])
    r5 = np.where(inside, (R0[..., 3] + r5) * f32(0.5), R0[..., 3])
    r6 = np.where(inside, (R0[..., 4] + r6) * f32(0.25), R0[..., 4] * f32(0.5))
    r2 = np.where(inside, r2, f32(0))
    r3 = np.where(inside, r3, f32(0))
    r2 = (R0[..., 0] - r2) * f32(0.5)
    r3 = (R0[..., 1] - r3) * f32(0.5)
    r2 = r2 + (r4 * dy + r6 * dx)
    r3 = r3 + (r6 * dy + r5 * dx)
    one5 = lambda c, i: np.where(c, _BORDER[np.clip(i, 0, 4)], one)
    sc = ((one5(xs < 5, xs) * one5(xs >= W - 5, W - xs - 1)) * one5(ys < 5, ys)) * one5(ys >= H - 5, H - ys - 1)
    edge = (xs < 5) | (xs >= W - 5) | (ys < 5) | (ys >= H - 5)
    r2, r3, r4, r5, r6 = (np.where(edge, v * sc, v) for v in (r2, r3, r4, r5, r6))
    M = np.stack([r4 * r4 + r6 * r6, (r4 + r5) * r6, r5 * r5 + r6 * r6, r4 * r2 + r6 * r3, r6 * r2 + r5 * r3], -1)
    return M.astype(f32)


def update_flow_blur(R0, R1, flow, M, bs: int, upd: bool):
    H, W = flow.shape[:2]
    m = bs // 2
    scale = 1.0 / (bs * bs)
    Mf = M.reshape(H, W * 5)
    vsum = (Mf[0] * f32(m + 2)).astype(np.float64)
    for y in range(1, m):
        vsum = vsum + Mf[min(y, H - 1)].astype(np.float64)
    V = np.zeros((H, W * 5))
    for y in range(H):
        vsum = vsum + (Mf[min(y + m, H - 1)] - Mf[max(y - m - 1, 0)]).astype(np.float64)
        V[y] = vsum
    V = V.reshape(H, W, 5)
    Vp = np.concatenate([np.repeat(V[:, :1], m + 1, 1), V, np.repeat(V[:, -1:], m + 1, 1)], 1)  # index x + m + 1
    acc = V[:, 0] * (m + 2)
    for x in range(1, m):
        acc = acc + V[:, x]
    new = np.zeros_like(flow)
    for x in range(W):
        acc = acc + (Vp[:, x + m + m + 1] - Vp[:, x - m - 1 + m + 1])
        g11, g12, g22, h1, h2 = (acc[:, i] * scale for i in range(5))
        idet = 1.0 / (g11 * g22 - g12 * g12 + 1e-3)
        new[:, x, 0] = ((g11 * h2 - g12 * h1) * idet).astype(f32)
        new[:, x, 1] = ((g22 * h1 - g12 * h2) * idet).astype(f32)
    flow[...] = new
    if upd:
        M[...] = update_matrices(R0, R1, flow)


def farneback(prev, nxt, pyr_scale=0.5, levels=3, winsize=15, iterations=3, poly_n=5, poly_sigma=1.2):
    rows, cols = prev.shape
    scale = 1.0
    k = 0
    while k < levels:
        scale *= pyr_scale
        if cols * scale < 32 or rows * scale < 32:
            break
        k += 1
    levels = k
    imgs = [prev.astype(f32), nxt.astype(f32)]
    prev_flow = None
    for k in range(levels, -1, -1):
        scale = 1.0
        for _ in range(k):
            scale *= pyr_scale
        sigma = (1.0 / scale - 1) * 0.5
        ks = max(cv_round(sigma * 5) | 1, 3)
        width, height = cv_round(cols * scale), cv_round(rows * scale)
        if prev_flow is None:
            flow = np.zeros((height, width, 2), f32)
        else:
            flow = resize(prev_flow, height, width) * f32(1.0 / pyr_scale) + f32(0)
        R = [poly_exp(resize(blur(im, ks, sigma), height, width), poly_n, poly_sigma) for im in imgs]
        M = update_matrices(R[0], R[1], flow)
        for i in range(iterations):
            update_flow_blur(R[0], R[1], flow, M, winsize, i < iterations - 1)
        prev_flow = flow
    return prev_flow
