"""Pure-Python restatement of the reference path, for SMALL inputs only — TEST INFRASTRUCTURE ONLY.

Written independently of oracle/dofs_oracle.cpp, line by line from the reference sources, to
cross-check the C++ oracle (tests/test_oracle_cross.py). float32 arithmetic is done with explicit
np.float32 operands on both sides (numpy ≥ 2 keeps float32 ⊗ float32 in float32); C++ double
arithmetic is done in Python floats. No FMA anywhere, like the reference's x86-64 -O0 build.

References (DmitriyZhuravlev/DenseOpticalFlowSegmentation3D @ v1):
  segment.cpp:20-72, graph.cpp:43-536, lifting_3d.cpp:63-439, draw.cpp:118-147.
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32


def fadd(a, b):
    return F(F(a) + F(b))


def fsub(a, b):
    return F(F(a) - F(b))


def fmul(a, b):
    return F(F(a) * F(b))


def fdiv(a, b):
    return F(F(a) / F(b))


# --- OpenCV Point2f semantics -------------------------------------------------------------------
def pt(x, y):
    return (F(x), F(y))


def padd(a, b):
    return (fadd(a[0], b[0]), fadd(a[1], b[1]))


def psub(a, b):
    return (fsub(a[0], b[0]), fsub(a[1], b[1]))


def pnorm(a):  # cv::norm(Point2f): sqrt((double)x*x + (double)y*y)
    x, y = float(a[0]), float(a[1])
    return math.sqrt(x * x + y * y)


def dmul(d, a):  # double * Point2f -> Point2f(float(x*d))
    return (F(float(a[0]) * d), F(float(a[1]) * d))


def pdivd(a, d):  # Point2f / double
    return (F(float(a[0]) / d), F(float(a[1]) / d))


# --- lifting_3d.cpp ---------------------------------------------------------------------------
def get_intersect(A, B, C, D):  # :63-89
    a1 = fsub(B[1], A[1])
    b1 = fsub(A[0], B[0])
    c1 = fadd(fmul(a1, A[0]), fmul(b1, A[1]))
    a2 = fsub(D[1], C[1])
    b2 = fsub(C[0], D[0])
    c2 = fadd(fmul(a2, C[0]), fmul(b2, C[1]))
    det = fsub(fmul(a1, b2), fmul(a2, b1))
    if float(abs(det)) < 1e-9:
        return (F("nan"), F("nan"))
    x = fdiv(fsub(fmul(b2, c1), fmul(b1, c2)), det)
    y = fdiv(fsub(fmul(a1, c2), fmul(a2, c1)), det)
    return (x, y)


def warp_perspective(p, m):  # :112-121, m = 3x3 float32
    den = fadd(fadd(fmul(m[2][0], p[0]), fmul(m[2][1], p[1])), m[2][2])
    px = fdiv(fadd(fadd(fmul(m[0][0], p[0]), fmul(m[0][1], p[1])), m[0][2]), den)
    py = fdiv(fadd(fadd(fmul(m[1][0], p[0]), fmul(m[1][1], p[1])), m[1][2]), den)
    return (px, py)


def iv(a):
    return (a[0], F(-a[1]))


def get_bottom(warp_corners, orient, w, h):  # :162-217
    a = [iv(p) for p in warp_corners]
    inf = F("inf")
    k = get_intersect(a[3], pt(float(a[3][0]) + math.cos(orient), float(a[3][1]) + math.sin(orient)), a[0], a[1])
    if k[0] == inf or k[1] == inf:
        return -1.0, []
    l = pnorm(psub(a[3], k))
    if l == 0:
        return -1.0, []
    c = pdivd(padd(dmul(l - w, a[0]), dmul(w, a[3])), l)
    b = get_intersect(c, pt(float(c[0]) + math.cos(orient), float(c[1]) + math.sin(orient)), a[0], a[1])
    if b[0] == inf:
        return -1.0, []
    ew = pnorm(psub(c, b))
    error_w = ew / w if ew < w else w / ew
    d = get_intersect(c, pt(float(c[0]) - math.sin(orient), float(c[1]) + math.cos(orient)), a[3], a[2])
    if d[0] == inf:
        return -1.0, []
    el = pnorm(psub(c, d))
    error_l = el / h if el < h else h / el
    s = padd(b, d)
    center = (fdiv(s[0], 2), fdiv(s[1], 2))
    f = psub((fmul(center[0], 2), fmul(center[1], 2)), c)
    return error_w * error_l, [iv(c), iv(b), iv(f), iv(d)]


def get_motion_direction(direction, box, persp):  # :219-253
    sum_x = box[0] + box[2]
    sum_y = box[1] + box[3]
    center = pt(sum_x // 2, sum_y // 2)
    nd = pdivd(direction, pnorm(direction))
    t1 = warp_perspective(center, persp)
    t2 = warp_perspective(padd(center, nd), persp)
    v_x = float(fsub(t2[0], t1[0]))
    v_y = float(fsub(t1[1], t2[1]))
    return math.atan2(v_y, v_x)


OBJ_SIZE = ((258, 84), (349, 165), (370, 180))  # :255-259


def get_upper_face(box, lf):  # :290-348
    xmin, ymin, xmax, ymax = box
    uf = [None] * 4
    uf[2] = psub(lf[2], (F(0), fsub(lf[2][1], ymin)))
    right_van = get_intersect(lf[1], lf[2], lf[0], lf[3])
    uf[1] = get_intersect(uf[2], right_van, pt(xmin, ymin), pt(xmin, ymax))
    left_van = get_intersect(lf[2], lf[3], lf[0], lf[1])
    uf[3] = get_intersect(uf[2], left_van, pt(xmax, ymin), pt(xmax, ymax))
    uf[0] = get_intersect(left_van, uf[1], right_van, uf[3])
    return uf


def get_bottom_variants(direction, box, mat, inv, inv_upper, cls, obj_size=OBJ_SIZE):  # :350-439
    mov_angle = get_motion_direction(direction, box, mat)
    xmin, ymin, xmax, ymax = box
    ps = [pt(xmin, ymax), pt(xmin, ymin), pt(xmax, ymin), pt(xmax, ymax)]
    ps_bev = [warp_perspective(p, mat) for p in ps]
    dim_l, dim_w = obj_size[cls]
    error, corners = get_bottom(ps_bev, mov_angle, float(dim_l), float(dim_w))
    if not corners:
        return dict(cls=cls, valid=0, w_error=0.0, h_error=0.0, orient=0.0)
    untop = [warp_perspective(p, inv) for p in corners]
    uf = get_upper_face(box, untop)
    expected_edge = warp_perspective(corners[0], inv_upper)
    expected_h = pnorm(psub(untop[0], expected_edge))
    computed_h = pnorm(psub(uf[0], untop[0]))
    h_error = computed_h / expected_h if computed_h < expected_h else expected_h / computed_h
    return dict(cls=cls, valid=1, ps_bev=ps_bev, lower_face=untop, upper_face=uf, rectangle=corners,
                w_error=error, h_error=h_error, orient=mov_angle)


def get_score(box, direction, persp, inv, inv_upper):  # graph.cpp:241-270
    max_score = -1.0
    best = None
    for cls in range(3):
        sol = get_bottom_variants(direction, box, persp, inv, inv_upper[cls], cls)
        if sol["valid"] and max_score < (sol["w_error"] + sol["h_error"]) / 2:
            max_score = (sol["w_error"] + sol["h_error"]) / 2
            best = sol
    return max_score, best


# --- segment.cpp:52 GaussianBlur (OpenCV 4.x scalar path) ---------------
def gaussian_kernel(n, sigma):
    scale2X = (-0.5 * 0.25) / (sigma * sigma)
    n2 = (n - 1) // 2
    vals = []
    s = 0.0
    x = 1 - n
    for _ in range(n2):
        t = math.exp(float(x * x) * scale2X)
        vals.append(t)
        s += t
        x += 2
    s *= 2.0
    s += 1.0
    mul1 = 1.0 / s
    s2 = 0.0
    for i in range(n2):
        vals[i] = vals[i] * mul1
        s2 += vals[i]
    s2 *= 2.0
    vals.append(1.0 - s2)
    half = [F(v) for v in vals]
    return half + half[-2::-1]


def refl(p, n):
    if 0 <= p < n:
        return p
    if n == 1:
        return 0
    while not (0 <= p < n):
        p = -p if p < 0 else 2 * n - 2 - p
    return p


def blur(flow, sigma=3.0):
    H, W = flow.shape[:2]
    n = int(round(sigma * 8 + 1)) | 1
    k = gaussian_kernel(n, sigma)
    r = n // 2
    tmp = np.zeros_like(flow)
    for y in range(H):
        for x in range(W):
            for c in range(2):
                s = fmul(k[0], flow[y, refl(x - r, W), c])
                for t in range(1, n):
                    s = fadd(s, fmul(k[t], flow[y, refl(x - r + t, W), c]))
                tmp[y, x, c] = s
    out = np.zeros_like(flow)
    for y in range(H):
        for x in range(W):
            for c in range(2):
                s = fadd(fmul(k[r], tmp[y, x, c]), F(0))
                for j in range(1, r + 1):
                    s = fadd(s, fmul(k[r + j], fadd(tmp[refl(y + j, H), x, c], tmp[refl(y - j, H), x, c])))
                out[y, x, c] = s
    return out


# --- segment.cpp:20-32 diff, graph.cpp:51-103 build_graph ---------------------------------------
def diff(flow, x1, y1, x2, y2):
    dx = float(fsub(flow[y1, x1, 0], flow[y2, x2, 0]))
    dy = float(fsub(flow[y1, x1, 1], flow[y2, x2, 1]))
    return math.sqrt(dx * dx + dy * dy)


def build_graph(flow, nbr8=True):
    H, W = flow.shape[:2]
    edges = []
    for y in range(H):
        for x in range(W):
            v = y * W + x
            if x > 0:
                edges.append((v, v - 1, diff(flow, x, y, x - 1, y)))
            if y > 0:
                edges.append((v, v - W, diff(flow, x, y, x, y - 1)))
            if nbr8:
                if x > 0 and y > 0:
                    edges.append((v, v - W - 1, diff(flow, x, y, x - 1, y - 1)))
                if x > 0 and y < H - 1:
                    edges.append((v, v + W - 1, diff(flow, x, y, x - 1, y + 1)))
    return sorted(edges, key=lambda e: e[2])  # Python sort is stable == multiset upper_bound insertion


# --- graph.cpp Forest + segment_graph ------------------------------------------------------------
def segment(flow_in, persp, inv, inv_upper, min_size=500, score_threshold=0.3, neighbor=8,
            min_conv=(3 / 4, 1 / 2, 20 / 29), overlay=0.7, sigma=3.0):
    flow = blur(np.asarray(flow_in, np.float32), sigma)
    H, W = flow.shape[:2]
    N = H * W
    edges = build_graph(flow, neighbor == 8)
    parent = list(range(N))
    rank = [0] * N
    size = [1] * N
    fv = [(flow[i // W, i % W, 0], flow[i // W, i % W, 1]) for i in range(N)]
    segs = [{i} for i in range(N)]
    bbox = [[i % W, i // W, i % W, i // W] for i in range(N)]
    hist = {}
    events = []

    def find(n):
        while parent[n] != n:
            parent[n] = parent[parent[n]]
            n = parent[n]
        return n

    for (s, e, w) in edges:
        a, b = find(s), find(e)
        if a == b:
            continue
        pa, pb = a, b
        if rank[pa] > rank[pb]:
            pa, pb = pb, pa
        parent[pa] = pb
        sa, sb = size[pa], size[pb]
        wa = (fmul(fv[pa][0], sa), fmul(fv[pa][1], sa))
        wb = (fmul(fv[pb][0], sb), fmul(fv[pb][1], sb))
        ia = 1.0 / (sa + sb)
        fv[pb] = (F(float(fadd(wa[0], wb[0])) * ia), F(float(fadd(wa[1], wb[1])) * ia))
        segs[pb] |= segs[pa]
        segs[pa] = set()
        size[pb] += sa
        size[pa] = 0
        bbox[pb] = [min(bbox[pb][0], bbox[pa][0]), min(bbox[pb][1], bbox[pa][1]),
                    max(bbox[pb][2], bbox[pa][2]), max(bbox[pb][3], bbox[pa][3])]
        if rank[pa] == rank[pb]:
            rank[pb] += 1
        events.append((s, e, w, pb, size[pb], rank[pb], tuple(bbox[pb]), fv[pb]))
        # new_merge filters, graph.cpp:280-356
        if size[pb] < min_size:
            continue
        y = pb // W
        if y < H // 10:
            continue
        mx, my = float(fv[pb][0]), float(fv[pb][1])
        move = math.sqrt(mx * mx + my * my)
        if move < 3 * (y + 1) / float(H):
            continue
        bx = bbox[pb]
        rect_area = float((bx[2] - bx[0] + 1) * (bx[3] - bx[1] + 1))
        convexity = size[pb] / rect_area
        score, sol = get_score(bx, fv[pb], persp, inv, inv_upper)
        if score == -1:
            continue
        if convexity < min_conv[sol["cls"]]:
            continue
        if score > score_threshold:
            if hist.get(pb, (-1.0,))[0] < score:
                hist[pb] = (score, frozenset(segs[pb]), sol, move, len(events) - 1)
    labels = np.full(N, -1, np.int32)
    for slot in sorted(hist):
        if hist[slot][0] > overlay:
            for v in hist[slot][1]:
                labels[v] = slot
    return dict(blurred=flow, edges=edges, events=events, hist=hist, labels=labels)
