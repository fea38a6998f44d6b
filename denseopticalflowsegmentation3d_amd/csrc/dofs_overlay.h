// dofs_overlay.h — the consumer of the snapshot list, on the device:
// plot_best_segments_simple(frame, bev, forest, 0.7) (cpp/src/draw.cpp:101-160) with draw_cube
// (draw.cpp:85-99), called by segment.cpp:166 and :258 after get_segmented_array.
//
// The reference, per history slot in ascending order with score > min_score: paints the slot's
// member pixels into `seg` (a copy of the frame) in its class colour (draw.cpp:127-145), then draws
// the 12 cube edges in blue, thickness 1, into both `frame` and `seg` (:146-147); finally
// addWeighted(frame, 0.6, seg, 0.4, 0, frame) (:157-158). Restated per pixel, with
//   P(p) = the largest qualifying slot whose member set holds p (the overlay label map, KLabel)
//   L(p) = the largest qualifying slot whose cube edges cover p (KCubeLines, atomic max)
// the reference's last write to p decides it: seg(p) = blue if L(p) >= P(p) (a slot's edges are
// drawn after its paint), else the colour of P(p)'s class, else the frame pixel; frame(p) = blue
// if L(p) >= 0. addWeighted then rounds (3 frame + 2 seg) / 5, which is never a tie, so the float
// weights of OpenCV (with or without FMA) and this integer form agree exactly.
//
// cv::line(img, Point2f, Point2f, color, 1) converts the end points with cvRound (x86: cvtss2si,
// nearest-even, INT_MIN for NaN and out-of-range), clips them with clipLine and walks
// LineIterator(8-connected, left to right). Each covered pixel is computed in closed form:
// after i major steps the minor offset is max(0, ceil((2 dy i - dx) / (2 dx))) — the Bresenham
// error recurrence err0 = dx - 2dy, err -= 2dy (+2dx when err < 0) solved — so one lane per pixel.
#pragma once

#include "dofs_common.h"

namespace dofs {

struct OverlayWs {
    const unsigned char* frame;  // B x H x W x 3 BGR (packed)
    unsigned char* out;          // same layout (may alias frame)
    int* lmap;                   // B x N: L(p), -1 = no edge
    const int* labels;           // B x N: P(p), -1 = none (KLabel)
    const dofs_snapshot* snaps;  // B x snap_cap, ascending slot
    const int* ctr;              // B x kCounters (snapshot count at C_SNAP)
    int snap_cap;
    int H, W;
    int64_t N;
    double min_score;
};

// cvRound(float) on x86-64 (saturate_cast<int>(float), the Point2f -> Point conversion of cv::line)
DOFS_HDM inline int cv_round_f(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int)0x80000000;  // NaN / out of range
    return (int)rintf(v);
}

// cv::clipLine(Size2l, Point2l&, Point2l&) (OpenCV 4.x drawing.cpp), same operation order.
DOFS_HDM inline bool clip_line(int64_t w, int64_t h, int64_t& x1, int64_t& y1, int64_t& x2, int64_t& y2) {
    if (w <= 0 || h <= 0) return false;
    const int64_t right = w - 1, bottom = h - 1;
    int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        int64_t a;
        if (c1 & 12) {
            a = c1 < 8 ? 0 : bottom;
            x1 += (int64_t)((double)(a - y1) * (double)(x2 - x1) / (double)(y2 - y1));
            y1 = a;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            a = c2 < 8 ? 0 : bottom;
            x2 += (int64_t)((double)(a - y2) * (double)(x2 - x1) / (double)(y2 - y1));
            y2 = a;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                a = c1 == 1 ? 0 : right;
                y1 += (int64_t)((double)(a - x1) * (double)(y2 - y1) / (double)(x2 - x1));
                x1 = a;
                c1 = 0;
            }
            if (c2) {
                a = c2 == 1 ? 0 : right;
                y2 += (int64_t)((double)(a - x2) * (double)(y2 - y1) / (double)(x2 - x1));
                x2 = a;
                c2 = 0;
            }
        }
    }
    return (c1 | c2) == 0;
}

// The pixels cv::line(img, a, b, color, 1, LINE_8) writes: count = major length + 1; pixel i is
// (x0 + i * mx + k_i * nx, y0 + i * my + k_i * ny) with k_i the minor offset above.
struct LineWalk {
    int x0, y0, mx, my, nx, ny;
    int64_t dx, dy;  // major, minor lengths
    int count;
    DOFS_HDM void at(int64_t i, int& x, int& y) const {
        int64_t k = 0;
        if (dx > 0) {
            const int64_t num = 2 * dy * i - dx;  // k_i = max(0, ceil(num / (2 dx)))
            k = num <= 0 ? 0 : (num + 2 * dx - 1) / (2 * dx);
        }
        x = x0 + (int)(i * mx + k * nx);
        y = y0 + (int)(i * my + k * ny);
    }
};

DOFS_HDM inline LineWalk line_walk(int W, int H, float ax, float ay, float bx, float by) {
    LineWalk L{};
    int64_t x1 = cv_round_f(ax), y1 = cv_round_f(ay), x2 = cv_round_f(bx), y2 = cv_round_f(by);
    if ((uint64_t)x1 >= (uint64_t)W || (uint64_t)x2 >= (uint64_t)W || (uint64_t)y1 >= (uint64_t)H ||
        (uint64_t)y2 >= (uint64_t)H) {
        if (!clip_line(W, H, x1, y1, x2, y2)) {
            L.count = 0;
            return L;
        }
    }
    int64_t dx = x2 - x1, dy = y2 - y1;
    if (dx < 0) {  // left to right
        dx = -dx;
        dy = -dy;
        int64_t t = x1;
        x1 = x2;
        x2 = t;
        t = y1;
        y1 = y2;
        y2 = t;
    }
    const int sy = dy < 0 ? -1 : 1;
    if (dy < 0) dy = -dy;
    L.x0 = (int)x1;
    L.y0 = (int)y1;
    if (dy > dx) {  // vertical: y is the major axis
        L.dx = dy;
        L.dy = dx;
        L.mx = 0;
        L.my = sy;
        L.nx = 1;
        L.ny = 0;
    } else {
        L.dx = dx;
        L.dy = dy;
        L.mx = 1;
        L.my = 0;
        L.nx = 0;
        L.ny = sy;
    }
    L.count = (int)L.dx + 1;
    return L;
}

// draw_cube edge e (0..11) of a Solution: lower[i]-lower[i+1], upper[i]-upper[i+1], lower[i]-upper[i]
// in the reference's drawing order (draw.cpp:92-97)
DOFS_HDM inline void cube_edge(const dofs_solution& s, int e, float& ax, float& ay, float& bx, float& by) {
    const int i = e / 3, j = (i + 1) & 3, t = e % 3;
    const float(*a)[2] = t == 1 ? s.upper_face : s.lower_face;
    const float(*b)[2] = t == 0 ? s.lower_face : s.upper_face;
    const int ib = t == 2 ? i : j;
    ax = a[i][0];
    ay = a[i][1];
    bx = b[ib][0];
    by = b[ib][1];
}

// One element per (edge e, pixel step t) of a frame; it loops over the frame's snapshots, so the
// launch size (12 x (max(H, W) + 1) per frame) does not depend on the snapshot count.
struct KCubeLines {
    OverlayWs o;
    int steps;  // max(H, W) + 1 >= any clipped line's pixel count
    DOFS_HD void operator()(int f, int64_t i) const {
        const int e = (int)(i / steps);
        const int64_t t = i % steps;
        int n = o.ctr[(int64_t)f * kCounters + C_SNAP];
        if (n > o.snap_cap) n = o.snap_cap;
        for (int s = 0; s < n; ++s) {
            const dofs_snapshot& sn = o.snaps[(int64_t)f * o.snap_cap + s];
            if (!(sn.score > o.min_score) || !sn.sol.valid) continue;
            float ax, ay, bx, by;
            cube_edge(sn.sol, e, ax, ay, bx, by);
            const LineWalk L = line_walk(o.W, o.H, ax, ay, bx, by);
            if (t >= L.count) continue;
            int x, y;
            L.at(t, x, y);
            if ((unsigned)x >= (unsigned)o.W || (unsigned)y >= (unsigned)o.H) continue;  // never after clip_line
            dofs_amax(o.lmap + (int64_t)f * o.N + (int64_t)y * o.W + x, sn.slot);
        }
    }
};

// Per pixel: addWeighted(frame + edges, 0.6, seg, 0.4, 0)
struct KOverlay {
    OverlayWs o;
    DOFS_HD void operator()(int f, int64_t p) const {
        const int64_t g = (int64_t)f * o.N + p;
        const int P = o.labels[g], L = o.lmap[g];
        const unsigned char* src = o.frame + 3 * g;
        int fr[3] = {src[0], src[1], src[2]};
        int sg[3] = {fr[0], fr[1], fr[2]};
        if (L >= 0) {
            fr[0] = 255;
            fr[1] = fr[2] = 0;
        }
        if (L >= 0 && L >= P) {
            sg[0] = 255;
            sg[1] = sg[2] = 0;
        } else if (P >= 0) {
            int n = o.ctr[(int64_t)f * kCounters + C_SNAP];
            if (n > o.snap_cap) n = o.snap_cap;
            const dofs_snapshot* sn = o.snaps + (int64_t)f * o.snap_cap;
            int lo = 0, hi = n - 1;  // the snapshot of slot P (present: P is a qualifying slot)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (sn[mid].slot < P)
                    lo = mid + 1;
                else
                    hi = mid;
            }
            const int cls = sn[lo].sol.cls;
            sg[0] = 0;  // cls 0 and 2 (0,255,255), cls 1 (0,255,0) in BGR (draw.cpp:129-140)
            sg[1] = 255;
            sg[2] = cls == 1 ? 0 : 255;
        }
        unsigned char* dst = o.out + 3 * g;
        for (int c = 0; c < 3; ++c) dst[c] = (unsigned char)((6 * fr[c] + 4 * sg[c] + 5) / 10);
    }
};

}  // namespace dofs
