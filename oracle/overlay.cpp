// overlay.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the step downstream of the hot path
// (SURVEY.md §8(f) #2), in the reference's own loop order:
//   plot_best_segments_simple(frame, bev, forest, 0.7)   cpp/src/draw.cpp:101-160
//   draw_cube(im, lower_face, upper_face, color, lw)     cpp/src/draw.cpp:85-99
// with the OpenCV operators it calls restated from OpenCV 4.x (imgproc/src/drawing.cpp:
// cv::line -> ThickLine -> Line -> LineIterator (8-connected, left to right) and clipLine;
// core arithm addWeighted on 8U: saturate_cast<uchar>(a * alpha + b * beta + gamma), float weights).
// The walk is the iterative Bresenham of LineIterator (err / plusDelta / minusDelta), not the closed
// form the GPU uses. OpenCV is absent here and unpinned (cpp/CMakeLists.txt:14): PARITY UNPINNED
// against OpenCV itself; the GPU path is checked bit-for-bit against this file.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <utility>
#include <vector>

#include "../include/dofs.h"

namespace {

// saturate_cast<int>(float) == cvRound(float) on x86-64 (cvtss2si: nearest-even, 0x80000000 when
// the value is NaN or does not fit)
int cv_round(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return INT32_MIN;
    return (int)nearbyintf(v);
}

bool clip_line(int64_t w, int64_t h, int64_t& x1, int64_t& y1, int64_t& x2, int64_t& y2) {
    if (w <= 0 || h <= 0) return false;
    int64_t right = w - 1, bottom = h - 1;
    int c1 = (x1 < 0) + (x1 > right) * 2 + (y1 < 0) * 4 + (y1 > bottom) * 8;
    int c2 = (x2 < 0) + (x2 > right) * 2 + (y2 < 0) * 4 + (y2 > bottom) * 8;
    if ((c1 & c2) == 0 && (c1 | c2) != 0) {
        int64_t a;
        if (c1 & 12) {
            a = c1 < 8 ? 0 : bottom;
            x1 += (int64_t)((double)(a - y1) * (x2 - x1) / (y2 - y1));
            y1 = a;
            c1 = (x1 < 0) + (x1 > right) * 2;
        }
        if (c2 & 12) {
            a = c2 < 8 ? 0 : bottom;
            x2 += (int64_t)((double)(a - y2) * (x2 - x1) / (y2 - y1));
            y2 = a;
            c2 = (x2 < 0) + (x2 > right) * 2;
        }
        if ((c1 & c2) == 0 && (c1 | c2) != 0) {
            if (c1) {
                a = c1 == 1 ? 0 : right;
                y1 += (int64_t)((double)(a - x1) * (y2 - y1) / (x2 - x1));
                x1 = a;
                c1 = 0;
            }
            if (c2) {
                a = c2 == 1 ? 0 : right;
                y2 += (int64_t)((double)(a - x2) * (y2 - y1) / (x2 - x1));
                x2 = a;
                c2 = 0;
            }
        }
    }
    return (c1 | c2) == 0;
}

struct Img {
    uint8_t* p;
    int H, W;
    uint8_t* at(int x, int y) { return p + ((size_t)y * W + x) * 3; }
};

// cv::line(img, Point(a), Point(b), color, 1, LINE_8, 0): ThickLine with thickness 1 and shift 0
// reduces to Line(img, p0, p1, color, 8) — a LineIterator walk writing every pixel.
void cv_line(Img& img, float ax, float ay, float bx, float by, const uint8_t color[3]) {
    int64_t x1 = cv_round(ax), y1 = cv_round(ay), x2 = cv_round(bx), y2 = cv_round(by);
    if ((unsigned)x1 >= (unsigned)img.W || (unsigned)x2 >= (unsigned)img.W || (unsigned)y1 >= (unsigned)img.H ||
        (unsigned)y2 >= (unsigned)img.H) {
        if (!clip_line(img.W, img.H, x1, y1, x2, y2)) return;  // count = 0
    }
    int px = (int)x1, py = (int)y1, qx = (int)x2, qy = (int)y2;
    int dx = qx - px, dy = qy - py;
    if (dx < 0) {  // leftToRight
        dx = -dx;
        dy = -dy;
        std::swap(px, qx);
        std::swap(py, qy);
    }
    int sx = 1, sy = 1;  // steps along x and y
    if (dy < 0) {
        dy = -dy;
        sy = -1;
    }
    const bool vert = dy > dx;
    // minus step (every iteration) along the major axis, plus step (err < 0) along the minor axis
    int minus_x = sx, minus_y = 0, plus_x = 0, plus_y = sy;
    if (vert) {
        std::swap(dx, dy);
        minus_x = 0;
        minus_y = sy;
        plus_x = sx;
        plus_y = 0;
    }
    int err = dx - (dy + dy);
    const int plusDelta = dx + dx, minusDelta = -(dy + dy);
    const int count = dx + 1;
    int x = px, y = py;
    for (int i = 0; i < count; ++i) {
        if ((unsigned)x < (unsigned)img.W && (unsigned)y < (unsigned)img.H) memcpy(img.at(x, y), color, 3);
        const int mask = err < 0 ? -1 : 0;
        err += minusDelta + (plusDelta & mask);
        x += minus_x + (plus_x & mask);
        y += minus_y + (plus_y & mask);
    }
}

void draw_cube(Img& im, const dofs_solution& s, const uint8_t color[3]) {
    for (int i = 0; i < 4; ++i) {
        const int j = (i + 1) % 4;
        cv_line(im, s.lower_face[i][0], s.lower_face[i][1], s.lower_face[j][0], s.lower_face[j][1], color);
        cv_line(im, s.upper_face[i][0], s.upper_face[i][1], s.upper_face[j][0], s.upper_face[j][1], color);
        cv_line(im, s.lower_face[i][0], s.lower_face[i][1], s.upper_face[i][0], s.upper_face[i][1], color);
    }
}

}  // namespace

extern "C" {

// One cv::line(img, a, b, color, 1) on an H x W mask: covered pixels set to 1.
void oracle_line(int32_t H, int32_t W, float ax, float ay, float bx, float by, uint8_t* mask) {
    std::vector<uint8_t> img((size_t)H * W * 3, 0);
    Img I{img.data(), H, W};
    const uint8_t one[3] = {1, 1, 1};
    cv_line(I, ax, ay, bx, by, one);
    for (size_t i = 0; i < (size_t)H * W; ++i) mask[i] = img[3 * i];
}

// plot_best_segments_simple on one frame: `snaps` = the non-empty history slots (ascending slot; the
// empty slots of get_best_segments have score -1 and draw nothing), members of snapshot k =
// leaf_order[seg_begin .. seg_begin + size). frame / out: H x W x 3 BGR, packed.
void oracle_overlay(const uint8_t* frame, int32_t H, int32_t W, const dofs_snapshot* snaps, int32_t n,
                    const int32_t* leaf_order, double min_score, uint8_t* out) {
    const size_t bytes = (size_t)H * W * 3;
    std::vector<uint8_t> fr(frame, frame + bytes), sg(frame, frame + bytes);  // frame, seg = frame.clone()
    Img F{fr.data(), H, W}, S{sg.data(), H, W};
    const uint8_t blue[3] = {255, 0, 0};
    for (int k = 0; k < n; ++k) {
        const dofs_snapshot& s = snaps[k];
        if (!(s.score > min_score)) continue;
        uint8_t color[3];
        if (s.sol.cls == 1) {
            color[0] = 0, color[1] = 255, color[2] = 0;  // Green
        } else {
            color[0] = 0, color[1] = 255, color[2] = 255;  // Yellow (cls 0), "Mint" (cls 2)
        }
        for (int32_t t = 0; t < s.size; ++t) {
            const int id = leaf_order[s.seg_begin + t];
            memcpy(S.at(id % W, id / W), color, 3);
        }
        if (s.sol.valid) {  // draw_cube returns early on empty faces (draw.cpp:89-92)
            draw_cube(F, s.sol, blue);
            draw_cube(S, s.sol, blue);
        }
    }
    const double opacity = 2.0 / 5.0;
    const float alpha = (float)(1.0 - opacity), beta = (float)opacity, gamma = 0.0f;
    for (size_t i = 0; i < bytes; ++i) {
        const float v = (float)fr[i] * alpha + (float)sg[i] * beta + gamma;
        const int r = cv_round(v);
        out[i] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    }
}

}  // extern "C"
