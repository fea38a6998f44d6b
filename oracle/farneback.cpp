// farneback.cpp — TEST INFRASTRUCTURE ONLY: CPU restatement of the step upstream of the hot path,
// cv::calcOpticalFlowFarneback as the reference calls it:
//   cv::cvtColor(im, gray, COLOR_BGR2GRAY)                                   cpp/src/segment.cpp:97-98
//   cv::calcOpticalFlowFarneback(gray1, gray2, flow, 0.5, 3, 15, 3, 5, 1.2, 0) cpp/src/segment.cpp:101,226
// OpenCV is not in this image and its version is unpinned (cpp/CMakeLists.txt:14), so this is a
// restatement of OpenCV 4.x's published algorithm (modules/video/src/optflowgf.cpp: the level loop,
// FarnebackPrepareGaussian, FarnebackPolyExp, FarnebackUpdateMatrices, FarnebackUpdateFlow_Blur;
// imgproc GaussianBlur / resize / cvtColor) in its scalar operation order, without FMA:
// PARITY UNPINNED against OpenCV itself (its SIMD paths may fuse or reassociate). The GPU
// implementation is checked bit-for-bit against this file.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../include/dofs.h"

namespace {

// cv::cvtColor(COLOR_BGR2GRAY) on 8-bit: fixed point with 14 fractional bits (R2Y 4899, G2Y 9617, B2Y 1868).
inline uint8_t bgr_gray(const uint8_t* p) { return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14); }

inline int cv_round(double v) { return (int)lrint(v); }  // cvRound: round half to even
inline int cv_floor(float v) {
    const int i = (int)v;
    return i - (i > v);
}
inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

// getGaussianKernel(n, sigma, CV_32F) of OpenCV 4.x (getGaussianKernelBitExact, then to float):
// the fixed small kernels for sigma <= 0, else exp(-x^2 / (2 sigma^2)) normalised with the centre
// tap = 1 - (sum of the others).
std::vector<float> gauss_kernel(int n, double sigma) {
    std::vector<float> k((size_t)n);
    if (sigma <= 0 && n == 3) {
        k[0] = 0.25f, k[1] = 0.5f, k[2] = 0.25f;
        return k;
    }
    if (sigma <= 0 && n == 1) {
        k[0] = 1.f;
        return k;
    }
    const double sx = sigma > 0 ? sigma : (double)n * 0.15 + 0.35;
    const double scale2 = -0.125 / (sx * sx);
    const int n2 = (n - 1) / 2;
    std::vector<double> v((size_t)n2 + 1);
    double sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        v[i] = exp((double)(x * x) * scale2);
        sum += v[i];
    }
    sum = sum * 2.0 + 1.0;
    const double mul = 1.0 / sum;
    double sum2 = 0.0;
    for (int i = 0; i < n2; i++) {
        v[i] *= mul;
        sum2 += v[i];
    }
    v[n2] = 1.0 - sum2 * 2.0;
    for (int i = 0; i <= n2; i++) k[i] = k[n - 1 - i] = (float)v[i];
    return k;
}

// GaussianBlur of a float image (BORDER_REFLECT_101), OpenCV's separable filter: for ksize 3 the
// small symmetric row/column filters, otherwise the generic row filter and the symmetric column filter.
void gauss_blur(const float* src, int H, int W, int ks, double sigma, float* dst) {
    const std::vector<float> k = gauss_kernel(ks, sigma);
    const int r = ks / 2;
    std::vector<float> t((size_t)H * W);
    for (int y = 0; y < H; ++y) {
        const float* s = src + (size_t)y * W;
        for (int x = 0; x < W; ++x) {
            float v;
            if (ks == 3) {  // SymmRowSmallFilter: S*k0 + (S[-1] + S[+1])*k1
                v = s[x] * k[1] + (s[reflect101(x - 1, W)] + s[reflect101(x + 1, W)]) * k[0];
            } else {  // RowFilter: k[0]*S[x-r] + k[1]*S[x-r+1] + ...
                v = k[0] * s[reflect101(x - r, W)];
                for (int i = 1; i < ks; ++i) v += k[i] * s[reflect101(x - r + i, W)];
            }
            t[(size_t)y * W + x] = v;
        }
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            float v;
            if (ks == 3) {  // SymmColumnSmallFilter: (S0 + S2)*k1 + S1*k0 + delta
                const float a = t[(size_t)reflect101(y - 1, H) * W + x], b = t[(size_t)reflect101(y + 1, H) * W + x];
                v = (a + b) * k[0] + t[(size_t)y * W + x] * k[1] + 0.0f;
            } else {  // SymmColumnFilter: k[c]*S0 + delta, += k[c+j]*(S[+j] + S[-j])
                v = k[r] * t[(size_t)y * W + x] + 0.0f;
                for (int j = 1; j <= r; ++j)
                    v += k[r + j] * (t[(size_t)reflect101(y + j, H) * W + x] + t[(size_t)reflect101(y - j, H) * W + x]);
            }
            dst[(size_t)y * W + x] = v;
        }
}

// cv::resize(src, dst, Size(dw, dh)) with INTER_LINEAR on float data (cn channels interleaved).
// dsize == ssize: copy. Exact 2x downscale: INTER_AREA fast path, ((a + b) + (c + d)) * 0.25f.
void resize_linear(const float* src, int sh, int sw, int cn, float* dst, int dh, int dw) {
    if (sh == dh && sw == dw) {
        memcpy(dst, src, sizeof(float) * (size_t)sh * sw * cn);
        return;
    }
    const double scale_x = (double)sw / dw, scale_y = (double)sh / dh;
    if (sw == 2 * dw && sh == 2 * dh) {
        for (int y = 0; y < dh; ++y)
            for (int x = 0; x < dw; ++x)
                for (int c = 0; c < cn; ++c) {
                    const float* s0 = src + ((size_t)(2 * y) * sw + 2 * x) * cn + c;
                    const float* s1 = s0 + (size_t)sw * cn;
                    dst[((size_t)y * dw + x) * cn + c] = ((s0[0] + s0[cn]) + (s1[0] + s1[cn])) * 0.25f;
                }
        return;
    }
    std::vector<int> xofs((size_t)dw);
    std::vector<float> ax((size_t)dw * 2);
    int xmin = 0, xmax = dw;
    for (int dx = 0; dx < dw; ++dx) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = cv_floor(fx);
        fx -= sx;
        if (sx < 0) {
            xmin = dx + 1;
            fx = 0, sx = 0;
        }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        ax[2 * dx] = 1.f - fx;
        ax[2 * dx + 1] = fx;
    }
    std::vector<float> rowbuf((size_t)dw * cn * 2);
    for (int dy = 0; dy < dh; ++dy) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = cv_floor(fy);
        fy -= sy;
        const float b0 = 1.f - fy, b1 = fy;
        for (int k = 0; k < 2; ++k) {  // HResizeLinear of source rows sy, sy + 1 (clipped)
            const int yy = std::min(std::max(sy + k, 0), sh - 1);
            const float* S = src + (size_t)yy * sw * cn;
            float* D = rowbuf.data() + (size_t)k * dw * cn;
            for (int dx = 0; dx < dw; ++dx)
                for (int c = 0; c < cn; ++c) {
                    const int s = xofs[dx] * cn + c;
                    D[dx * cn + c] = (dx < xmin || dx >= xmax) ? S[s] * ax[2 * dx] : S[s] * ax[2 * dx] + S[s + cn] * ax[2 * dx + 1];
                }
        }
        const float* S0 = rowbuf.data();
        const float* S1 = S0 + (size_t)dw * cn;
        for (int i = 0; i < dw * cn; ++i) dst[(size_t)dy * dw * cn + i] = S0[i] * b0 + S1[i] * b1;
    }
}

// OpenCV hal::Cholesky (CholImpl) solving A X = I: the inverse used by FarnebackPrepareGaussian.
void cholesky_inverse(double* A, int m, double* X) {
    double* L = A;
    for (int i = 0; i < m; i++) {
        int j;
        for (j = 0; j < i; j++) {
            double s = A[i * m + j];
            for (int k = 0; k < j; k++) s -= L[i * m + k] * L[j * m + k];
            L[i * m + j] = s * L[j * m + j];
        }
        double s = A[i * m + i];
        for (int k = 0; k < j; k++) {
            const double t = L[i * m + k];
            s -= t * t;
        }
        L[i * m + i] = 1. / sqrt(s);
    }
    for (int i = 0; i < m * m; ++i) X[i] = 0;
    for (int i = 0; i < m; ++i) X[i * m + i] = 1;
    for (int i = 0; i < m; i++)
        for (int j = 0; j < m; j++) {
            double s = X[i * m + j];
            for (int k = 0; k < i; k++) s -= L[i * m + k] * X[k * m + j];
            X[i * m + j] = s * L[i * m + i];
        }
    for (int i = m - 1; i >= 0; i--)
        for (int j = 0; j < m; j++) {
            double s = X[i * m + j];
            for (int k = m - 1; k > i; k--) s -= L[k * m + i] * X[k * m + j];
            X[i * m + j] = s * L[i * m + i];
        }
}

// FarnebackPrepareGaussian: g, xg, xxg indexed -n..n (arrays of 2n+1 with the centre at n).
void prepare_gaussian(int n, double sigma, float* g, float* xg, float* xxg, double ig[4]) {
    if (sigma < 1.1920929e-07) sigma = n * 0.3;
    double s = 0.;
    for (int x = -n; x <= n; x++) {
        g[x + n] = (float)exp(-x * x / (2 * sigma * sigma));
        s += g[x + n];
    }
    s = 1. / s;
    for (int x = -n; x <= n; x++) {
        g[x + n] = (float)(g[x + n] * s);
        xg[x + n] = (float)(x * g[x + n]);
        xxg[x + n] = (float)(x * x * g[x + n]);
    }
    double G[36] = {0};
    for (int y = -n; y <= n; y++)
        for (int x = -n; x <= n; x++) {
            const float gy = g[y + n], gx = g[x + n];
            G[0] += gy * gx;
            G[7] += gy * gx * x * x;
            G[21] += gy * gx * x * x * x * x;
            G[35] += gy * gx * x * x * y * y;
        }
    G[14] = G[3] = G[4] = G[18] = G[24] = G[7];  // (2,2) (0,3) (0,4) (3,0) (4,0) = (1,1)
    G[28] = G[21];                               // (4,4) = (3,3)
    G[22] = G[27] = G[35];                       // (3,4) (4,3) = (5,5)
    double inv[36];
    cholesky_inverse(G, 6, inv);
    ig[0] = inv[7];   // (1,1)
    ig[1] = inv[3];   // (0,3)
    ig[2] = inv[21];  // (3,3)
    ig[3] = inv[35];  // (5,5)
}

// FarnebackPolyExp: per pixel r2..r6 (5 floats), from a float image.
void poly_exp(const float* src, int H, int W, int n, double sigma, float* dst) {
    std::vector<float> kb((size_t)(2 * n + 1) * 3);
    float *g = kb.data() + n, *xg = g + 2 * n + 1, *xxg = xg + 2 * n + 1;
    double ig[4];
    prepare_gaussian(n, sigma, g - n, xg - n, xxg - n, ig);
    std::vector<float> rb((size_t)(W + 2 * n) * 3);
    float* row = rb.data() + n * 3;
    for (int y = 0; y < H; y++) {
        const float* s0 = src + (size_t)y * W;
        for (int x = 0; x < W; x++) {
            row[x * 3] = s0[x] * g[0];
            row[x * 3 + 1] = row[x * 3 + 2] = 0.f;
        }
        for (int k = 1; k <= n; k++) {
            const float g0 = g[k], g1 = xg[k], g2 = xxg[k];
            const float* a = src + (size_t)std::max(y - k, 0) * W;
            const float* b = src + (size_t)std::min(y + k, H - 1) * W;
            for (int x = 0; x < W; x++) {
                const float p = a[x] + b[x];
                const float t0 = row[x * 3] + g0 * p;
                const float t1 = row[x * 3 + 1] + g1 * (b[x] - a[x]);
                const float t2 = row[x * 3 + 2] + g2 * p;
                row[x * 3] = t0;
                row[x * 3 + 1] = t1;
                row[x * 3 + 2] = t2;
            }
        }
        for (int x = 0; x < n * 3; x++) {
            row[-1 - x] = row[2 - x];
            row[W * 3 + x] = row[W * 3 + x - 3];
        }
        float* d = dst + (size_t)y * W * 5;
        for (int x = 0; x < W; x++) {
            double b1 = row[x * 3] * g[0], b2 = 0, b3 = row[x * 3 + 1] * g[0], b4 = 0, b5 = row[x * 3 + 2] * g[0], b6 = 0;
            for (int k = 1; k <= n; k++) {
                const double tg = row[(x + k) * 3] + row[(x - k) * 3];
                const float g0 = g[k];
                b1 += tg * g0;
                b4 += tg * xxg[k];
                b2 += (row[(x + k) * 3] - row[(x - k) * 3]) * xg[k];
                b3 += (row[(x + k) * 3 + 1] + row[(x - k) * 3 + 1]) * g0;
                b6 += (row[(x + k) * 3 + 1] - row[(x - k) * 3 + 1]) * xg[k];
                b5 += (row[(x + k) * 3 + 2] + row[(x - k) * 3 + 2]) * g0;
            }
            d[x * 5 + 1] = (float)(b2 * ig[0]);
            d[x * 5] = (float)(b3 * ig[0]);
            d[x * 5 + 3] = (float)(b1 * ig[1] + b4 * ig[2]);
            d[x * 5 + 2] = (float)(b1 * ig[1] + b5 * ig[2]);
            d[x * 5 + 4] = (float)(b6 * ig[3]);
        }
    }
}

// FarnebackUpdateMatrices for rows [y0, y1).
void update_matrices(const float* R0, const float* R1, const float* flow, int H, int W, float* M, int y0, int y1) {
    static const float border[5] = {0.14f, 0.14f, 0.4472f, 0.4472f, 0.4472f};
    for (int y = y0; y < y1; y++) {
        const float* fl = flow + (size_t)y * W * 2;
        const float* r0 = R0 + (size_t)y * W * 5;
        float* m = M + (size_t)y * W * 5;
        for (int x = 0; x < W; x++) {
            const float dx = fl[x * 2], dy = fl[x * 2 + 1];
            float fx = x + dx, fy = y + dy;
            const int x1 = cv_floor(fx), y1_ = cv_floor(fy);
            float r2, r3, r4, r5, r6;
            fx -= x1;
            fy -= y1_;
            if ((unsigned)x1 < (unsigned)(W - 1) && (unsigned)y1_ < (unsigned)(H - 1)) {
                const float* p = R1 + ((size_t)y1_ * W + x1) * 5;
                const size_t st = (size_t)W * 5;
                const float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
                r2 = a00 * p[0] + a01 * p[5] + a10 * p[st] + a11 * p[st + 5];
                r3 = a00 * p[1] + a01 * p[6] + a10 * p[st + 1] + a11 * p[st + 6];
                r4 = a00 * p[2] + a01 * p[7] + a10 * p[st + 2] + a11 * p[st + 7];
                r5 = a00 * p[3] + a01 * p[8] + a10 * p[st + 3] + a11 * p[st + 8];
                r6 = a00 * p[4] + a01 * p[9] + a10 * p[st + 4] + a11 * p[st + 9];
                r4 = (r0[x * 5 + 2] + r4) * 0.5f;
                r5 = (r0[x * 5 + 3] + r5) * 0.5f;
                r6 = (r0[x * 5 + 4] + r6) * 0.25f;
            } else {
                r2 = r3 = 0.f;
                r4 = r0[x * 5 + 2];
                r5 = r0[x * 5 + 3];
                r6 = r0[x * 5 + 4] * 0.5f;
            }
            r2 = (r0[x * 5] - r2) * 0.5f;
            r3 = (r0[x * 5 + 1] - r3) * 0.5f;
            r2 += r4 * dy + r6 * dx;
            r3 += r6 * dy + r5 * dx;
            if ((unsigned)(x - 5) >= (unsigned)(W - 10) || (unsigned)(y - 5) >= (unsigned)(H - 10)) {
                const float sc = (x < 5 ? border[x] : 1.f) * (x >= W - 5 ? border[W - x - 1] : 1.f) *
                                 (y < 5 ? border[y] : 1.f) * (y >= H - 5 ? border[H - y - 1] : 1.f);
                r2 *= sc;
                r3 *= sc;
                r4 *= sc;
                r5 *= sc;
                r6 *= sc;
            }
            m[x * 5] = r4 * r4 + r6 * r6;
            m[x * 5 + 1] = (r4 + r5) * r6;
            m[x * 5 + 2] = r5 * r5 + r6 * r6;
            m[x * 5 + 3] = r4 * r2 + r6 * r3;
            m[x * 5 + 4] = r6 * r2 + r5 * r3;
        }
    }
}

// FarnebackUpdateFlow_Blur: box filter of M by running double sums (vertical then horizontal), flow
// = G^-1 h per pixel; then (all but the last iteration) M from the new flow. The reference updates
// M in row stripes behind the running window; every row is rewritten only after the window has
// passed it, so this equals "all flow rows, then all M rows".
void update_flow_blur(const float* R0, const float* R1, float* flow, float* M, int H, int W, int bs, bool upd) {
    const int m = bs / 2;
    const double scale = 1. / (bs * bs);
    std::vector<double> vb((size_t)(W + m * 2 + 2) * 5);
    double* vsum = vb.data() + (m + 1) * 5;
    const float* s0 = M;
    for (int x = 0; x < W * 5; x++) vsum[x] = s0[x] * (m + 2);
    for (int y = 1; y < m; y++) {
        s0 = M + (size_t)std::min(y, H - 1) * W * 5;
        for (int x = 0; x < W * 5; x++) vsum[x] += s0[x];
    }
    for (int y = 0; y < H; y++) {
        float* fl = flow + (size_t)y * W * 2;
        s0 = M + (size_t)std::max(y - m - 1, 0) * W * 5;
        const float* s1 = M + (size_t)std::min(y + m, H - 1) * W * 5;
        for (int x = 0; x < W * 5; x++) vsum[x] += s1[x] - s0[x];
        for (int x = 0; x < (m + 1) * 5; x++) {
            vsum[-1 - x] = vsum[4 - x];
            vsum[W * 5 + x] = vsum[W * 5 + x - 5];
        }
        double g11 = vsum[0] * (m + 2), g12 = vsum[1] * (m + 2), g22 = vsum[2] * (m + 2), h1 = vsum[3] * (m + 2),
               h2 = vsum[4] * (m + 2);
        for (int x = 1; x < m; x++) {
            g11 += vsum[x * 5];
            g12 += vsum[x * 5 + 1];
            g22 += vsum[x * 5 + 2];
            h1 += vsum[x * 5 + 3];
            h2 += vsum[x * 5 + 4];
        }
        for (int x = 0; x < W; x++) {
            g11 += vsum[(x + m) * 5] - vsum[(x - m) * 5 - 5];
            g12 += vsum[(x + m) * 5 + 1] - vsum[(x - m) * 5 - 4];
            g22 += vsum[(x + m) * 5 + 2] - vsum[(x - m) * 5 - 3];
            h1 += vsum[(x + m) * 5 + 3] - vsum[(x - m) * 5 - 2];
            h2 += vsum[(x + m) * 5 + 4] - vsum[(x - m) * 5 - 1];
            const double g11_ = g11 * scale, g12_ = g12 * scale, g22_ = g22 * scale, h1_ = h1 * scale, h2_ = h2 * scale;
            const double idet = 1. / (g11_ * g22_ - g12_ * g12_ + 1e-3);
            fl[x * 2] = (float)((g11_ * h2_ - g12_ * h1_) * idet);
            fl[x * 2 + 1] = (float)((g22_ * h1_ - g12_ * h2_) * idet);
        }
    }
    if (upd) update_matrices(R0, R1, flow, H, W, M, 0, H);
}

}  // namespace

extern "C" {

void oracle_bgr_to_gray(const uint8_t* bgr, int32_t H, int32_t W, uint8_t* gray) {
    for (int64_t i = 0; i < (int64_t)H * W; ++i) gray[i] = bgr_gray(bgr + 3 * i);
}

// Exposed stages (for the unit tests of the GPU stages).
void oracle_fb_gauss_kernel(int32_t n, double sigma, float* out) {
    const std::vector<float> k = gauss_kernel(n, sigma);
    for (int i = 0; i < n; ++i) out[i] = k[i];
}
void oracle_fb_poly_consts(int32_t n, double sigma, float* g, float* xg, float* xxg, double ig[4]) {
    prepare_gaussian(n, sigma, g, xg, xxg, ig);
}
void oracle_fb_blur(const float* src, int32_t H, int32_t W, int32_t ks, double sigma, float* dst) {
    gauss_blur(src, H, W, ks, sigma, dst);
}
void oracle_fb_resize(const float* src, int32_t sh, int32_t sw, int32_t cn, float* dst, int32_t dh, int32_t dw) {
    resize_linear(src, sh, sw, cn, dst, dh, dw);
}
void oracle_fb_poly_exp(const float* src, int32_t H, int32_t W, int32_t n, double sigma, float* dst) {
    poly_exp(src, H, W, n, sigma, dst);
}

// calcOpticalFlowFarneback(prev, next, flow, pyr_scale, levels, winsize, iterations, poly_n,
// poly_sigma, flags = 0) on 8-bit single-channel frames; flow = H x W x 2 float. Returns the number
// of pyramid levels used + 1, or -1 for unsupported flags.
int32_t oracle_farneback(const uint8_t* prev, const uint8_t* next, int32_t rows, int32_t cols, double pyr_scale,
                         int32_t levels, int32_t winsize, int32_t iterations, int32_t poly_n, double poly_sigma,
                         int32_t flags, float* flow0) {
    if (flags != 0) return -1;
    const int min_size = 32;
    int k;
    double scale = 1;
    for (k = 0; k < levels; k++) {
        scale *= pyr_scale;
        if (cols * scale < min_size || rows * scale < min_size) break;
    }
    levels = k;
    const size_t N0 = (size_t)rows * cols;
    std::vector<float> fimg[2], blurred(N0), prev_flow;
    for (int i = 0; i < 2; ++i) {
        const uint8_t* im = i ? next : prev;
        fimg[i].resize(N0);
        for (size_t p = 0; p < N0; ++p) fimg[i][p] = (float)im[p];
    }
    int pw = 0, ph = 0;
    for (k = levels; k >= 0; k--) {
        scale = 1;
        for (int i = 0; i < k; i++) scale *= pyr_scale;
        const double sigma = (1. / scale - 1) * 0.5;
        int smooth_sz = cv_round(sigma * 5) | 1;
        smooth_sz = std::max(smooth_sz, 3);
        const int width = cv_round(cols * scale), height = cv_round(rows * scale);
        const size_t N = (size_t)width * height;
        std::vector<float> flow(N * 2, 0.f);
        if (!prev_flow.empty()) {
            resize_linear(prev_flow.data(), ph, pw, 2, flow.data(), height, width);
            const float s = (float)(1. / pyr_scale);
            for (size_t i = 0; i < N * 2; ++i) flow[i] = flow[i] * s + 0.0f;
        }
        std::vector<float> R[2], I(N), M(N * 5);
        for (int i = 0; i < 2; i++) {
            gauss_blur(fimg[i].data(), rows, cols, smooth_sz, sigma, blurred.data());
            resize_linear(blurred.data(), rows, cols, 1, I.data(), height, width);
            R[i].resize(N * 5);
            poly_exp(I.data(), height, width, poly_n, poly_sigma, R[i].data());
        }
        update_matrices(R[0].data(), R[1].data(), flow.data(), height, width, M.data(), 0, height);
        for (int i = 0; i < iterations; i++)
            update_flow_blur(R[0].data(), R[1].data(), flow.data(), M.data(), height, width, winsize, i < iterations - 1);
        prev_flow.swap(flow);
        pw = width;
        ph = height;
    }
    memcpy(flow0, prev_flow.data(), sizeof(float) * N0 * 2);
    return levels + 1;
}

}  // extern "C"
