// dofs_flow.h — the step upstream of the hot path: dense optical flow (cv::calcOpticalFlowFarneback
// as the reference calls it, cpp/src/segment.cpp:101,226: pyr_scale 0.5, levels 3, winsize 15,
// iterations 3, poly_n 5, poly_sigma 1.2, flags 0) and cv::cvtColor(BGR2GRAY) (segment.cpp:97-98),
// on batches of device-resident 8-bit frame pairs. SURVEY.md §8(f) #1.
//
// Same arithmetic, operation for operation, as the oracle restatement (oracle/farneback.cpp;
// OpenCV 4.x optflowgf.cpp + the imgproc filters, scalar order, no FMA — this TU is compiled with
// -ffp-contract=off), so the GPU flow is bit-identical to it. Per pyramid level and image:
//   FB1 row Gaussian (u8 in)  FB2 column Gaussian  FB3 resize (INTER_LINEAR / 2x INTER_AREA)
//   FB4 polynomial expansion, vertical  FB5 horizontal (5 coefficients per pixel)
// per level and frame: FB6 UpdateMatrices, then `iterations` x (FB7 box filter, vertical running
// sums — one lane per column channel, sequential in y like the reference's double accumulators;
// FB8 horizontal running sums — one wave per row, the five sequential chains on five lanes over
// 64-pixel chunks staged in LDS, then the per-pixel 2x2 solve; FB6 again except after the last).
// Everything here is HBM/latency-bound elementwise and stencil work: no MFMA.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <vector>

namespace dofs {
namespace flow {

constexpr int kMaxTaps = 32;  // Gaussian pre-blur taps (ksize <= 31: pyramid levels <= 5)
constexpr int kMaxPolyN = 7;

struct Taps {
    float k[kMaxTaps];
    int n;
};
struct PolyConsts {
    float g[kMaxPolyN + 1], xg[kMaxPolyN + 1], xxg[kMaxPolyN + 1];  // index 0..n (symmetric)
    double ig11, ig03, ig33, ig55;
    int n;
};

// ---- host constants (restated from the published algorithm; the oracle is a separate restatement)
inline int cv_round(double v) { return (int)lrint(v); }

inline Taps gauss_taps(int n, double sigma) {  // getGaussianKernel(n, sigma, CV_32F), OpenCV 4.x
    Taps t{};
    t.n = n;
    if (sigma <= 0 && n == 3) {
        t.k[0] = 0.25f, t.k[1] = 0.5f, t.k[2] = 0.25f;
        return t;
    }
    const double sx = sigma > 0 ? sigma : (double)n * 0.15 + 0.35;
    const double scale2 = -0.125 / (sx * sx);
    const int n2 = (n - 1) / 2;
    double v[kMaxTaps];
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
    for (int i = 0; i <= n2; i++) t.k[i] = t.k[n - 1 - i] = (float)v[i];
    return t;
}

inline PolyConsts poly_consts(int n, double sigma) {  // FarnebackPrepareGaussian
    PolyConsts c{};
    c.n = n;
    if (sigma < 1.1920929e-07) sigma = n * 0.3;
    float g[2 * kMaxPolyN + 1];
    double s = 0.;
    for (int x = -n; x <= n; x++) {
        g[x + n] = (float)exp(-x * x / (2 * sigma * sigma));
        s += g[x + n];
    }
    s = 1. / s;
    for (int x = -n; x <= n; x++) g[x + n] = (float)(g[x + n] * s);
    for (int x = 0; x <= n; x++) {
        c.g[x] = g[x + n];
        c.xg[x] = (float)(x * g[x + n]);
        c.xxg[x] = (float)(x * x * g[x + n]);
    }
    double G[6][6] = {};
    for (int y = -n; y <= n; y++)
        for (int x = -n; x <= n; x++) {
            const float gy = g[y + n], gx = g[x + n];
            G[0][0] += gy * gx;
            G[1][1] += gy * gx * x * x;
            G[3][3] += gy * gx * x * x * x * x;
            G[5][5] += gy * gx * x * x * y * y;
        }
    G[2][2] = G[0][3] = G[0][4] = G[3][0] = G[4][0] = G[1][1];
    G[4][4] = G[3][3];
    G[3][4] = G[4][3] = G[5][5];
    // G.inv(DECOMP_CHOLESKY): L L^T X = I (hal::Cholesky order; diagonal kept inverted)
    double L[6][6], X[6][6];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) L[i][j] = G[i][j], X[i][j] = i == j;
    for (int i = 0; i < 6; i++) {
        for (int j = 0; j < i; j++) {
            double a = L[i][j];
            for (int k = 0; k < j; k++) a -= L[i][k] * L[j][k];
            L[i][j] = a * L[j][j];
        }
        double a = L[i][i];
        for (int k = 0; k < i; k++) a -= L[i][k] * L[i][k];
        L[i][i] = 1. / sqrt(a);
    }
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) {
            double a = X[i][j];
            for (int k = 0; k < i; k++) a -= L[i][k] * X[k][j];
            X[i][j] = a * L[i][i];
        }
    for (int i = 5; i >= 0; i--)
        for (int j = 0; j < 6; j++) {
            double a = X[i][j];
            for (int k = 5; k > i; k--) a -= L[k][i] * X[k][j];
            X[i][j] = a * L[i][i];
        }
    c.ig11 = X[1][1];
    c.ig03 = X[0][3];
    c.ig33 = X[3][3];
    c.ig55 = X[5][5];
    return c;
}

// ---- device helpers ------------------------------------------------------------------------------
__device__ inline int refl101(int p, int n) {
    if (n == 1) return 0;
    while ((unsigned)p >= (unsigned)n) p = p < 0 ? -p : 2 * n - p - 2;
    return p;
}
__device__ inline int fl_floor(float v) {
    const int i = (int)v;
    return i - (i > v);
}
__device__ inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Image i of a batch of B frame pairs: i = 2f + (0 prev | 1 next).
struct Pair {
    const unsigned char* prev;
    const unsigned char* next;
    __device__ const unsigned char* img(int i, int64_t n) const { return ((i & 1) ? next : prev) + (int64_t)(i >> 1) * n; }
};

// FB1: u8 -> float, GaussianBlur row pass (ksize 3: SymmRowSmallFilter; else RowFilter), reflect-101.
__global__ __launch_bounds__(256) void k_fb_blur_row(Pair in, int H, int W, Taps t, float* tmp) {
    const int i = blockIdx.y;
    const int64_t n = (int64_t)H * W;
    const unsigned char* s = in.img(i, n);
    float* d = tmp + i * n;
    const int r = t.n / 2;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p % W);
        const unsigned char* row = s + (int64_t)y * W;
        float v;
        if (t.n == 3) {
            v = (float)row[x] * t.k[1] + ((float)row[refl101(x - 1, W)] + (float)row[refl101(x + 1, W)]) * t.k[0];
        } else {
            v = t.k[0] * (float)row[refl101(x - r, W)];
            for (int k = 1; k < t.n; ++k) v += t.k[k] * (float)row[refl101(x - r + k, W)];
        }
        d[p] = v;
    }
}

// FB2: column pass (ksize 3: SymmColumnSmallFilter; else SymmColumnFilter), delta 0.
__global__ __launch_bounds__(256) void k_fb_blur_col(const float* tmp, int H, int W, Taps t, float* out) {
    const int i = blockIdx.y;
    const int64_t n = (int64_t)H * W;
    const float* s = tmp + i * n;
    float* d = out + i * n;
    const int r = t.n / 2;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p % W);
        float v;
        if (t.n == 3) {
            v = (s[(int64_t)refl101(y - 1, H) * W + x] + s[(int64_t)refl101(y + 1, H) * W + x]) * t.k[0] + s[p] * t.k[1] +
                0.0f;
        } else {
            v = t.k[r] * s[p] + 0.0f;
            for (int j = 1; j <= r; ++j)
                v += t.k[r + j] * (s[(int64_t)refl101(y + j, H) * W + x] + s[(int64_t)refl101(y - j, H) * W + x]);
        }
        d[p] = v;
    }
}

// cv::resize INTER_LINEAR, one destination element (channel c of pixel (dx, dy)); cn channels.
__device__ inline float resize_px(const float* src, int sh, int sw, int cn, int dh, int dw, int dx, int dy, int c) {
    if (sw == 2 * dw && sh == 2 * dh) {  // INTER_LINEAR at exactly 1/2 is INTER_AREA's fast path
        const float* s0 = src + ((int64_t)(2 * dy) * sw + 2 * dx) * cn + c;
        const float* s1 = s0 + (int64_t)sw * cn;
        return ((s0[0] + s0[cn]) + (s1[0] + s1[cn])) * 0.25f;
    }
    const double scale_x = (double)sw / dw, scale_y = (double)sh / dh;
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = fl_floor(fx);
    fx -= sx;
    bool one = false;
    if (sx < 0) one = true, fx = 0, sx = 0;
    if (sx + 1 >= sw) one = true, fx = 0, sx = sw - 1;
    const float a0 = 1.f - fx, a1 = fx;
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    const int sy = fl_floor(fy);
    fy -= sy;
    float r[2];
    for (int k = 0; k < 2; ++k) {
        const float* S = src + (int64_t)clampi(sy + k, 0, sh - 1) * sw * cn;
        const int s = sx * cn + c;
        r[k] = one ? S[s] * a0 : S[s] * a0 + S[s + cn] * a1;
    }
    return r[0] * (1.f - fy) + r[1] * fy;
}

// FB3: image to the level size (a copy when the sizes agree).
__global__ __launch_bounds__(256) void k_fb_resize(const float* src, int sh, int sw, float* dst, int dh, int dw) {
    const int i = blockIdx.y;
    const float* s = src + (int64_t)i * sh * sw;
    float* d = dst + (int64_t)i * dh * dw;
    const int64_t n = (int64_t)dh * dw;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / dw), x = (int)(p % dw);
        d[p] = (sh == dh && sw == dw) ? s[p] : resize_px(s, sh, sw, 1, dh, dw, x, y, 0);
    }
}

// Flow of the previous (coarser) level up to this level: resize (2 channels) then *= 1/pyr_scale.
__global__ __launch_bounds__(256) void k_fb_flow_up(const float* src, int sh, int sw, float* dst, int dh, int dw,
                                                    float s) {
    const int f = blockIdx.y;
    const float* a = src + (int64_t)f * sh * sw * 2;
    float* d = dst + (int64_t)f * dh * dw * 2;
    const int64_t n = (int64_t)dh * dw * 2;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(p & 1);
        const int64_t q = p >> 1;
        const int y = (int)(q / dw), x = (int)(q % dw);
        d[p] = resize_px(a, sh, sw, 2, dh, dw, x, y, c) * s + 0.0f;
    }
}

// FB4: polynomial expansion, vertical part: per pixel (row0, row1, row2) of the reference's row buffer.
__global__ __launch_bounds__(256) void k_fb_poly_v(const float* img, int H, int W, PolyConsts pc, float* vt) {
    const int i = blockIdx.y;
    const int64_t n = (int64_t)H * W;
    const float* s = img + i * n;
    float* d = vt + i * n * 3;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p % W);
        float r0 = s[p] * pc.g[0], r1 = 0.f, r2 = 0.f;
        for (int k = 1; k <= pc.n; k++) {
            const float a = s[(int64_t)max(y - k, 0) * W + x], b = s[(int64_t)min(y + k, H - 1) * W + x];
            const float q = a + b;
            r0 = r0 + pc.g[k] * q;
            r1 = r1 + pc.xg[k] * (b - a);
            r2 = r2 + pc.xxg[k] * q;
        }
        d[p * 3] = r0;
        d[p * 3 + 1] = r1;
        d[p * 3 + 2] = r2;
    }
}

// FB5: horizontal part (double accumulators), replicate border; R = 5 floats per pixel.
__global__ __launch_bounds__(256) void k_fb_poly_h(const float* vt, int H, int W, PolyConsts pc, float* R) {
    const int i = blockIdx.y;
    const int64_t n = (int64_t)H * W;
    const float* s = vt + i * n * 3;
    float* d = R + i * n * 5;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int x = (int)(p % W);
        const float* row = s + (p - x) * 3;
        double b1 = row[x * 3] * pc.g[0], b2 = 0, b3 = row[x * 3 + 1] * pc.g[0], b4 = 0, b5 = row[x * 3 + 2] * pc.g[0],
               b6 = 0;
        for (int k = 1; k <= pc.n; k++) {
            const int xp = min(x + k, W - 1) * 3, xm = max(x - k, 0) * 3;
            const double tg = row[xp] + row[xm];
            const float g0 = pc.g[k];
            b1 += tg * g0;
            b4 += tg * pc.xxg[k];
            b2 += (row[xp] - row[xm]) * pc.xg[k];
            b3 += (row[xp + 1] + row[xm + 1]) * g0;
            b6 += (row[xp + 1] - row[xm + 1]) * pc.xg[k];
            b5 += (row[xp + 2] + row[xm + 2]) * g0;
        }
        d[p * 5 + 1] = (float)(b2 * pc.ig11);
        d[p * 5] = (float)(b3 * pc.ig11);
        d[p * 5 + 3] = (float)(b1 * pc.ig03 + b4 * pc.ig33);
        d[p * 5 + 2] = (float)(b1 * pc.ig03 + b5 * pc.ig33);
        d[p * 5 + 4] = (float)(b6 * pc.ig55);
    }
}

// FB6: FarnebackUpdateMatrices (frame f: R of images 2f, 2f+1).
__global__ __launch_bounds__(256) void k_fb_update_matrices(const float* R, const float* flow, int H, int W, float* M) {
    const int f = blockIdx.y;
    const int64_t n = (int64_t)H * W;
    const float* R0 = R + (int64_t)(2 * f) * n * 5;
    const float* R1 = R0 + n * 5;
    const float* fl = flow + (int64_t)f * n * 2;
    float* m = M + (int64_t)f * n * 5;
    const float border[5] = {0.14f, 0.14f, 0.4472f, 0.4472f, 0.4472f};
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const int y = (int)(p / W), x = (int)(p % W);
        const float dx = fl[p * 2], dy = fl[p * 2 + 1];
        float fx = x + dx, fy = y + dy;
        const int x1 = fl_floor(fx), y1 = fl_floor(fy);
        float r2, r3, r4, r5, r6;
        fx -= x1;
        fy -= y1;
        const float* r0 = R0 + p * 5;
        if ((unsigned)x1 < (unsigned)(W - 1) && (unsigned)y1 < (unsigned)(H - 1)) {
            const float* q = R1 + ((int64_t)y1 * W + x1) * 5;
            const int64_t st = (int64_t)W * 5;
            const float a00 = (1.f - fx) * (1.f - fy), a01 = fx * (1.f - fy), a10 = (1.f - fx) * fy, a11 = fx * fy;
            r2 = a00 * q[0] + a01 * q[5] + a10 * q[st] + a11 * q[st + 5];
            r3 = a00 * q[1] + a01 * q[6] + a10 * q[st + 1] + a11 * q[st + 6];
            r4 = a00 * q[2] + a01 * q[7] + a10 * q[st + 2] + a11 * q[st + 7];
            r5 = a00 * q[3] + a01 * q[8] + a10 * q[st + 3] + a11 * q[st + 8];
            r6 = a00 * q[4] + a01 * q[9] + a10 * q[st + 4] + a11 * q[st + 9];
            r4 = (r0[2] + r4) * 0.5f;
            r5 = (r0[3] + r5) * 0.5f;
            r6 = (r0[4] + r6) * 0.25f;
        } else {
            r2 = r3 = 0.f;
            r4 = r0[2];
            r5 = r0[3];
            r6 = r0[4] * 0.5f;
        }
        r2 = (r0[0] - r2) * 0.5f;
        r3 = (r0[1] - r3) * 0.5f;
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
        float* o = m + p * 5;
        o[0] = r4 * r4 + r6 * r6;
        o[1] = (r4 + r5) * r6;
        o[2] = r5 * r5 + r6 * r6;
        o[3] = r4 * r2 + r6 * r3;
        o[4] = r6 * r2 + r5 * r3;
    }
}

// FB7: box filter, vertical running sums (double), one lane per (column, channel): V[y] = the
// reference's vsum after row y. Sequential in y, as the reference accumulates.
__global__ __launch_bounds__(256) void k_fb_box_v(const float* M, int H, int W, int m, double* V) {
    const int f = blockIdx.y;
    const int64_t rs = (int64_t)W * 5;
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= rs) return;
    const float* mm = M + (int64_t)f * H * rs + c;
    double* v = V + (int64_t)f * H * rs + c;
    double acc = (double)(mm[0] * (float)(m + 2));
    for (int y = 1; y < m; y++) acc += mm[(int64_t)min(y, H - 1) * rs];
    for (int y = 0; y < H; y++) {
        acc += mm[(int64_t)min(y + m, H - 1) * rs] - mm[(int64_t)max(y - m - 1, 0) * rs];
        v[(int64_t)y * rs] = acc;
    }
}

// FB8: box filter, horizontal running sums + the 2x2 solve. One wave per (row, frame): per 64-pixel
// chunk the lanes stage the window differences in LDS, lanes 0..4 carry the five sequential
// accumulators (g11, g12, g22, h1, h2) across it, then every lane solves its pixel.
__global__ __launch_bounds__(64) void k_fb_box_h(const double* V, int H, int W, int m, double scale, float* flow) {
    __shared__ double dlt[5][64];
    __shared__ double acc[5][64];
    const int y = blockIdx.x, f = blockIdx.y;
    const int lane = threadIdx.x;
    const double* v = V + ((int64_t)f * H + y) * W * 5;
    float* fl = flow + ((int64_t)f * H + y) * W * 2;
    double a = 0.0;
    if (lane < 5) {  // the reference's initial window: pixel 0 x (m + 2), pixels 1 .. m-1
        a = v[lane] * (m + 2);
        for (int x = 1; x < m; x++) a += v[(int64_t)min(x, W - 1) * 5 + lane];
    }
    for (int x0 = 0; x0 < W; x0 += 64) {
        const int x = x0 + lane;
        const int cnt = min(64, W - x0);
        if (x < W) {
            const double* hi = v + (int64_t)min(x + m, W - 1) * 5;
            const double* lo = v + (int64_t)max(x - m - 1, 0) * 5;
            for (int c = 0; c < 5; ++c) dlt[c][lane] = hi[c] - lo[c];
        }
        __syncthreads();
        if (lane < 5) {
            for (int k = 0; k < cnt; ++k) {
                a += dlt[lane][k];
                acc[lane][k] = a;
            }
        }
        __syncthreads();
        if (x < W) {
            const double g11 = acc[0][lane] * scale, g12 = acc[1][lane] * scale, g22 = acc[2][lane] * scale,
                         h1 = acc[3][lane] * scale, h2 = acc[4][lane] * scale;
            const double idet = 1. / (g11 * g22 - g12 * g12 + 1e-3);
            fl[x * 2] = (float)((g11 * h2 - g12 * h1) * idet);
            fl[x * 2 + 1] = (float)((g22 * h1 - g12 * h2) * idet);
        }
        __syncthreads();
    }
}

// cvtColor(COLOR_BGR2GRAY), 8-bit fixed point.
__global__ __launch_bounds__(256) void k_bgr_gray(const unsigned char* bgr, int64_t n, unsigned char* gray) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const unsigned char* q = bgr + 3 * p;
        gray[p] = (unsigned char)((q[0] * 1868 + q[1] * 9617 + q[2] * 4899 + (1 << 13)) >> 14);
    }
}

// ---- host driver -----------------------------------------------------------------------------------
struct Engine {
    float *tmp = nullptr, *blur = nullptr, *img = nullptr, *vt = nullptr, *R = nullptr, *M = nullptr;
    float *flow[2] = {nullptr, nullptr};
    double* V = nullptr;
    int64_t cap = 0;  // frames x pixels allocated
    std::string err;

    ~Engine() { release(); }
    void release() {
        for (void* p : {(void*)tmp, (void*)blur, (void*)img, (void*)vt, (void*)R, (void*)M, (void*)flow[0],
                        (void*)flow[1], (void*)V})
            if (p) (void)hipFree(p);
        tmp = blur = img = vt = R = M = flow[0] = flow[1] = nullptr;
        V = nullptr;
        cap = 0;
    }
    bool reserve(int64_t px) {  // px = frames x H x W
        if (px <= cap) return true;
        release();
        bool ok = hipMalloc(&tmp, sizeof(float) * 2 * px) == hipSuccess &&
                  hipMalloc(&blur, sizeof(float) * 2 * px) == hipSuccess &&
                  hipMalloc(&img, sizeof(float) * 2 * px) == hipSuccess &&
                  hipMalloc(&vt, sizeof(float) * 6 * px) == hipSuccess &&
                  hipMalloc(&R, sizeof(float) * 10 * px) == hipSuccess &&
                  hipMalloc(&M, sizeof(float) * 5 * px) == hipSuccess &&
                  hipMalloc(&flow[0], sizeof(float) * 2 * px) == hipSuccess &&
                  hipMalloc(&flow[1], sizeof(float) * 2 * px) == hipSuccess &&
                  hipMalloc(&V, sizeof(double) * 5 * px) == hipSuccess;
        if (!ok) {
            release();
            err = "farneback workspace allocation failed";
            return false;
        }
        cap = px;
        return true;
    }
    static dim3 grid(int64_t n, int rows) {
        int64_t gx = (n + 255) / 256;
        const int64_t capx = std::max<int64_t>(1, 16384 / rows);
        return dim3((unsigned)std::min(gx, capx), (unsigned)rows);
    }

    // calcOpticalFlowFarneback for B frame pairs (frames B x H x W u8, contiguous) -> d_out B x H x W x 2.
    int run(const unsigned char* prev, const unsigned char* next, int B, int rows, int cols, const dofs_flow_params& p,
            float* d_out, hipStream_t s) {
        if (p.flags != 0 || p.poly_n < 1 || p.poly_n > kMaxPolyN || p.winsize < 1 || p.iterations < 1 ||
            !(p.pyr_scale > 0 && p.pyr_scale < 1) || p.levels < 0) {
            err = "unsupported Farneback parameters (flags must be 0; poly_n 1..7)";
            return DOFS_ERR_INVALID_ARG;
        }
        if (!reserve((int64_t)B * rows * cols)) return DOFS_ERR_OOM;
        const int min_size = 32;
        int levels = 0;
        double scale = 1;
        for (levels = 0; levels < p.levels; levels++) {
            scale *= p.pyr_scale;
            if (cols * scale < min_size || rows * scale < min_size) break;
        }
        const PolyConsts pc = poly_consts(p.poly_n, p.poly_sigma);
        const Pair in{prev, next};
        int ph = 0, pw = 0, cur = 0;
        for (int k = levels; k >= 0; k--) {
            scale = 1;
            for (int i = 0; i < k; i++) scale *= p.pyr_scale;
            const double sigma = (1. / scale - 1) * 0.5;
            const int ks = std::max(cv_round(sigma * 5) | 1, 3);
            if (ks > kMaxTaps) {
                err = "Farneback pyramid too deep for the pre-blur kernel";
                return DOFS_ERR_INVALID_ARG;
            }
            const Taps taps = gauss_taps(ks, sigma);
            const int w = cv_round(cols * scale), h = cv_round(rows * scale);
            const int64_t N0 = (int64_t)rows * cols, N = (int64_t)w * h;
            float* fl = k == 0 ? d_out : flow[cur ^ 1];
            if (k == levels) {
                if (hipMemsetAsync(fl, 0, sizeof(float) * 2 * N * B, s) != hipSuccess) return fail("memset");
            } else {
                hipLaunchKernelGGL(k_fb_flow_up, grid(N * 2, B), dim3(256), 0, s, flow[cur], ph, pw, fl, h, w,
                                   (float)(1. / p.pyr_scale));
            }
            hipLaunchKernelGGL(k_fb_blur_row, grid(N0, 2 * B), dim3(256), 0, s, in, rows, cols, taps, tmp);
            hipLaunchKernelGGL(k_fb_blur_col, grid(N0, 2 * B), dim3(256), 0, s, tmp, rows, cols, taps, blur);
            const float* lvl = blur;
            if (h != rows || w != cols) {
                hipLaunchKernelGGL(k_fb_resize, grid(N, 2 * B), dim3(256), 0, s, blur, rows, cols, img, h, w);
                lvl = img;
            }
            hipLaunchKernelGGL(k_fb_poly_v, grid(N, 2 * B), dim3(256), 0, s, lvl, h, w, pc, vt);
            hipLaunchKernelGGL(k_fb_poly_h, grid(N, 2 * B), dim3(256), 0, s, vt, h, w, pc, R);
            hipLaunchKernelGGL(k_fb_update_matrices, grid(N, B), dim3(256), 0, s, R, fl, h, w, M);
            const int m = p.winsize / 2;
            const double bscale = 1. / (p.winsize * p.winsize);
            for (int it = 0; it < p.iterations; ++it) {
                hipLaunchKernelGGL(k_fb_box_v, dim3((unsigned)((w * 5 + 255) / 256), (unsigned)B), dim3(256), 0, s, M,
                                   h, w, m, V);
                hipLaunchKernelGGL(k_fb_box_h, dim3((unsigned)h, (unsigned)B), dim3(64), 0, s, V, h, w, m, bscale, fl);
                if (it < p.iterations - 1)
                    hipLaunchKernelGGL(k_fb_update_matrices, grid(N, B), dim3(256), 0, s, R, fl, h, w, M);
            }
            if (hipGetLastError() != hipSuccess) return fail("farneback kernel launch");
            cur ^= 1;
            ph = h;
            pw = w;
        }
        return DOFS_OK;
    }
    int fail(const char* what) {
        err = std::string("HIP error in ") + what;
        return DOFS_ERR_DEVICE;
    }
};

}  // namespace flow
}  // namespace dofs
