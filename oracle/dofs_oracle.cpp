// oracle/dofs_oracle.cpp — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the
// product path (denseopticalflowsegmentation3d_amd/). Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg load it (as the checker / the timed CPU baseline).
//
// A from-scratch CPU restatement of the reference's dense-optical-flow clustering + 3D-lifting path
// (DmitriyZhuravlev/DenseOpticalFlowSegmentation3D @ v1, read as text; its C++ cannot be compiled
// here: OpenCV and spdlog are absent). Each function cites the reference file:line it restates.
//
// Parity pins: the lifting math is pinned by the reference's own gtest known-answer vectors
// (cpp/tests/test_liftig_3d.cpp:69-89, :179-227) — see tests/test_oracle_kat.py. The clustering
// path (graph.cpp / segment.cpp) has no reference test and no runnable reference: it is
// "parity unpinned" by the reference and is cross-checked against an independent pure-Python
// restatement (oracle/ref_py.py) on small inputs. GaussianBlur and getPerspectiveTransform are
// third-party (OpenCV, version unpinned by cpp/CMakeLists.txt:14); the restatement declares the
// OpenCV 4.x scalar-path semantics it follows.
//
// Floating point: build with -ffp-contract=off and no -march flags: the reference forces a Debug
// (-O0) x86-64 build (cpp/CMakeLists.txt:8), i.e. SSE2 float/double arithmetic with no FMA.
//
// Two modes with identical outputs:
//   faithful (mode 1): the reference's data structures — std::multiset edge sort (graph.cpp:60),
//       std::set per component merged on every union (graph.cpp:192), std::set copies into the
//       snapshot history (graph.cpp:354), vector-valued bboxes — used as the timed CPU baseline.
//   fast (mode 0): sorted vector + flat union-find arrays + a Kruskal reconstruction tree.

#include "../include/dofs.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <set>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------------
// OpenCV Point2f / Vec2f operator semantics used by the reference (OpenCV 4.x types.hpp, matx.hpp).
// ---------------------------------------------------------------------------------------------
struct P2 {
    float x, y;
};
inline P2 p2(float x, float y) { return P2{x, y}; }
inline P2 add(P2 a, P2 b) { return P2{a.x + b.x, a.y + b.y}; }           // Point2f + Point2f
inline P2 sub(P2 a, P2 b) { return P2{a.x - b.x, a.y - b.y}; }           // Point2f - Point2f
inline P2 mul_d(double a, P2 b) {                                         // double * Point2f
    return P2{(float)((double)b.x * a), (float)((double)b.y * a)};
}
inline P2 div_d(P2 a, double b) {                                         // Point2f / double
    return P2{(float)((double)a.x / b), (float)((double)a.y / b)};
}
inline P2 div_i(P2 a, int b) { return P2{a.x / (float)b, a.y / (float)b}; }  // Point2f / int
inline P2 mul_i(int a, P2 b) { return P2{b.x * (float)a, b.y * (float)a}; }  // int * Point2f
inline double norm(P2 a) {                                                // cv::norm(Point2f)
    return std::sqrt((double)a.x * (double)a.x + (double)a.y * (double)a.y);
}
inline double norm_vec(float x, float y) {  // cv::norm(Vec2f): normL2Sqr<float,double>, s=0; s+=v*v
    double s = 0.0;
    double v0 = x;
    s += v0 * v0;
    double v1 = y;
    s += v1 * v1;
    return std::sqrt(s);
}

// ---------------------------------------------------------------------------------------------
// 3D lifting — cpp/src/lifting_3d.cpp
// ---------------------------------------------------------------------------------------------
// get_intersect, lifting_3d.cpp:63-89 (float arithmetic, NaN when |det| < 1e-9).
P2 get_intersect(P2 A, P2 B, P2 C, P2 D) {
    float a1 = B.y - A.y;
    float b1 = A.x - B.x;
    float c1 = a1 * (A.x) + b1 * (A.y);
    float a2 = D.y - C.y;
    float b2 = C.x - D.x;
    float c2 = a2 * (C.x) + b2 * (C.y);
    float det = a1 * b2 - a2 * b1;
    if ((double)std::fabs(det) < 1e-9) {
        return P2{std::numeric_limits<float>::quiet_NaN(), std::numeric_limits<float>::quiet_NaN()};
    }
    float x = (b2 * c1 - b1 * c2) / det;
    float y = (a1 * c2 - a2 * c1) / det;
    return P2{x, y};
}

// warp_perspective, lifting_3d.cpp:112-121 (m is a row-major Matx33f).
P2 warp_perspective(P2 p, const float* m) {
    float px = (m[0] * p.x + m[1] * p.y + m[2]) / (m[6] * p.x + m[7] * p.y + m[8]);
    float py = (m[3] * p.x + m[4] * p.y + m[5]) / (m[6] * p.x + m[7] * p.y + m[8]);
    return P2{px, py};
}

inline P2 iv(P2 a) { return P2{a.x, -a.y}; }  // lifting_3d.cpp:141-144

// get_bottom, lifting_3d.cpp:162-217. Returns false where the reference returns an empty corner list.
bool get_bottom(const P2 warp_corners[4], double orient, double w, double h, double* error_out,
                P2 corners_out[4]) {
    P2 a[4];
    for (int i = 0; i < 4; ++i) a[i] = iv(warp_corners[i]);  // :166
    const float inf = std::numeric_limits<float>::infinity();
    P2 k = get_intersect(a[3], p2((float)(a[3].x + std::cos(orient)), (float)(a[3].y + std::sin(orient))),
                         a[0], a[1]);  // :167-168
    if (k.x == inf || k.y == inf) return false;  // :170-174 (never true: get_intersect returns NaN)
    double l = norm(sub(a[3], k));               // :176
    if (l == 0) return false;                    // :178-182
    P2 c = div_d(add(mul_d(l - w, a[0]), mul_d(w, a[3])), l);  // :184
    P2 b = get_intersect(c, p2((float)(c.x + std::cos(orient)), (float)(c.y + std::sin(orient))), a[0],
                         a[1]);  // :188
    if (b.x == inf) return false;  // :190-194
    double ew = norm(sub(c, b));   // :196
    double error_w = (ew < w) ? ew / w : w / ew;
    P2 d = get_intersect(c, p2((float)(c.x - std::sin(orient)), (float)(c.y + std::cos(orient))), a[3],
                         a[2]);  // :199
    if (d.x == inf) return false;  // :201-205
    double el = norm(sub(c, d));   // :207
    double error_l = (el < h) ? el / h : h / el;
    P2 center = div_i(add(b, d), 2);  // :210
    P2 f = sub(mul_i(2, center), c);  // :211
    corners_out[0] = iv(c);           // :213
    corners_out[1] = iv(b);
    corners_out[2] = iv(f);
    corners_out[3] = iv(d);
    *error_out = error_w * error_l;  // :214
    return true;
}

// get_motion_direction, lifting_3d.cpp:219-253.
double get_motion_direction(P2 direction, const int box[4], const float* persp) {
    int sum_x = box[0] + box[2];
    int sum_y = box[1] + box[3];
    P2 center = p2((float)(sum_x / 2), (float)(sum_y / 2));  // :231 integer division
    P2 nd = div_d(direction, norm(direction));               // :234
    P2 t1 = warp_perspective(center, persp);                 // :239
    P2 t2 = warp_perspective(add(center, nd), persp);        // :240
    double v_x = t2.x - t1.x;                                // :242 (float subtraction)
    double v_y = t1.y - t2.y;                                // :243
    return std::atan2(v_y, v_x);                             // :244
}

// get_upper_face, lifting_3d.cpp:290-348 (the catch branch :325-338 is unreachable).
void get_upper_face(const int box[4], const P2 lf[4], P2 uf[4]) {
    int xmin = box[0], ymin = box[1], xmax = box[2], ymax = box[3];
    uf[2] = sub(lf[2], p2(0.0f, lf[2].y - (float)ymin));  // :304
    P2 right_van = get_intersect(lf[1], lf[2], lf[0], lf[3]);  // :311
    uf[1] = get_intersect(uf[2], right_van, p2((float)xmin, (float)ymin), p2((float)xmin, (float)ymax));
    P2 left_van = get_intersect(lf[2], lf[3], lf[0], lf[1]);  // :317
    uf[3] = get_intersect(uf[2], left_van, p2((float)xmax, (float)ymin), p2((float)xmax, (float)ymax));
    uf[0] = get_intersect(left_van, uf[1], right_van, uf[3]);  // :322
}

// get_upper_face_simple, lifting_3d.cpp:261-288 (public, lifting_3d.hpp:23-24; not called by the path).
void get_upper_face_simple(const int box[4], const P2 lf[4], P2 uf[4]) {
    double ymin = box[1];                                        // :267 (xmin/xmax/ymax unused)
    double h_min = 0 - ymin + std::min(lf[1].y, lf[2].y);        // :272 (h_max, :271, is unused)
    const P2 dh = p2(0.0f, (float)h_min);                        // cv::Point2f(0, h_min): double -> float
    uf[0] = sub(lf[0], dh);                                      // :274
    uf[3] = sub(lf[3], dh);                                      // :275
    uf[1] = sub(lf[1], dh);                                      // :277
    uf[2] = sub(lf[2], dh);                                      // :278
}

const int kDefaultObjSize[3][2] = {{258, 84}, {349, 165}, {370, 180}};  // lifting_3d.cpp:255-259
const double kObjSizeD[3][2] = {{258, 84}, {349, 165}, {370, 180}};     // get_obj_size, lifting_3d.cpp:524-528

// get_bottom_variants, lifting_3d.cpp:350-439.
void get_bottom_variants(P2 dir, const int box[4], const float* mat, const float* inv, const float* inv_upper,
                         int cls, const int obj_size[3][2], dofs_solution* s) {
    std::memset(s, 0, sizeof(*s));
    s->cls = cls;
    double mov_angle = get_motion_direction(dir, box, mat);  // :358
    if (std::isinf(mov_angle)) {                             // :360-364 -> Solution()
        s->cls = -1;
        s->valid = 0;
        s->w_error = -1.0;
        s->h_error = -1.0;
        return;
    }
    int xmin = box[0], ymin = box[1], xmax = box[2], ymax = box[3];
    P2 ps[4] = {p2((float)xmin, (float)ymax), p2((float)xmin, (float)ymin), p2((float)xmax, (float)ymin),
                p2((float)xmax, (float)ymax)};  // :373-375
    P2 ps_bev[4];
    for (int i = 0; i < 4; ++i) ps_bev[i] = warp_perspective(ps[i], mat);  // :378
    int dim_l = obj_size[cls][0], dim_w = obj_size[cls][1];                // :381
    double error = 0.0;
    P2 corners[4];
    if (!get_bottom(ps_bev, mov_angle, (double)dim_l, (double)dim_w, &error, corners)) {  // :399
        s->valid = 0;  // Solution(cls, {}, {}, {}, {}, 0.0, 0.0, 0.0), :401-406
        s->w_error = 0.0;
        s->h_error = 0.0;
        s->orient = 0.0;
        return;
    }
    P2 untop[4];
    for (int i = 0; i < 4; ++i) untop[i] = warp_perspective(corners[i], inv);  // :412
    P2 uf[4];
    get_upper_face(box, untop, uf);                                      // :418
    P2 expected_edge = warp_perspective(corners[0], inv_upper);          // :429
    double expected_h = norm(sub(untop[0], expected_edge));              // :430
    double computed_h = norm(sub(uf[0], untop[0]));                      // :431
    double h_error = (computed_h < expected_h) ? (computed_h / expected_h) : (expected_h / computed_h);
    s->valid = 1;
    for (int i = 0; i < 4; ++i) {
        s->ps_bev[i][0] = ps_bev[i].x;
        s->ps_bev[i][1] = ps_bev[i].y;
        s->lower_face[i][0] = untop[i].x;
        s->lower_face[i][1] = untop[i].y;
        s->upper_face[i][0] = uf[i].x;
        s->upper_face[i][1] = uf[i].y;
        s->rectangle[i][0] = corners[i].x;
        s->rectangle[i][1] = corners[i].y;
    }
    s->w_error = error;  // :426
    s->h_error = h_error;
    s->orient = mov_angle;
}

// get_score, graph.cpp:241-270: max over classes of (w_error + h_error)/2, -1 when none.
double get_score(const int box[4], float mx, float my, const float* persp, const float* inv,
                 const float* inv_upper27, const int obj_size[3][2], dofs_solution* best) {
    double max_score = -1.0;
    std::memset(best, 0, sizeof(*best));
    best->cls = -1;  // default Solution (cls uninitialised in the reference, graph.hpp:37-38)
    best->w_error = -1.0;
    best->h_error = -1.0;
    for (int cls = 0; cls < 3; ++cls) {
        dofs_solution sol;
        get_bottom_variants(p2(mx, my), box, persp, inv, inv_upper27 + 9 * cls, cls, obj_size, &sol);
        if (sol.valid && max_score < (sol.w_error + sol.h_error) / 2) {  // :257
            max_score = (sol.w_error + sol.h_error) / 2;
            *best = sol;
        }
    }
    return max_score;
}

// ---------------------------------------------------------------------------------------------
// Calibration — cv::getPerspectiveTransform (OpenCV 4.x imgproc/imgwarp.cpp) restated:
// 8×8 system in double (products of the float points computed in float), solved by
// hal::LU64f-style Gaussian elimination with partial pivoting (back substitution divides by the
// pivot); M(2,2) = 1; result → float.
// ---------------------------------------------------------------------------------------------
bool lu_solve8(double A[8][8], double b[8]) {
    const int m = 8;
    const double eps = std::numeric_limits<double>::epsilon() * 100;
    for (int i = 0; i < m; i++) {
        int k = i;
        for (int j = i + 1; j < m; j++)
            if (std::fabs(A[j][i]) > std::fabs(A[k][i])) k = j;
        if (std::fabs(A[k][i]) < eps) return false;
        if (k != i) {
            for (int j = i; j < m; j++) std::swap(A[i][j], A[k][j]);
            std::swap(b[i], b[k]);
        }
        double d = -1 / A[i][i];
        for (int j = i + 1; j < m; j++) {
            double alpha = A[j][i] * d;
            for (int kk = i + 1; kk < m; kk++) A[j][kk] += alpha * A[i][kk];
            b[j] += alpha * b[i];
        }
    }
    for (int i = m - 1; i >= 0; i--) {
        double s = b[i];
        for (int kk = i + 1; kk < m; kk++) s -= A[i][kk] * b[kk];
        b[i] = s / A[i][i];  // division: reproduces the exact 0/-0 entries of the KAT literal (test_liftig_3d.cpp:185)
    }
    return true;
}

void get_perspective_transform(const P2 src[4], const P2 dst[4], double M[9]) {
    double a[8][8], b[8];
    for (int i = 0; i < 4; ++i) {
        a[i][0] = a[i + 4][3] = src[i].x;
        a[i][1] = a[i + 4][4] = src[i].y;
        a[i][2] = a[i + 4][5] = 1;
        a[i][3] = a[i][4] = a[i][5] = a[i + 4][0] = a[i + 4][1] = a[i + 4][2] = 0;
        a[i][6] = -src[i].x * dst[i].x;  // float products (Point2f members)
        a[i][7] = -src[i].y * dst[i].x;
        a[i + 4][6] = -src[i].x * dst[i].y;
        a[i + 4][7] = -src[i].y * dst[i].y;
        b[i] = dst[i].x;
        b[i + 4] = dst[i].y;
    }
    lu_solve8(a, b);
    for (int i = 0; i < 8; ++i) M[i] = b[i];
    M[8] = 1.0;
}

// get_mat, lifting_3d.cpp:482-514 and get_mat_upper, :441-480.
void calib(float persp[9], float inv[9], float inv_upper[27]) {
    const double x_offset = 100, y_offset = 6000, h = 7000, w = 700;
    P2 dst[4] = {p2((float)(0 + x_offset), (float)(0 + h + y_offset)), p2((float)(0 + x_offset), (float)(0 + y_offset)),
                 p2((float)(w + x_offset), (float)(0 + y_offset)), p2((float)(w + x_offset), (float)(h + y_offset))};
    P2 src[4] = {p2(215, 265), p2(90, 121), p2(294, 120), p2(625, 265)};
    double M[9];
    get_perspective_transform(src, dst, M);
    for (int i = 0; i < 9; ++i) persp[i] = (float)M[i];
    get_perspective_transform(dst, src, M);
    for (int i = 0; i < 9; ++i) inv[i] = (float)M[i];
    const float up[3][4][2] = {{{215, 176}, {90, 85}, {294, 85}, {625, 176}},
                               {{215, 185}, {90, 80}, {294, 80}, {625, 185}},
                               {{215, 140}, {90, 55}, {294, 55}, {625, 140}}};
    for (int cls = 0; cls < 3; ++cls) {
        P2 s2[4];
        for (int i = 0; i < 4; ++i) s2[i] = p2(up[cls][i][0], up[cls][i][1]);
        get_perspective_transform(dst, s2, M);
        for (int i = 0; i < 9; ++i) inv_upper[9 * cls + i] = (float)M[i];
    }
}

// ---------------------------------------------------------------------------------------------
// Gaussian blur — cv::GaussianBlur(flow, flow, Size(0,0), sigma) (segment.cpp:52), OpenCV 4.x:
// ksize = cvRound(sigma*4*2+1)|1 for float input; kernel = getGaussianKernelBitExact (double,
// glibc exp in place of softdouble exp) rounded to float; sepFilter2D scalar path: RowFilter
// (taps k = 0..ksize-1 left to right, s = k0*S0; s += kk*Sk) then SymmColumnFilter
// (s = k_c*S_0 + 0; s += k_j*(S_+j + S_-j)), BORDER_REFLECT_101. No FMA.
// ---------------------------------------------------------------------------------------------
int gaussian_ksize(double sigma) { return ((int)std::nearbyint(sigma * 4 * 2 + 1)) | 1; }

std::vector<float> gaussian_kernel(int n, double sigma) {
    std::vector<double> values((size_t)(n / 2 + 1));
    double sigmaX = sigma > 0 ? sigma : (double)n * 0.15 + 0.35;
    double scale2X = (-0.5 * 0.25) / (sigmaX * sigmaX);
    int n2 = (n - 1) / 2;
    double sum = 0.0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = std::exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2.0;
    sum += 1.0;
    if ((n & 1) == 0) sum += 1.0;
    double mul1 = 1.0 / sum;
    double sum2 = 0.0;
    for (int i = 0; i < n2; i++) {
        double t = values[i] * mul1;
        values[i] = t;
        sum2 += t;
    }
    sum2 *= 2.0;
    values[n2] = 1.0 - sum2;
    std::vector<float> k((size_t)n);
    for (int i = 0; i <= n2; i++) {
        k[i] = (float)values[i];
        k[n - 1 - i] = (float)values[i];
    }
    return k;
}

inline int reflect101(int p, int len) {  // cv::borderInterpolate(p, len, BORDER_REFLECT_101)
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p;
        else
            p = len - 1 - (p - len) - 1;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

void blur_flow(const float* in, int H, int W, double sigma, float* out) {
    int n = gaussian_ksize(sigma);
    std::vector<float> k = gaussian_kernel(n, sigma);
    int r = n / 2;
    std::vector<float> tmp((size_t)H * W * 2);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 2; ++c) {
                const float* row = in + (size_t)y * W * 2;
                float s = k[0] * row[reflect101(x - r, W) * 2 + c];
                for (int t = 1; t < n; ++t) s += k[t] * row[reflect101(x - r + t, W) * 2 + c];
                tmp[((size_t)y * W + x) * 2 + c] = s;
            }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 2; ++c) {
                float s = k[r] * tmp[((size_t)y * W + x) * 2 + c] + 0.0f;
                for (int j = 1; j <= r; ++j) {
                    float a = tmp[((size_t)reflect101(y + j, H) * W + x) * 2 + c];
                    float b = tmp[((size_t)reflect101(y - j, H) * W + x) * 2 + c];
                    s += k[r + j] * (a + b);
                }
                out[((size_t)y * W + x) * 2 + c] = s;
            }
}

// ---------------------------------------------------------------------------------------------
// Graph — diff (segment.cpp:20-32), create_edge (graph.cpp:43-49), build_graph (graph.cpp:51-103).
// ---------------------------------------------------------------------------------------------
struct Edge {
    int start;
    int end;
    double weight;
};

inline double diff(const float* flow, int W, int x1, int y1, int x2, int y2) {
    const float* f1 = flow + ((size_t)y1 * W + x1) * 2;
    const float* f2 = flow + ((size_t)y2 * W + x2) * 2;
    double delta_x = f1[0] - f2[0];  // float subtraction, then widened
    double delta_y = f1[1] - f2[1];
    return std::sqrt(delta_x * delta_x + delta_y * delta_y);
}

template <class Emit>
void for_each_edge(const float* flow, int W, int H, bool nbr8, Emit emit) {
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int v = y * W + x;
            if (x > 0) emit(Edge{v, v - 1, diff(flow, W, x, y, x - 1, y)});
            if (y > 0) emit(Edge{v, v - W, diff(flow, W, x, y, x, y - 1)});
            if (nbr8) {
                if (x > 0 && y > 0) emit(Edge{v, v - W - 1, diff(flow, W, x, y, x - 1, y - 1)});
                if (x > 0 && y < H - 1) emit(Edge{v, v + W - 1, diff(flow, W, x, y, x - 1, y + 1)});
            }
        }
}

bool edge_less(const Edge& a, const Edge& b) { return a.weight < b.weight; }  // graph.cpp:55-58

std::vector<Edge> build_graph_faithful(const float* flow, int W, int H, bool nbr8) {
    std::multiset<Edge, bool (*)(const Edge&, const Edge&)> edges(edge_less);  // graph.cpp:60
    for_each_edge(flow, W, H, nbr8, [&](const Edge& e) { edges.insert(e); });
    std::vector<Edge> out;
    out.reserve(edges.size());
    std::move(edges.begin(), edges.end(), std::back_inserter(out));
    return out;
}

std::vector<Edge> build_graph_fast(const float* flow, int W, int H, bool nbr8) {
    std::vector<Edge> out;
    out.reserve((size_t)W * H * 4);
    for_each_edge(flow, W, H, nbr8, [&](const Edge& e) { out.push_back(e); });
    // multiset insertion at upper_bound == stable sort by weight in emission order
    std::stable_sort(out.begin(), out.end(), edge_less);
    return out;
}

// ---------------------------------------------------------------------------------------------
// Kruskal replay — Forest (graph.hpp:59-114, graph.cpp:129-218, 272-384), segment_graph (:503-536).
// ---------------------------------------------------------------------------------------------
struct Ctx {
    int W, H;
    const float *persp, *inv, *inv_upper;
    const dofs_params* prm;
    dofs_stats st;
};

struct Slot {
    double score = -1.0;
    int event = -1;
    double move = 0.0;
    dofs_solution sol;
    int size = 0;
    int bbox[4] = {0, 0, 0, 0};
};

// Shared per-merge scoring of new_merge (graph.cpp:280-356). Returns true when the slot improved.
// last_score (optional) is Forest::segment_scores[root]: written for every scored candidate, before the
// convexity and threshold tests (graph.cpp:326), so it ends as the root's last scored score.
bool score_merge(Ctx& cx, int root, int size, float mx, float my, const int bbox[4], Slot& slot, int event,
                 double* last_score) {
    if (size < cx.prm->min_size) return false;  // :280
    int y = root / cx.W;
    if (y < cx.H / 10) return false;  // :286-292
    double move = norm_vec(mx, my);   // :294
    if (move < 3 * (y + 1) / static_cast<double>(cx.H)) return false;  // :296
    cx.st.n_candidates++;
    double rect_area = (double)((bbox[2] - bbox[0] + 1) * (bbox[3] - bbox[1] + 1));  // :303
    double convexity = size / rect_area;                                            // :305
    dofs_solution sol;
    double score = get_score(bbox, mx, my, cx.persp, cx.inv, cx.inv_upper, cx.prm->obj_size, &sol);  // :312
    if (score == -1) return false;  // :318
    cx.st.n_scored++;
    if (last_score) *last_score = score;  // :326
    double min_convexity = 1.0 / 2.0;
    if (sol.cls == 0) min_convexity = cx.prm->min_convexity[0];  // :328-339
    if (sol.cls == 1) min_convexity = cx.prm->min_convexity[1];
    if (sol.cls == 2) min_convexity = cx.prm->min_convexity[2];
    if (convexity < min_convexity) return false;  // :342
    if (!(score > cx.prm->score_threshold)) return false;  // :348
    cx.st.n_qualified++;
    if (slot.score < score) {  // :352
        slot.score = score;
        slot.event = event;
        slot.move = move;
        slot.sol = sol;
        slot.size = size;
        std::memcpy(slot.bbox, bbox, sizeof(slot.bbox));
        return true;
    }
    return false;
}

// Kruskal reconstruction tree bookkeeping shared by both modes (not part of the reference:
// used to express SegmentData::seg as a range of one leaf order).
struct Krt {
    int N;
    std::vector<int> cl, cr;  // children of merge node k (node ids: pixel < N, merge k -> N + k)
    std::vector<int> cur;     // current KRT node of each union-find root
    void init(int n) {
        N = n;
        cur.resize(n);
        for (int i = 0; i < n; ++i) cur[i] = i;
        cl.reserve(n);
        cr.reserve(n);
    }
    void merge(int ra, int rb, int root) {  // ra = find(start), rb = find(end)
        cl.push_back(cur[ra]);
        cr.push_back(cur[rb]);
        cur[root] = N + (int)cl.size() - 1;
    }
    // Leaf order (DFS, start side first) and the first leaf position of every merge node.
    void order(std::vector<int>& leaf_order, std::vector<int>& first) const {
        int M = (int)cl.size();
        leaf_order.clear();
        leaf_order.reserve(N);
        first.assign(M, 0);
        std::vector<int> stack;
        std::vector<int> roots;
        // forest roots: nodes that are nobody's child (one root when the grid is connected)
        std::vector<char> is_child(N + M, 0);
        for (int k = 0; k < M; ++k) is_child[cl[k]] = is_child[cr[k]] = 1;
        for (int v = 0; v < N + M; ++v)
            if (!is_child[v]) roots.push_back(v);
        for (int r : roots) {
            stack.push_back(r);
            while (!stack.empty()) {
                int x = stack.back();
                stack.pop_back();
                if (x < N) {
                    leaf_order.push_back(x);
                } else {
                    first[x - N] = (int)leaf_order.size();
                    stack.push_back(cr[x - N]);
                    stack.push_back(cl[x - N]);
                }
            }
        }
    }
};

struct Output {
    std::vector<dofs_event>* events;  // optional
};

void fill_snapshot(dofs_snapshot* s, int slot, const Slot& sl, int seg_begin) {
    std::memset(s, 0, sizeof(*s));
    s->slot = slot;
    s->event = sl.event;
    s->size = sl.size;
    s->seg_begin = seg_begin;
    for (int i = 0; i < 4; ++i) s->bbox[i] = sl.bbox[i];
    s->score = sl.score;
    s->move = sl.move;
    s->sol = sl.sol;
}

// --- fast mode ------------------------------------------------------------------------------
// given: segment_graph on a caller's edge list (graph.cpp:503-536), else build_graph's (graph.cpp:51-103)
// Optional Forest state after the run: scores = segment_scores (N, graph.cpp:139,326), boxes = bboxes
// (N x 4; {-1,-1,-1,-1} where merge cleared it, graph.cpp:208 — every node but the final roots).
struct Extras {
    double* scores = nullptr;
    int32_t* boxes = nullptr;
};

int segment_fast(Ctx& cx, const float* blurred, std::vector<Slot>& hist, Krt& krt, std::vector<dofs_event>* ev,
                 const std::vector<Edge>* given, const Extras& x) {
    const int W = cx.W, H = cx.H, N = W * H;
    bool nbr8 = (cx.prm->neighbor == 8);
    std::vector<Edge> built;
    if (!given) built = build_graph_fast(blurred, W, H, nbr8);
    const std::vector<Edge>& edges = given ? *given : built;
    cx.st.n_edges = (int64_t)edges.size();
    std::vector<int> parent(N), rank(N, 0), size(N, 1);
    std::vector<float> fx(N), fy(N);
    std::vector<std::array<int, 4>> bb(N);
    for (int i = 0; i < N; ++i) {
        parent[i] = i;
        fx[i] = blurred[2 * (size_t)i];
        fy[i] = blurred[2 * (size_t)i + 1];
        bb[i] = {i % W, i / W, i % W, i / W};
    }
    auto find = [&](int n) {
        int r = n;
        while (parent[r] != r) r = parent[r];
        while (parent[n] != r) {
            int nx = parent[n];
            parent[n] = r;
            n = nx;
        }
        return r;
    };
    krt.init(N);
    hist.assign(N, Slot());
    if (x.scores) std::fill(x.scores, x.scores + N, 0.0);  // segment_scores.resize(N), graph.cpp:139
    int event = 0;
    for (const Edge& e : edges) {
        int a = find(e.start), b = find(e.end);
        if (a == b) continue;
        // Forest::merge(a, b), graph.cpp:170-218
        int pa = a, pb = b;
        if (rank[pa] > rank[pb]) std::swap(pa, pb);
        parent[pa] = pb;
        int sa = size[pa], sb = size[pb];
        float wax = fx[pa] * (float)sa, way = fy[pa] * (float)sa;
        float wbx = fx[pb] * (float)sb, wby = fy[pb] * (float)sb;
        double ialpha = 1. / (sa + sb);
        fx[pb] = (float)((double)(wax + wbx) * ialpha);
        fy[pb] = (float)((double)(way + wby) * ialpha);
        size[pb] += sa;
        size[pa] = 0;
        bb[pb] = {std::min(bb[pb][0], bb[pa][0]), std::min(bb[pb][1], bb[pa][1]), std::max(bb[pb][2], bb[pa][2]),
                  std::max(bb[pb][3], bb[pa][3])};
        if (rank[pa] == rank[pb]) rank[pb] += 1;
        krt.merge(a, b, pb);
        if (ev) {
            dofs_event& r = (*ev)[event];
            r.start = e.start;
            r.end = e.end;
            r.weight = e.weight;
            r.root = pb;
            r.size = size[pb];
            r.rank = rank[pb];
            for (int i = 0; i < 4; ++i) r.bbox[i] = bb[pb][i];
            r.mean[0] = fx[pb];
            r.mean[1] = fy[pb];
        }
        int box[4] = {bb[pb][0], bb[pb][1], bb[pb][2], bb[pb][3]};
        score_merge(cx, pb, size[pb], fx[pb], fy[pb], box, hist[pb], event, x.scores ? x.scores + pb : nullptr);
        ++event;
    }
    if (x.boxes)
        for (int i = 0; i < N; ++i)
            for (int k = 0; k < 4; ++k) x.boxes[4 * (size_t)i + k] = parent[i] == i ? bb[i][k] : -1;
    return event;
}

// --- faithful mode: the reference's containers --------------------------------------------------
struct FNode {  // graph.hpp:59-70
    int id, parent, rank, size;
    float fx, fy;
};
struct FSegmentData {  // graph.hpp:48-57
    double score = -1.0;
    std::set<int> seg;
    dofs_solution sol;
    double move = 0.0;
};

int segment_faithful(Ctx& cx, const float* blurred, std::vector<Slot>& hist, Krt& krt, std::vector<dofs_event>* ev,
                     std::vector<std::set<int>>* snap_sets, const std::vector<Edge>* given, const Extras& x) {
    const int W = cx.W, H = cx.H, N = W * H;
    bool nbr8 = (cx.prm->neighbor == 8);
    std::vector<Edge> built;
    if (!given) built = build_graph_faithful(blurred, W, H, nbr8);  // graph.cpp:51-103
    const std::vector<Edge>& edges = given ? *given : built;
    cx.st.n_edges = (int64_t)edges.size();
    // Forest ctor, graph.cpp:129-148
    std::vector<FNode> nodes((size_t)N);
    std::vector<std::set<int>> segments;
    segments.reserve(N);
    std::vector<FSegmentData> segment_history((size_t)N);
    std::vector<double> segment_scores((size_t)N);
    std::vector<std::vector<std::pair<int, int>>> bboxes((size_t)N);
    for (int i = 0; i < N; ++i) {
        nodes[i] = FNode{i, i, 0, 1, blurred[2 * (size_t)i], blurred[2 * (size_t)i + 1]};
        segments.emplace_back(std::set<int>{i});
        bboxes[i] = {{i % W, i / W}, {i % W, i / W}};
    }
    std::function<int(int)> find = [&](int n) -> int {  // graph.cpp:150-157 (recursive)
        if (n != nodes[n].parent) nodes[n].parent = find(nodes[n].parent);
        return nodes[n].parent;
    };
    krt.init(N);
    hist.assign(N, Slot());
    int event = 0;
    for (const Edge& e : edges) {  // graph.cpp:519-531
        int a = find(e.start);
        int b = find(e.end);
        if (a == b) continue;
        // new_merge -> merge, graph.cpp:170-218
        int parent_a = find(a), parent_b = find(b);
        if (nodes[parent_a].rank > nodes[parent_b].rank) std::swap(parent_a, parent_b);
        nodes[parent_a].parent = parent_b;
        int size_a = nodes[parent_a].size, size_b = nodes[parent_b].size;
        float wax = nodes[parent_a].fx * (float)size_a, way = nodes[parent_a].fy * (float)size_a;
        float wbx = nodes[parent_b].fx * (float)size_b, wby = nodes[parent_b].fy * (float)size_b;
        double ialpha = 1. / (size_a + size_b);
        nodes[parent_b].fx = (float)((double)(wax + wbx) * ialpha);
        nodes[parent_b].fy = (float)((double)(way + wby) * ialpha);
        segments[parent_b].insert(segments[parent_a].begin(), segments[parent_a].end());
        segments[parent_a].clear();
        nodes[parent_b].size += size_a;
        nodes[parent_a].size = 0;
        bboxes[parent_b] = {{std::min(bboxes[parent_b][0].first, bboxes[parent_a][0].first),
                             std::min(bboxes[parent_b][0].second, bboxes[parent_a][0].second)},
                            {std::max(bboxes[parent_b][1].first, bboxes[parent_a][1].first),
                             std::max(bboxes[parent_b][1].second, bboxes[parent_a][1].second)}};
        bboxes[parent_a].clear();
        if (nodes[parent_a].rank == nodes[parent_b].rank) nodes[parent_b].rank += 1;
        krt.merge(a, b, parent_b);
        const int pb = parent_b;
        if (ev) {
            dofs_event& r = (*ev)[event];
            r.start = e.start;
            r.end = e.end;
            r.weight = e.weight;
            r.root = pb;
            r.size = nodes[pb].size;
            r.rank = nodes[pb].rank;
            r.bbox[0] = bboxes[pb][0].first;
            r.bbox[1] = bboxes[pb][0].second;
            r.bbox[2] = bboxes[pb][1].first;
            r.bbox[3] = bboxes[pb][1].second;
            r.mean[0] = nodes[pb].fx;
            r.mean[1] = nodes[pb].fy;
        }
        // new_merge scoring, graph.cpp:280-356 (bbox copy as in get_bounding_box, :446-452)
        std::vector<std::pair<int, int>> bbox = bboxes[pb];
        int box[4] = {bbox[0].first, bbox[0].second, bbox[1].first, bbox[1].second};
        if (score_merge(cx, pb, nodes[pb].size, nodes[pb].fx, nodes[pb].fy, box, hist[pb], event, &segment_scores[pb])) {
            // SegmentData(score, seg, solution, move) — copies the member set, graph.cpp:354
            segment_history[pb] = FSegmentData{hist[pb].score, segments[pb], hist[pb].sol, hist[pb].move};
        }
        ++event;
    }
    if (x.scores) std::memcpy(x.scores, segment_scores.data(), sizeof(double) * (size_t)N);
    if (x.boxes)
        for (int i = 0; i < N; ++i) {
            const bool has = !bboxes[i].empty();  // Forest::get_bounding_box(i), graph.cpp:446-452
            x.boxes[4 * (size_t)i + 0] = has ? bboxes[i][0].first : -1;
            x.boxes[4 * (size_t)i + 1] = has ? bboxes[i][0].second : -1;
            x.boxes[4 * (size_t)i + 2] = has ? bboxes[i][1].first : -1;
            x.boxes[4 * (size_t)i + 3] = has ? bboxes[i][1].second : -1;
        }
    if (snap_sets) {
        snap_sets->assign((size_t)N, std::set<int>());
        for (int i = 0; i < N; ++i)
            if (segment_history[i].score != -1.0) (*snap_sets)[i] = segment_history[i].seg;
    }
    return event;
}

}  // namespace

// =============================================================================================
// C ABI (ctypes)
// =============================================================================================
extern "C" {

void oracle_default_params(dofs_params* p) {
    p->blur_sigma = 3.0;
    p->neighbor = 8;
    p->min_size = 500;
    p->score_threshold = 0.3;
    p->overlay_min_score = 0.7;
    p->min_convexity[0] = 3.0 / 4.0;
    p->min_convexity[1] = 1.0 / 2.0;
    p->min_convexity[2] = 20.0 / 29.0;
    for (int c = 0; c < 3; ++c) {
        p->obj_size[c][0] = kDefaultObjSize[c][0];
        p->obj_size[c][1] = kDefaultObjSize[c][1];
    }
}

int32_t oracle_gaussian_kernel(double sigma, float* out, int32_t cap) {
    int n = gaussian_ksize(sigma);
    std::vector<float> k = gaussian_kernel(n, sigma);
    for (int i = 0; i < n && i < cap; ++i) out[i] = k[i];
    return n;
}

void oracle_blur(const float* in, int32_t H, int32_t W, double sigma, float* out) { blur_flow(in, H, W, sigma, out); }

void oracle_intersect(const float a1[2], const float a2[2], const float b1[2], const float b2[2], float out[2]) {
    P2 r = get_intersect(p2(a1[0], a1[1]), p2(a2[0], a2[1]), p2(b1[0], b1[1]), p2(b2[0], b2[1]));
    out[0] = r.x;
    out[1] = r.y;
}

void oracle_lift(const float dir[2], const int32_t box[4], const float mat[9], const float inv[9],
                 const float inv_upper[9], int32_t cls, dofs_solution* out) {
    int b[4] = {box[0], box[1], box[2], box[3]};
    get_bottom_variants(p2(dir[0], dir[1]), b, mat, inv, inv_upper, cls, kDefaultObjSize, out);
}

double oracle_score(const int32_t box[4], const float dir[2], const float persp[9], const float inv[9],
                    const float inv_upper[27], dofs_solution* best) {
    int b[4] = {box[0], box[1], box[2], box[3]};
    return get_score(b, dir[0], dir[1], persp, inv, inv_upper, kDefaultObjSize, best);
}

void oracle_calib(float persp[9], float inv[9], float inv_upper[27]) { calib(persp, inv, inv_upper); }

// get_upper_face (simple = 0) / get_upper_face_simple (simple = 1) on box {xmin, ymin, xmax, ymax}.
void oracle_upper_face(const int32_t box[4], const float lf[8], int32_t simple, float uf[8]) {
    int b[4] = {box[0], box[1], box[2], box[3]};
    P2 l[4], u[4];
    for (int k = 0; k < 4; ++k) l[k] = p2(lf[2 * k], lf[2 * k + 1]);
    if (simple)
        get_upper_face_simple(b, l, u);
    else
        get_upper_face(b, l, u);
    for (int k = 0; k < 4; ++k) {
        uf[2 * k] = u[k].x;
        uf[2 * k + 1] = u[k].y;
    }
}

// get_obj_size(cls), lifting_3d.cpp:524-528 (cls must be 0..2).
void oracle_obj_size(int32_t cls, double out[2]) {
    out[0] = kObjSizeD[cls][0];
    out[1] = kObjSizeD[cls][1];
}

void oracle_perspective_transform(const float src[8], const float dst[8], double out[9]) {
    P2 s[4], d[4];
    for (int i = 0; i < 4; ++i) {
        s[i] = p2(src[2 * i], src[2 * i + 1]);
        d[i] = p2(dst[2 * i], dst[2 * i + 1]);
    }
    get_perspective_transform(s, d, out);
}

// Sorted edge list of build_graph on an (already blurred) field; returns E (writes min(E, cap)).
int64_t oracle_build_graph(const float* flow, int32_t H, int32_t W, int32_t neighbor, int32_t* start, int32_t* end,
                           double* weight, int64_t cap) {
    std::vector<Edge> e = build_graph_fast(flow, W, H, neighbor == 8);
    for (int64_t i = 0; i < (int64_t)e.size() && i < cap; ++i) {
        start[i] = e[i].start;
        end[i] = e[i].end;
        weight[i] = e[i].weight;
    }
    return (int64_t)e.size();
}

// Synthetic flow field of the benchmark spec (DESIGN.md §Synthetic input).
static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_synth_flow(float* out, int32_t H, int32_t W, uint64_t seed) {
    const int64_t N = (int64_t)H * W;
    for (int64_t p = 0; p < N; ++p)
        for (int c = 0; c < 2; ++c) {
            uint64_t z = splitmix64((seed << 32) + (uint64_t)(2 * p + c));
            int q = (int)((z >> 11) % 205ull) - 102;
            out[2 * p + c] = (float)q * (1.0f / 1024.0f);
        }
    const int rect[3][4] = {{550, 900, 250, 800}, {100, 350, 400, 750}, {400, 500, 500, 900}};
    const float uv[3][2] = {{2.5f, 1.9f}, {-1.8f, 0.6f}, {0.3f, 2.2f}};
    for (int r = 0; r < 3; ++r) {
        int x0 = (int)((int64_t)W * rect[r][0] / 1000), x1 = (int)((int64_t)W * rect[r][1] / 1000);
        int y0 = (int)((int64_t)H * rect[r][2] / 1000), y1 = (int)((int64_t)H * rect[r][3] / 1000);
        if (seed != 0) {
            uint64_t zx = splitmix64((seed << 32) + 0xF0000000ull + 2 * (uint64_t)r);
            uint64_t zy = splitmix64((seed << 32) + 0xF0000000ull + 2 * (uint64_t)r + 1);
            int jx = (int)((int64_t)(zx % 101ull) * W / 1000) - (int)((int64_t)50 * W / 1000);
            int jy = (int)((int64_t)(zy % 101ull) * H / 1000) - (int)((int64_t)50 * H / 1000);
            x0 = std::min(std::max(x0 + jx, 0), W);
            x1 = std::min(std::max(x1 + jx, 0), W);
            y0 = std::min(std::max(y0 + jy, 0), H);
            y1 = std::min(std::max(y1 + jy, 0), H);
        }
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                out[2 * ((int64_t)y * W + x)] = uv[r][0];
                out[2 * ((int64_t)y * W + x) + 1] = uv[r][1];
            }
    }
}

// get_segmented_array + get_best_segments + overlay labels. mode 0 = fast, 1 = faithful,
// 2 = faithful with a self-check of every snapshot's std::set against its leaf range.
// events (optional) must hold H*W-1 records. Returns DOFS_OK or an error code.
static int32_t segment_common(const float* flow_uv, int32_t H, int32_t W, const float persp[9], const float inv[9],
                              const float inv_upper[27], const dofs_params* params, int32_t mode, dofs_result* out,
                              dofs_event* events, const std::vector<Edge>* given, const Extras& x = Extras());

int32_t oracle_segment(const float* flow_uv, int32_t H, int32_t W, const float persp[9], const float inv[9],
                       const float inv_upper[27], const dofs_params* params, int32_t mode, dofs_result* out,
                       dofs_event* events) {
    return segment_common(flow_uv, H, W, persp, inv, inv_upper, params, mode, out, events, nullptr);
}

// segment_graph(flow, sorted_graph, ...) (graph.cpp:503-536) on a caller's edge list, taken in the given
// order; the flow is used as given (no blur: get_segmented_array blurs before build_graph, segment.cpp:52).
// events (optional) must hold H*W-1 records; n_merges in the stats says how many are written.
int32_t oracle_segment_graph(const float* flow_uv, int32_t H, int32_t W, const int32_t* start, const int32_t* end,
                             const double* weight, int64_t E, const float persp[9], const float inv[9],
                             const float inv_upper[27], const dofs_params* params, int32_t mode, dofs_result* out,
                             dofs_event* events) {
    if (E < 0 || (E > 0 && (!start || !end || !weight))) return DOFS_ERR_INVALID_ARG;
    const int64_t N = (int64_t)H * W;
    std::vector<Edge> edges((size_t)E);
    for (int64_t i = 0; i < E; ++i) {
        if (start[i] < 0 || start[i] >= N || end[i] < 0 || end[i] >= N) return DOFS_ERR_INVALID_ARG;
        edges[(size_t)i] = Edge{start[i], end[i], weight[i]};
    }
    return segment_common(flow_uv, H, W, persp, inv, inv_upper, params, mode, out, events, &edges);
}

// Either form (E < 0: get_segmented_array; else segment_graph on the list) plus the Forest state after
// the run: scores[N] = Forest::get_segment_best_score(id) (graph.cpp:386-389), boxes[N x 4] =
// Forest::get_bounding_box(id) (graph.cpp:446-452; {-1,-1,-1,-1} = the empty vector). Either may be NULL.
int32_t oracle_segment_ex(const float* flow_uv, int32_t H, int32_t W, const int32_t* start, const int32_t* end,
                          const double* weight, int64_t E, const float persp[9], const float inv[9],
                          const float inv_upper[27], const dofs_params* params, int32_t mode, dofs_result* out,
                          dofs_event* events, double* scores, int32_t* boxes) {
    Extras x;
    x.scores = scores;
    x.boxes = boxes;
    if (E < 0) return segment_common(flow_uv, H, W, persp, inv, inv_upper, params, mode, out, events, nullptr, x);
    const int64_t N = (int64_t)H * W;
    if (E > 0 && (!start || !end || !weight)) return DOFS_ERR_INVALID_ARG;
    std::vector<Edge> edges((size_t)E);
    for (int64_t i = 0; i < E; ++i) {
        if (start[i] < 0 || start[i] >= N || end[i] < 0 || end[i] >= N) return DOFS_ERR_INVALID_ARG;
        edges[(size_t)i] = Edge{start[i], end[i], weight[i]};
    }
    return segment_common(flow_uv, H, W, persp, inv, inv_upper, params, mode, out, events, &edges, x);
}

static int32_t segment_common(const float* flow_uv, int32_t H, int32_t W, const float persp[9], const float inv[9],
                              const float inv_upper[27], const dofs_params* params, int32_t mode, dofs_result* out,
                              dofs_event* events, const std::vector<Edge>* given, const Extras& x) {
    if (H <= 0 || W <= 0 || !flow_uv || !out) return DOFS_ERR_INVALID_ARG;
    dofs_params prm;
    if (params)
        prm = *params;
    else
        oracle_default_params(&prm);
    const int N = W * H;
    Ctx cx{W, H, persp, inv, inv_upper, &prm, dofs_stats{}};
    std::vector<float> blurred((size_t)N * 2);
    if (given)
        std::memcpy(blurred.data(), flow_uv, sizeof(float) * 2 * (size_t)N);
    else
        blur_flow(flow_uv, H, W, prm.blur_sigma, blurred.data());  // segment.cpp:52
    std::vector<Slot> hist;
    Krt krt;
    std::vector<dofs_event> ev;
    if (events) ev.resize(N > 0 ? (size_t)N - 1 : 0);
    std::vector<std::set<int>> sets;
    int merges;
    if (mode == 0)
        merges = segment_fast(cx, blurred.data(), hist, krt, events ? &ev : nullptr, given, x);
    else
        merges = segment_faithful(cx, blurred.data(), hist, krt, events ? &ev : nullptr, mode == 2 ? &sets : nullptr,
                                  given, x);
    cx.st.n_merges = merges;
    std::vector<int> leaf_order, first;
    krt.order(leaf_order, first);
    // snapshots sorted by slot
    int ns = 0;
    for (int s = 0; s < N; ++s)
        if (hist[s].event >= 0) ++ns;
    cx.st.n_snapshots = ns;
    out->stats = cx.st;
    out->n_snapshots = ns;
    if (mode == 2) {  // self-check: faithful std::set == KRT leaf range
        for (int s = 0; s < N; ++s) {
            if (hist[s].event < 0) continue;
            int b = first[hist[s].event];
            std::vector<int> r(leaf_order.begin() + b, leaf_order.begin() + b + hist[s].size);
            std::sort(r.begin(), r.end());
            if ((int)sets[s].size() != hist[s].size || !std::equal(r.begin(), r.end(), sets[s].begin()))
                return DOFS_ERR_DEVICE;
        }
    }
    if (out->snapshots) {
        if (ns > out->snapshot_capacity) return DOFS_ERR_CAPACITY;
        int j = 0;
        for (int s = 0; s < N; ++s)
            if (hist[s].event >= 0) fill_snapshot(&out->snapshots[j++], s, hist[s], first[hist[s].event]);
    }
    if (out->labels) {  // draw.cpp:118-147: paint slots with score > min_score in ascending slot order
        for (int i = 0; i < N; ++i) out->labels[i] = -1;
        for (int s = 0; s < N; ++s) {
            if (hist[s].event < 0 || !(hist[s].score > prm.overlay_min_score)) continue;
            int b = first[hist[s].event];
            for (int t = 0; t < hist[s].size; ++t) out->labels[leaf_order[b + t]] = s;
        }
    }
    if (out->leaf_order) std::memcpy(out->leaf_order, leaf_order.data(), sizeof(int) * (size_t)N);
    if (out->blurred) std::memcpy(out->blurred, blurred.data(), sizeof(float) * 2 * (size_t)N);
    if (events && merges > 0) std::memcpy(events, ev.data(), sizeof(dofs_event) * (size_t)merges);
    return DOFS_OK;
}

}  // extern "C"
