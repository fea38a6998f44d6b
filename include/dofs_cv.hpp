// dofs_cv.hpp — header-only C++ adapter that restores the reference's OpenCV signatures over the C-ABI of
// include/dofs.h, for hosts built against OpenCV (compiled only when <opencv2/core.hpp> is available).
//
//   reference (DmitriyZhuravlev/DenseOpticalFlowSegmentation3D)                     here (namespace dofs_cv)
//   Forest get_segmented_array(flow, bev, persp, inv, inv_upper, neighbor = 8)      get_segmented_array
//       cpp/src/segment.cpp:34-72 (no header; segment.hpp is commented out)
//   std::vector<Edge> build_graph(img, width, height, diff, neighborhood_8 = false) build_graph<Edge>
//       cpp/inc/graph.hpp:22-23, cpp/src/graph.cpp:51-103
//   Forest segment_graph(flow, sorted_graph, bev, persp, inv, inv_upper)            segment_graph
//       cpp/inc/graph.hpp:120-122, cpp/src/graph.cpp:503-536
//   Solution get_bottom_variants(dir, box_2d, mat, inv, inv_upper, cls)             get_bottom_variants<Solution>
//       cpp/inc/lifting_3d.hpp:13-16, cpp/src/lifting_3d.cpp:350-439
//   std::pair<Matx33f, Matx33f> get_mat(); Matx33f get_mat_upper(int cls)           get_mat, get_mat_upper
//       cpp/inc/lifting_3d.hpp:17-18, cpp/src/lifting_3d.cpp:441-514
//   cv::Point2f get_intersect(a1, a2, b1, b2)                                        get_intersect
//       cpp/inc/lifting_3d.hpp:26, cpp/src/lifting_3d.cpp:63-110
//   std::vector<cv::Point2f> get_upper_face(box_2d, lower_face)                      get_upper_face
//       cpp/inc/lifting_3d.hpp:21-22, cpp/src/lifting_3d.cpp:290-348
//   std::vector<cv::Point2f> get_upper_face_simple(box_2d, lower_face)               get_upper_face_simple
//       cpp/inc/lifting_3d.hpp:23-24, cpp/src/lifting_3d.cpp:261-288
//   std::pair<double, double> get_obj_size(int cls)                                  get_obj_size
//       cpp/inc/lifting_3d.hpp:25, cpp/src/lifting_3d.cpp:524-528
//
// What the adapter returns instead of a Forest. The Forest's public accessors are get_best_segments()
// (graph.cpp:391-429 — it returns the whole private segment_history vector, graph.hpp:109),
// get_bounding_box (graph.cpp:446-452) and get_segment_best_score (graph.cpp:386-389);
// plot_best_segments_simple (draw.cpp:101-160) takes the Forest to call exactly get_best_segments().
// dofs_cv::Segmentation offers those three with the results a Forest gives after segment_graph returns
// (every non-root box cleared by merge, graph.cpp:208; segment_scores as new_merge left it, :326), so a
// call site changes from
//     Forest forest = get_segmented_array(flow, bev, persp, inv, inv_upper);
//     std::vector<SegmentData> history = forest.get_best_segments();
// to
//     dofs_cv::Segmentation forest = dofs_cv::get_segmented_array(flow, bev, persp, inv, inv_upper);
//     std::vector<SegmentData> history = forest.get_best_segments();
// and plot_best_segments_simple gains an overload on the history vector (its body only iterates it), or
// uses Segmentation::labels() (the overlay label map of draw.cpp:118-147) directly. No Forest is built and
// no private member is touched; the reference's own Edge / Solution / SegmentData types are filled when
// graph.hpp is included before this header (they are the default template arguments then).
//
// Behaviour kept: the flow is blurred IN PLACE, as cv::GaussianBlur(flow, flow, ...) does at
// segment.cpp:52 (set blur_in_place = false to keep the caller's field); neighbor != 4, 8 segments with the
// 4-neighbourhood (segment.cpp:38-43). Errors throw std::runtime_error (the C-ABI returns status codes).
// One dofs_ctx per host thread (context()), on device 0 unless dofs_cv::set_device() says otherwise.
#pragma once

#if defined(__has_include)
#if __has_include(<opencv2/core.hpp>)
#define DOFS_CV_HAVE_OPENCV 1
#endif
#endif

#ifdef DOFS_CV_HAVE_OPENCV
#include <opencv2/core.hpp>

#include <cstring>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "dofs.h"

namespace dofs_cv {

#ifdef GRAPH_HPP  // the reference's graph.hpp was included first: its types are the defaults
using DefaultEdge = ::Edge;
using DefaultSolution = ::Solution;
using DefaultSegmentData = ::SegmentData;
#else
using DefaultEdge = dofs_edge;
using DefaultSolution = dofs_solution;
using DefaultSegmentData = void;  // get_best_segments<YourSegmentData, YourSolution>() must name them
#endif

inline int& device_index() {
    static int d = 0;
    return d;
}
inline void set_device(int device) { device_index() = device; }

inline dofs_ctx* context() {
    thread_local std::unique_ptr<dofs_ctx, void (*)(dofs_ctx*)> ctx(dofs_create(device_index()), dofs_destroy);
    if (!ctx) throw std::runtime_error("dofs_cv: no gfx950 device (dofs_create failed)");
    return ctx.get();
}

inline void check(int32_t rc, const char* what) {
    if (rc != DOFS_OK) throw std::runtime_error(std::string("dofs_cv: ") + what + " failed: " + dofs_last_error(context()));
}

inline void to9(const cv::Matx33f& m, float out[9]) {
    for (int i = 0; i < 9; ++i) out[i] = m.val[i];  // Matx33f is row-major
}
inline cv::Matx33f from9(const float m[9]) {
    cv::Matx33f r;
    for (int i = 0; i < 9; ++i) r.val[i] = m[i];
    return r;
}
inline void mats(const cv::Matx33f& persp, const cv::Matx33f& inv, const std::vector<cv::Matx33f>& inv_upper,
                 float p[9], float i[9], float u[27]) {
    if (inv_upper.size() < 3) throw std::runtime_error("dofs_cv: inv_upper needs the 3 class homographies");
    to9(persp, p);
    to9(inv, i);
    for (int c = 0; c < 3; ++c) to9(inv_upper[c], u + 9 * c);
}

inline std::vector<cv::Point2f> pts(const float (*a)[2]) {
    std::vector<cv::Point2f> v;
    for (int k = 0; k < 4; ++k) v.emplace_back(a[k][0], a[k][1]);
    return v;
}

// dofs_solution -> the caller's Solution type (graph.hpp:25-46): the three shapes get_bottom_variants returns
// (lifting_3d.cpp:358-362 default Solution(), :396-408 empty faces, :437-438 full).
template <class SolutionT>
SolutionT to_solution(const dofs_solution& s) {
    if constexpr (std::is_same_v<SolutionT, dofs_solution>) {
        return s;
    } else {
        if (!s.valid && s.w_error == -1.0 && s.h_error == -1.0) return SolutionT();
        if (!s.valid) return SolutionT(s.cls, {}, {}, {}, {}, 0.0, 0.0, 0.0);
        return SolutionT(s.cls, pts(s.ps_bev), pts(s.lower_face), pts(s.upper_face), pts(s.rectangle), s.w_error,
                         s.h_error, s.orient);
    }
}

// The result of get_segmented_array / segment_graph: the non-empty history slots and the leaf order that
// holds every slot's member set as one range.
class Segmentation {
public:
    int width = 0, height = 0;
    std::vector<dofs_snapshot> snapshots;  // non-empty segment_history slots, ascending slot id
    std::vector<int32_t> leaf_order;       // pixel ids; slot s's members = leaf_order[seg_begin, + size)
    std::vector<int32_t> label;            // overlay label per pixel (draw.cpp:118-147), -1 = none
    std::vector<double> segment_scores;    // Forest::segment_scores (graph.cpp:139, :326), H*W
    std::vector<int32_t> final_roots;      // {root, xmin, ymin, xmax, ymax} of every final union-find root
    dofs_stats stats{};

    std::set<int> members(const dofs_snapshot& s) const {
        return std::set<int>(leaf_order.begin() + s.seg_begin, leaf_order.begin() + s.seg_begin + s.size);
    }
    // Forest::get_best_segments (graph.cpp:391-429): all H*W history slots; empty ones default-constructed
    // (score -1), the others SegmentData(score, seg, sol, move) as new_merge stores them (graph.cpp:354).
    template <class SegmentDataT = DefaultSegmentData, class SolutionT = DefaultSolution>
    std::vector<SegmentDataT> get_best_segments() const {
        static_assert(!std::is_void_v<SegmentDataT>, "name the SegmentData type (or include graph.hpp first)");
        std::vector<SegmentDataT> h((size_t)width * height);
        for (const dofs_snapshot& s : snapshots)
            h[(size_t)s.slot] = SegmentDataT(s.score, members(s), to_solution<SolutionT>(s.sol), s.move);
        return h;
    }
    // Forest::get_bounding_box (graph.cpp:446-452) after the loop: {(xmin, ymin), (xmax, ymax)} inclusive
    // for a final union-find root, the empty vector for every other id (merge cleared it, graph.cpp:208).
    std::vector<cv::Point2i> get_bounding_box(int node_id) const {
        for (size_t k = 0; k + 4 < final_roots.size(); k += 5)
            if (final_roots[k] == node_id)
                return {cv::Point2i(final_roots[k + 1], final_roots[k + 2]), cv::Point2i(final_roots[k + 3], final_roots[k + 4])};
        return {};
    }
    // Forest::get_segment_best_score (graph.cpp:386-389): the score of root node_id's LAST scored
    // candidate (written before the convexity / threshold tests, graph.cpp:326), 0.0 if it had none.
    double get_segment_best_score(int node_id) const { return segment_scores.at((size_t)node_id); }
    // Not a Forest accessor: a history slot's box at its winning merge (the snapshot's box).
    std::vector<cv::Point2i> get_snapshot_bounding_box(int slot) const {
        for (const dofs_snapshot& s : snapshots)
            if (s.slot == slot) return {cv::Point2i(s.bbox[0], s.bbox[1]), cv::Point2i(s.bbox[2], s.bbox[3])};
        throw std::runtime_error("dofs_cv: slot has no snapshot");
    }
    // The overlay label map (CV_32S, H x W): the largest slot with score > 0.7 containing the pixel, else -1.
    cv::Mat labels() const {
        cv::Mat m(height, width, CV_32S);
        std::memcpy(m.data, label.data(), sizeof(int32_t) * label.size());
        return m;
    }
};

namespace detail {
inline void check_flow(const cv::Mat& flow) {
    if (flow.type() != CV_32FC2 || flow.dims != 2) throw std::runtime_error("dofs_cv: flow must be CV_32FC2");
}
// Runs `call(result)` with growing snapshot capacity.
template <class Call>
Segmentation collect(const cv::Mat& flow, bool want_blur, std::vector<float>* blurred, Call&& call) {
    Segmentation r;
    r.width = flow.cols;
    r.height = flow.rows;
    const size_t N = (size_t)flow.rows * flow.cols;
    r.leaf_order.resize(N);
    r.label.resize(N);
    if (want_blur) blurred->resize(2 * N);
    for (int32_t cap = 4096;; cap *= 2) {
        r.snapshots.resize((size_t)cap);
        dofs_result res{};
        res.snapshots = r.snapshots.data();
        res.snapshot_capacity = cap;
        res.labels = r.label.data();
        res.leaf_order = r.leaf_order.data();
        res.blurred = want_blur ? blurred->data() : nullptr;
        const int32_t rc = call(res);
        if (rc == DOFS_ERR_CAPACITY && res.n_snapshots > cap) continue;
        check(rc, "segment");
        r.snapshots.resize((size_t)res.n_snapshots);
        r.stats = res.stats;
        // the Forest state after the loop: segment_scores and the final roots' boxes
        r.segment_scores.resize(N);
        check(dofs_segment_scores(context(), -1, 0, r.segment_scores.data(), (int64_t)N), "segment_scores");
        int64_t n = 0;
        check(dofs_final_roots(context(), -1, 0, nullptr, 0, &n), "final_roots");
        r.final_roots.resize(5 * (size_t)n);
        check(dofs_final_roots(context(), -1, 0, r.final_roots.data(), n, &n), "final_roots");
        return r;
    }
}
}  // namespace detail

// get_segmented_array (segment.cpp:34-72). bev is unused by the path (graph.hpp:78, graph.cpp:133).
inline Segmentation get_segmented_array(const cv::Mat& flow, const cv::Mat& bev, const cv::Matx33f& persp,
                                        const cv::Matx33f& inv, const std::vector<cv::Matx33f>& inv_upper,
                                        int neighbor = 8, bool blur_in_place = true) {
    (void)bev;
    detail::check_flow(flow);
    float p[9], i[9], u[27];
    mats(persp, inv, inv_upper, p, i, u);
    dofs_params prm;
    dofs_default_params(&prm);
    prm.neighbor = neighbor;
    std::vector<float> blurred;
    Segmentation r = detail::collect(flow, blur_in_place, &blurred, [&](dofs_result& res) {
        return dofs_segment(context(), flow.ptr<float>(), flow.rows, flow.cols, flow.step, p, i, u, &prm, &res);
    });
    if (blur_in_place)  // cv::GaussianBlur(flow, flow, ...) mutates the caller's field (segment.cpp:52)
        for (int y = 0; y < flow.rows; ++y)
            std::memcpy(const_cast<float*>(flow.ptr<float>(y)), blurred.data() + (size_t)2 * flow.cols * y,
                        sizeof(float) * 2 * flow.cols);
    return r;
}

// build_graph (graph.cpp:51-103): the weight is the reference's diff (segment.cpp:20-32), the only
// DiffFunction the reference passes; EdgeT must have Edge's {int start; int end; double weight;} layout.
template <class EdgeT = DefaultEdge>
std::vector<EdgeT> build_graph(const cv::Mat& img, int width, int height, bool neighborhood_8 = false) {
    static_assert(sizeof(EdgeT) == sizeof(dofs_edge), "EdgeT must be {int start; int end; double weight;}");
    detail::check_flow(img);
    if (width != img.cols || height != img.rows) throw std::runtime_error("dofs_cv: width / height != img size");
    int64_t n = 0;
    const int64_t cap = 4 * (int64_t)width * height;
    std::vector<EdgeT> out((size_t)cap);
    check(dofs_build_graph(context(), img.ptr<float>(), height, width, img.step, neighborhood_8 ? 1 : 0,
                           reinterpret_cast<dofs_edge*>(out.data()), cap, &n),
          "build_graph");
    out.resize((size_t)n);
    return out;
}
template <class EdgeT = DefaultEdge, class Diff>
std::vector<EdgeT> build_graph(const cv::Mat& img, int width, int height, const Diff& /*reference diff*/,
                               bool neighborhood_8 = false) {
    return build_graph<EdgeT>(img, width, height, neighborhood_8);
}

// segment_graph (graph.cpp:503-536): Kruskal over the caller's list in its order, on the flow as given.
template <class EdgeT>
Segmentation segment_graph(const cv::Mat& flow, const std::vector<EdgeT>& edges, const cv::Mat& bev,
                           const cv::Matx33f& persp, const cv::Matx33f& inv, const std::vector<cv::Matx33f>& inv_upper) {
    static_assert(sizeof(EdgeT) == sizeof(dofs_edge), "EdgeT must be {int start; int end; double weight;}");
    (void)bev;
    detail::check_flow(flow);
    float p[9], i[9], u[27];
    mats(persp, inv, inv_upper, p, i, u);
    dofs_params prm;
    dofs_default_params(&prm);
    return detail::collect(flow, false, nullptr, [&](dofs_result& res) {
        return dofs_segment_graph(context(), flow.ptr<float>(), flow.rows, flow.cols, flow.step,
                                  reinterpret_cast<const dofs_edge*>(edges.data()), (int64_t)edges.size(), p, i, u,
                                  &prm, &res);
    });
}

// get_bottom_variants (lifting_3d.cpp:350-439), on the device.
template <class SolutionT = DefaultSolution>
SolutionT get_bottom_variants(const cv::Point2f& dir, const std::vector<cv::Point2i>& box_2d, const cv::Matx33f& mat,
                              const cv::Matx33f& inv_mat, const cv::Matx33f& inv_matrix_upper, int cls) {
    if (box_2d.size() < 2) throw std::runtime_error("dofs_cv: box_2d needs {min, max} corners");
    const float d[2] = {dir.x, dir.y};
    const int32_t box[4] = {box_2d[0].x, box_2d[0].y, box_2d[1].x, box_2d[1].y};
    float m[9], i[9], u[9];
    to9(mat, m);
    to9(inv_mat, i);
    to9(inv_matrix_upper, u);
    dofs_solution s;
    check(dofs_lift(context(), d, box, m, i, u, cls, &s), "get_bottom_variants");
    return to_solution<SolutionT>(s);
}

// get_mat (lifting_3d.cpp:482-514) and get_mat_upper (:441-480): host code, no device needed.
inline std::pair<cv::Matx33f, cv::Matx33f> get_mat() {
    float p[9], i[9], u[27];
    if (dofs_calib(p, i, u) != DOFS_OK) throw std::runtime_error("dofs_cv: dofs_calib failed");
    return {from9(p), from9(i)};
}
inline cv::Matx33f get_mat_upper(int cls) {
    float p[9], i[9], u[27];
    if (cls < 0 || cls > 2 || dofs_calib(p, i, u) != DOFS_OK) throw std::runtime_error("dofs_cv: get_mat_upper");
    return from9(u + 9 * cls);
}

// get_intersect (lifting_3d.cpp:63-110): host code.
inline cv::Point2f get_intersect(cv::Point2f a1, cv::Point2f a2, cv::Point2f b1, cv::Point2f b2) {
    const float A1[2] = {a1.x, a1.y}, A2[2] = {a2.x, a2.y}, B1[2] = {b1.x, b1.y}, B2[2] = {b2.x, b2.y};
    float r[2];
    dofs_intersect(A1, A2, B1, B2, r);
    return cv::Point2f(r[0], r[1]);
}

// get_upper_face (lifting_3d.cpp:290-348) and get_upper_face_simple (:261-288): host code.
namespace detail {
template <class F>
std::vector<cv::Point2f> upper(const std::vector<cv::Point2i>& box_2d, const std::vector<cv::Point2f>& lower_face, F f) {
    if (box_2d.size() < 2 || lower_face.size() < 4) throw std::runtime_error("dofs_cv: box_2d / lower_face size");
    const int32_t box[4] = {box_2d[0].x, box_2d[0].y, box_2d[1].x, box_2d[1].y};
    float lf[8], uf[8];
    for (int k = 0; k < 4; ++k) lf[2 * k] = lower_face[k].x, lf[2 * k + 1] = lower_face[k].y;
    f(box, lf, uf);
    std::vector<cv::Point2f> out;
    for (int k = 0; k < 4; ++k) out.emplace_back(uf[2 * k], uf[2 * k + 1]);
    return out;
}
}  // namespace detail
inline std::vector<cv::Point2f> get_upper_face(const std::vector<cv::Point2i>& box_2d,
                                               const std::vector<cv::Point2f>& lower_face) {
    return detail::upper(box_2d, lower_face, dofs_upper_face);
}
inline std::vector<cv::Point2f> get_upper_face_simple(std::vector<cv::Point2i> box_2d, std::vector<cv::Point2f> lower_face) {
    return detail::upper(box_2d, lower_face, dofs_upper_face_simple);
}

// get_obj_size (lifting_3d.cpp:524-528): host code.
inline std::pair<double, double> get_obj_size(int cls) {
    double o[2];
    if (dofs_obj_size(cls, o) != DOFS_OK) throw std::runtime_error("dofs_cv: get_obj_size: cls must be 0..2");
    return {o[0], o[1]};
}

}  // namespace dofs_cv
#endif  // DOFS_CV_HAVE_OPENCV
