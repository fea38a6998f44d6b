// Compile-and-behaviour test of include/dofs_cv.hpp (the reference's OpenCV signatures over include/dofs.h),
// built against the test double in mock/ (OpenCV is absent here). The reference's graph.hpp data types are
// restated below with the shapes its header declares (graph.hpp:13-57) so the adapter's default template
// arguments are exercised as in a real reference build. CPU: get_mat / get_mat_upper / get_intersect
// (test_liftig_3d.cpp:69-89, :183-185). "device": get_segmented_array, build_graph + segment_graph,
// get_best_segments, get_bounding_box and get_bottom_variants on the reference's KAT (:179-227, tol 0.1).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <set>
#include <vector>

#include <opencv2/core.hpp>

// --- stand-ins for the reference's graph.hpp types (field order and constructors as declared there) ---
#define GRAPH_HPP 1
struct Edge {
    int start;
    int end;
    double weight;
};
class Solution {
public:
    int cls;
    std::vector<cv::Point2f> ps_bev, lower_face, upper_face, rectangle;
    double w_error, h_error, orient;
    Solution() : cls(0), w_error(-1.0), h_error(-1.0), orient(0) {}
    Solution(int c, const std::vector<cv::Point2f>& a, const std::vector<cv::Point2f>& b,
             const std::vector<cv::Point2f>& u, const std::vector<cv::Point2f>& r, double we, double he, double o)
        : cls(c), ps_bev(a), lower_face(b), upper_face(u), rectangle(r), w_error(we), h_error(he), orient(o) {}
};
class SegmentData {
public:
    double score;
    std::set<int> seg;
    Solution sol;
    double move;
    SegmentData() : score(-1.0), move(0) {}
    SegmentData(double s, const std::set<int>& g, const Solution& so, double m) : score(s), seg(g), sol(so), move(m) {}
};

#include "dofs_cv.hpp"

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

static double diff_unused(const cv::Mat&, int, int, int, int) { return 0.0; }  // a DiffFunction-shaped argument

static cv::Mat synth(int H, int W) {  // noise plus two moving boxes
    cv::Mat m(H, W, CV_32FC2);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            uint32_t h = (uint32_t)(y * 7919 + x * 104729) * 2654435761u;
            float* p = m.ptr<float>(y) + 2 * x;
            p[0] = (float)((int)(h >> 24) % 41 - 20) / 256.f;
            p[1] = (float)((int)((h >> 16) & 0xFF) % 41 - 20) / 256.f;
            if (x > W / 2 && x < W * 9 / 10 && y > H / 4 && y < H * 8 / 10) p[0] = 2.5f, p[1] = 1.9f;
            if (x > W / 10 && x < W / 3 && y > H * 4 / 10 && y < H * 3 / 4) p[0] = -1.8f, p[1] = 0.6f;
        }
    return m;
}

int main(int argc, char** argv) {
    auto [persp, inv] = dofs_cv::get_mat();
    float p9[9], i9[9], u27[27];
    CHECK(dofs_calib(p9, i9, u27) == DOFS_OK);
    for (int k = 0; k < 9; ++k) CHECK(persp.val[k] == p9[k] && inv.val[k] == i9[k]);
    const cv::Matx33f up2 = dofs_cv::get_mat_upper(2);
    for (int k = 0; k < 9; ++k) CHECK(up2.val[k] == u27[18 + k]);
    // test_liftig_3d.cpp:183-185: get_mat / get_mat_upper(2) literals
    CHECK(std::fabs(persp(0, 0) - 20.1377838f) < 1e-3f && std::fabs(inv(2, 1) + 4.97462083e-05f) < 1e-9f);
    const cv::Point2f r = dofs_cv::get_intersect({1, 1}, {4, 4}, {1, 8}, {2, 4});  // :69-78
    CHECK(std::fabs(r.x - 2.4f) < 1e-2f && std::fabs(r.y - 2.4f) < 1e-2f);
    const cv::Point2f n = dofs_cv::get_intersect({1, 1}, {1, 2}, {3, 3}, {3, 4});  // :80-89
    CHECK(std::isnan(n.x) && std::isnan(n.y));
    // get_upper_face / get_upper_face_simple / get_obj_size (lifting_3d.hpp:21-25): host code, same results
    // as the C-ABI entries (which tests/test_forest_accessors.py pins against the oracle)
    {
        const std::vector<cv::Point2i> box = {cv::Point2i(375, 92), cv::Point2i(576, 286)};
        const std::vector<cv::Point2f> lf = {{385.3f, 283.1f}, {380.2f, 215.7f}, {560.9f, 210.4f}, {570.5f, 280.6f}};
        const int32_t b4[4] = {375, 92, 576, 286};
        float l8[8], u8[8];
        for (int k = 0; k < 4; ++k) l8[2 * k] = lf[k].x, l8[2 * k + 1] = lf[k].y;
        std::vector<cv::Point2f> u = dofs_cv::get_upper_face(box, lf);
        dofs_upper_face(b4, l8, u8);
        CHECK(u.size() == 4 && u[2].x == u8[4] && u[2].y == 92.0f && u[0].x == u8[0] && u[3].y == u8[7]);
        std::vector<cv::Point2f> us = dofs_cv::get_upper_face_simple(box, lf);
        dofs_upper_face_simple(b4, l8, u8);
        CHECK(us.size() == 4 && us[1].y == u8[3] && us[0].x == lf[0].x);
        CHECK(us[1].y == lf[1].y - (float)(0 - 92.0 + (double)std::min(lf[1].y, lf[2].y)));  // :272-277
        CHECK(dofs_cv::get_obj_size(1) == std::make_pair(349.0, 165.0));
        bool threw = false;
        try {
            dofs_cv::get_obj_size(3);
        } catch (const std::runtime_error&) {
            threw = true;
        }
        CHECK(threw);
    }

    if (argc > 1 && std::strcmp(argv[1], "device") == 0) {
        std::vector<cv::Matx33f> ups = {dofs_cv::get_mat_upper(0), dofs_cv::get_mat_upper(1), up2};
        const int H = 90, W = 160;
        cv::Mat flow = synth(H, W), orig = flow.clone(), bev;
        dofs_cv::Segmentation a = dofs_cv::get_segmented_array(flow, bev, persp, inv, ups);
        CHECK(a.stats.n_merges == (int64_t)H * W - 1 && !a.snapshots.empty());
        // the field was blurred in place (segment.cpp:52): segmenting the blurred field's sorted edge list
        // through build_graph + segment_graph gives the same history
        CHECK(std::memcmp(flow.data, orig.data, (size_t)H * W * 8) != 0);
        std::vector<Edge> edges = dofs_cv::build_graph<Edge>(flow, W, H, diff_unused, true);
        CHECK(edges.size() == (size_t)(4 * W * H - 3 * W - 3 * H + 2));
        for (size_t k = 1; k < edges.size(); ++k) CHECK(edges[k - 1].weight <= edges[k].weight);
        dofs_cv::Segmentation b = dofs_cv::segment_graph(flow, edges, bev, persp, inv, ups);
        CHECK(a.snapshots.size() == b.snapshots.size());
        for (size_t k = 0; k < a.snapshots.size() && k < b.snapshots.size(); ++k) {
            CHECK(a.snapshots[k].slot == b.snapshots[k].slot && a.snapshots[k].event == b.snapshots[k].event);
            CHECK(a.snapshots[k].score == b.snapshots[k].score && a.members(a.snapshots[k]) == b.members(b.snapshots[k]));
        }
        CHECK(a.label == b.label);
        // Forest::get_best_segments: all H*W slots, the non-empty ones carrying seg / sol / move
        std::vector<SegmentData> hist = a.get_best_segments();
        CHECK(hist.size() == (size_t)H * W);
        size_t nonempty = 0;
        for (const SegmentData& s : hist) nonempty += s.score != -1.0;
        CHECK(nonempty == a.snapshots.size());
        const dofs_snapshot& s0 = a.snapshots[0];
        CHECK((int)hist[s0.slot].seg.size() == s0.size && hist[s0.slot].sol.cls == s0.sol.cls);
        std::vector<cv::Point2i> bb = a.get_snapshot_bounding_box(s0.slot);
        CHECK(bb[0].x == s0.bbox[0] && bb[1].y == s0.bbox[3]);
        // Forest::get_bounding_box after the loop: only the final root keeps a box — the whole frame
        CHECK(a.final_roots.size() == 5);
        if (a.final_roots.size() == 5) {
            std::vector<cv::Point2i> fb = a.get_bounding_box(a.final_roots[0]);
            CHECK(fb.size() == 2 && fb[0].x == 0 && fb[0].y == 0 && fb[1].x == W - 1 && fb[1].y == H - 1);
            CHECK(a.get_bounding_box(a.final_roots[0] == 0 ? 1 : 0).empty());
        }
        // get_segment_best_score: a scored slot's last score (the snapshot slots were all scored)
        for (const dofs_snapshot& s : a.snapshots) CHECK(a.get_segment_best_score(s.slot) != 0.0);
        CHECK(a.segment_scores == b.segment_scores && a.final_roots == b.final_roots);
        cv::Mat lab = a.labels();
        CHECK(lab.rows == H && lab.cols == W && lab.type() == CV_32S);
        // get_bottom_variants on the reference's KAT (test_liftig_3d.cpp:179-227, tolerance 0.1)
        cv::Matx33f km, ki, ku;
        const float M[9] = {20.1377838f, -13.4744920f, 402.174272f, 5.11635077f, 800.335022f, -62251.3321f,
                            0.000393565444f, 0.0397205947f, 1.0f};
        const float I[9] = {0.202212552f, 0.00181942728f, 31.9370859f, -0.00182975914f, 0.00123437589f, 77.5774258f,
                            -6.90475148e-06f, -4.97462083e-05f, 1.0f};
        const float U[9] = {0.203701900f, 0.00169508037f, 32.3672674f, 0.0f, 0.00146371164f, 29.6614710f, 0.0f,
                            -5.01704822e-05f, 1.0f};
        for (int k = 0; k < 9; ++k) km.val[k] = M[k], ki.val[k] = I[k], ku.val[k] = U[k];
        Solution sol = dofs_cv::get_bottom_variants(cv::Point2f(2.5470946f, 1.9316475f),
                                                    {cv::Point2i(375, 92), cv::Point2i(576, 286)}, km, ki, ku, 2);
        CHECK(sol.cls == 2 && sol.lower_face.size() == 4 && sol.upper_face.size() == 4);
        if (sol.lower_face.size() == 4) {
            CHECK(std::fabs(sol.lower_face[0].x - 385.305f) < 0.1f && std::fabs(sol.upper_face[2].y - 92.0f) < 0.1f);
            CHECK(std::fabs(sol.w_error - 0.5987518562843858) < 0.1 && std::fabs(sol.h_error - 0.7156805292391223) < 0.1);
            CHECK(std::fabs(sol.orient + 1.6261444189491607) < 0.1);
        }
    }
    if (fails) return 1;
    std::printf("cv adapter ok\n");
    return 0;
}
