// dofs_api.h — implementation of the C-ABI of include/dofs.h over a pipeline backend.
// dofs_hip.hip instantiates it with the HIP backend and exports the extern "C" symbols.
#pragma once

#include <stdio.h>
#include <string.h>

#include <stdlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "dofs_knobs.h"
#include "dofs_overlay.h"
#include "dofs_pipeline.h"

namespace dofs {

// ---- host-side constants (boundary helpers, not on the hot path) ------------------------------

inline void default_params(dofs_params* p) {
    p->blur_sigma = 3.0;              // segment.cpp:52
    p->neighbor = 8;                  // segment.cpp:154
    p->min_size = 500;                // graph.hpp:93
    p->score_threshold = 0.3;         // graph.hpp:93
    p->overlay_min_score = 0.7;       // segment.cpp:166
    p->min_convexity[0] = 3.0 / 4.0;  // graph.cpp:328-339
    p->min_convexity[1] = 1.0 / 2.0;
    p->min_convexity[2] = 20.0 / 29.0;
    const int sz[3][2] = {{258, 84}, {349, 165}, {370, 180}};  // lifting_3d.cpp:257
    for (int c = 0; c < 3; ++c) {
        p->obj_size[c][0] = sz[c][0];
        p->obj_size[c][1] = sz[c][1];
    }
}

// cv::getPerspectiveTransform: 8x8 system (float point products), Gaussian elimination with
// partial pivoting in double, back substitution by division, M(2,2) = 1.
inline void perspective_transform(const float src[4][2], const float dst[4][2], float out[9]) {
    double a[8][9];
    for (int i = 0; i < 4; ++i) {
        const float sx = src[i][0], sy = src[i][1], dx = dst[i][0], dy = dst[i][1];
        double* r0 = a[i];
        double* r1 = a[i + 4];
        for (int j = 0; j < 9; ++j) r0[j] = r1[j] = 0.0;
        r0[0] = r1[3] = sx;
        r0[1] = r1[4] = sy;
        r0[2] = r1[5] = 1.0;
        r0[6] = -sx * dx;
        r0[7] = -sy * dx;
        r1[6] = -sx * dy;
        r1[7] = -sy * dy;
        r0[8] = dx;
        r1[8] = dy;
    }
    for (int c = 0; c < 8; ++c) {
        int piv = c;
        for (int r = c + 1; r < 8; ++r)
            if (fabs(a[r][c]) > fabs(a[piv][c])) piv = r;
        if (piv != c)
            for (int j = c; j < 9; ++j) {
                double t = a[c][j];
                a[c][j] = a[piv][j];
                a[piv][j] = t;
            }
        const double nd = -1 / a[c][c];
        for (int r = c + 1; r < 8; ++r) {
            const double al = a[r][c] * nd;
            for (int j = c + 1; j < 9; ++j) a[r][j] += al * a[c][j];
        }
    }
    double x[8];
    for (int r = 7; r >= 0; --r) {
        double s = a[r][8];
        for (int j = r + 1; j < 8; ++j) s -= a[r][j] * x[j];
        x[r] = s / a[r][r];
    }
    for (int i = 0; i < 8; ++i) out[i] = (float)x[i];
    out[8] = 1.0f;
}

// get_mat (lifting_3d.cpp:482-514) + get_mat_upper (:441-480)
inline void calib(float persp[9], float inv[9], float inv_upper[27]) {
    const float bev[4][2] = {{100.f, 13000.f}, {100.f, 6000.f}, {800.f, 6000.f}, {800.f, 13000.f}};
    const float img[4][2] = {{215.f, 265.f}, {90.f, 121.f}, {294.f, 120.f}, {625.f, 265.f}};
    perspective_transform(img, bev, persp);
    perspective_transform(bev, img, inv);
    const float up[3][4][2] = {{{215, 176}, {90, 85}, {294, 85}, {625, 176}},
                               {{215, 185}, {90, 80}, {294, 80}, {625, 185}},
                               {{215, 140}, {90, 55}, {294, 55}, {625, 140}}};
    for (int c = 0; c < 3; ++c) perspective_transform(bev, up[c], inv_upper + 9 * c);
}

inline int64_t graph_edges(int H, int W, bool nbr8) {  // build_graph size (graph.cpp:62-93)
    int64_t e = (int64_t)(W - 1) * H + (int64_t)W * (H - 1);
    if (nbr8) e += 2 * (int64_t)(W - 1) * (H - 1);
    return e;
}

struct KLiftBatch {
    const F2* dirs;
    const int* boxes;
    const int* cls;
    dofs_solution* out;
    LiftMats L;
    DOFS_HD void operator()(int, int64_t i) const {
        lift_one(mk(dirs[i].x, dirs[i].y), boxes + 4 * i, L, cls[i], out + i);
    }
};

// get_intersect (lifting_3d.cpp:63-89) on the device: the same intersect() the lifting kernels call
struct KIntersectBatch {
    const float* pts;  // n x (a1, a2, b1, b2) x (x, y)
    float* out;        // n x 2
    DOFS_HD void operator()(int, int64_t i) const {
        const float* q = pts + 8 * i;
        P2 r = intersect(mk(q[0], q[1]), mk(q[2], q[3]), mk(q[4], q[5]), mk(q[6], q[7]));
        out[2 * i] = r.x;
        out[2 * i + 1] = r.y;
    }
};

// Synthetic benchmark flow (DESIGN.md §Synthetic input): splitmix64 noise quantised to 2^-10 in
// [-0.0996, 0.0996] plus three constant-flow rectangles, jittered by ±5 % for seeds != 0.
DOFS_HD inline unsigned long long splitmix64(unsigned long long x) {
    unsigned long long z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
DOFS_HD inline int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

struct KSynth {
    F2* out;
    int H, W;
    unsigned long long seed0;
    DOFS_HD void operator()(int f, int64_t p) const {
        const unsigned long long seed = seed0 + (unsigned long long)f;
        const int64_t N = (int64_t)H * W;
        F2 v;
        {
            unsigned long long z0 = splitmix64((seed << 32) + (unsigned long long)(2 * p));
            unsigned long long z1 = splitmix64((seed << 32) + (unsigned long long)(2 * p + 1));
            v.x = (float)((int)((z0 >> 11) % 205ull) - 102) * (1.0f / 1024.0f);
            v.y = (float)((int)((z1 >> 11) % 205ull) - 102) * (1.0f / 1024.0f);
        }
        const int x = (int)(p % W), y = (int)(p / W);
        const int rect[3][4] = {{550, 900, 250, 800}, {100, 350, 400, 750}, {400, 500, 500, 900}};
        const float uv[3][2] = {{2.5f, 1.9f}, {-1.8f, 0.6f}, {0.3f, 2.2f}};
        for (int r = 0; r < 3; ++r) {
            int x0 = (int)((int64_t)W * rect[r][0] / 1000), x1 = (int)((int64_t)W * rect[r][1] / 1000);
            int y0 = (int)((int64_t)H * rect[r][2] / 1000), y1 = (int)((int64_t)H * rect[r][3] / 1000);
            if (seed != 0) {
                unsigned long long zx = splitmix64((seed << 32) + 0xF0000000ull + 2ull * r);
                unsigned long long zy = splitmix64((seed << 32) + 0xF0000000ull + 2ull * r + 1);
                int jx = (int)((int64_t)(zx % 101ull) * W / 1000) - (int)((int64_t)50 * W / 1000);
                int jy = (int)((int64_t)(zy % 101ull) * H / 1000) - (int)((int64_t)50 * H / 1000);
                x0 = clampi(x0 + jx, 0, W);
                x1 = clampi(x1 + jx, 0, W);
                y0 = clampi(y0 + jy, 0, H);
                y1 = clampi(y1 + jy, 0, H);
            }
            if (x >= x0 && x < x1 && y >= y0 && y < y1) {
                v.x = uv[r][0];
                v.y = uv[r][1];
            }
        }
        out[(int64_t)f * N + p] = v;
    }
};

// ---- context -----------------------------------------------------------------------------------

// the message of DOFS_ERR_INVALID_RESULT, which every result accessor returns for a batch whose C_FLOWERR is set
inline std::string result_err_msg(int bits) {
    std::string m = "the results of this batch are invalid:";
    if (bits & kErrGiveUp) m += " its replay gave up a bounded wait;";
    if (bits & kErrRecord) m += " a replay record held a union-find root outside its frame (refused on the device);";
    if (bits & kErrMst) m += " a frame's minimum spanning tree did not have N - 1 edges;";
    return m;
}

template <class Backend>
struct Context {
    // Workspaces used in turn by consecutive batches (kSlots). A batch runs
    // phase A (graph) on stream sA and phase B (replay + scoring) on stream sB, so batch k's phase B
    // overlaps the next batches' phase A. A workspace is reused only after its previous batch's
    // phase B (evDone) ended: with three, the latency-bound phase B of batch k may run as long as
    // the phase A of batches k+1 and k+2 together before it holds the graph stage up.
    static constexpr int kSlots = 3;
    struct Meta {
        int B = 0, H = 0, W = 0;
        dofs_params prm;
        int64_t n_edges = -1;  // segment_graph: the caller's edge count (else build_graph's)
        int64_t mreal = -1;    // segment_graph: merges of the caller's graph (else H*W - 1)
        bool lean = false;     // the batch kept only the replay records its results read (no dofs_events)
    };
    Backend be;
    Pipeline<Backend> p0, p1, p2;
    Pipeline<Backend> pband;  // row-band minimum spanning forests (api_band_msf)
    std::string err;
    void* d_in = nullptr;
    size_t d_in_bytes = 0;
    void* d_scratch = nullptr;
    size_t d_scratch_bytes = 0;
    void* d_graph = nullptr;  // caller edge lists (segment_graph) and build_graph's sort buffers
    size_t d_graph_bytes = 0;
    int* d_lmap[kSlots] = {nullptr, nullptr, nullptr};  // overlay edge maps per workspace (api_overlay)
    size_t d_lmap_bytes[kSlots] = {0, 0, 0};
    int64_t nbatch = 0;  // batches issued; batch id b uses workspace b % nslots
    int nslots = kSlots;
    int64_t snap_cap = 4096;
    bool used[kSlots] = {false, false, false};
    Meta meta[kSlots];
    void* sA = nullptr;
    void* sB = nullptr;
    void* evIn = nullptr;
    void* evA[kSlots] = {nullptr, nullptr, nullptr};
    void* evRead[kSlots] = {nullptr, nullptr, nullptr};  // the batch's input consumed (after the blur)
    void* evDone[kSlots] = {nullptr, nullptr, nullptr};

    bool serial = false;
    bool skip_b = false;  // DOFS_SKIP_B=1 (measurement builds only): graph stage alone, results invalid
    // dofs_keep_events: batches keep every merge's replay record for dofs_events (default: only the records
    // the results read — path tops, parked states, merges of >= min_size pixels; Ws::rv_lean)
    bool keep_events = false;

    Context(int device, const Knobs& knobs) : be(device, knobs), p0(be), p1(be), p2(be), pband(be) {
        const Knobs& kn = be.kn;  // the knobs dofs_create read for this context (dofs_knobs.h), kept by the backend
        serial = kn.serial != 0;
        skip_b = kn.skip_b != 0;
        p0.skip_mask = p1.skip_mask = p2.skip_mask = kn.skip_mask;
        if (kn.long_path > 0) p0.long_path = p1.long_path = p2.long_path = kn.long_path;
        p0.krt_mode = p1.krt_mode = p2.krt_mode = kn.krt_dnc;
        // stream priorities: the graph stage (Borůvka, sort, KRT) bounds the step, so its stream is the most
        // urgent and the replay + scoring stage's the least — a freed CU takes the graph stage's next
        // workgroup first (round 3, B = 112, same box: 1,559 / 1,561 Mpix/s against 1,499 / 1,499 with the
        // replay stage urgent and 1,253 / 1,255 with equal priorities); the long-path replay workers keep
        // a top-priority stream of their own
        sA = be.new_stream(1);
        sB = be.new_stream(-1);
        evIn = be.new_event();
        for (int s = 0; s < kSlots; ++s) {
            evA[s] = be.new_event();
            evRead[s] = be.new_event();
            evDone[s] = be.new_event();
        }
    }
    ~Context() {
        drain();
        if (d_in) be.free(d_in);
        if (d_scratch) be.free(d_scratch);
        if (d_graph) be.free(d_graph);
        for (int k = 0; k < kSlots; ++k)
            if (d_lmap[k]) be.free(d_lmap[k]);
    }
    Pipeline<Backend>& pipe(int slot) { return slot == 0 ? p0 : (slot == 1 ? p1 : p2); }
    int slot_of(int64_t id) const { return (int)(id % nslots); }
    bool have_batch() const { return nbatch > 0; }
    int last_slot() const { return slot_of(nbatch - 1); }
    // valid batch ids for result access: the last nslots issued
    bool live(int64_t id) const { return id >= 0 && id < nbatch && id >= nbatch - nslots; }
    // make the current stream wait for batch id's results
    void join(int64_t id) { be.wait(be.cur_stream(), evDone[slot_of(id)]); }
    void drain() {
        for (int s = 0; s < kSlots; ++s)
            if (used[s]) be.event_sync(evDone[s]);
    }
    void* scratch(size_t bytes) {
        if (bytes > d_scratch_bytes) {
            if (d_scratch) be.free(d_scratch);
            d_scratch = be.alloc(bytes);
            d_scratch_bytes = d_scratch ? bytes : 0;
        }
        return d_scratch;
    }
    void* graph_buf(size_t bytes) {
        if (bytes > d_graph_bytes) {
            if (d_graph) {
                be.sync();
                be.free(d_graph);
            }
            d_graph = be.alloc(bytes);
            d_graph_bytes = d_graph ? bytes : 0;
        }
        return d_graph;
    }
    int fail(int code, const std::string& msg) {
        err = msg;
        return code;
    }
    int check() {
        if (!be.ok()) return fail(DOFS_ERR_DEVICE, be.error());
        return DOFS_OK;
    }
};

// Waits for batch id `batch` and returns its result error bits (C_FLOWERR of frame 0: the replay gave up a
// bounded wait, or a record held an out-of-range root): every accessor of the batch's results then fails with
// DOFS_ERR_INVALID_RESULT instead of returning invalid data
template <class Backend>
int result_err(Context<Backend>* cx, int64_t batch) {
    const int slot = cx->slot_of(batch);
    cx->be.event_sync(cx->evDone[slot]);
    return cx->be.read_int(cx->pipe(slot).w.ctr + C_FLOWERR);
}
template <class Backend>
int fail_result(Context<Backend>* cx, int bits) {
    return cx->fail(DOFS_ERR_INVALID_RESULT, result_err_msg(bits));
}

// Enqueue one batch on the context's streams, ordered after the work already on the caller's
// (current) stream. On return the caller's stream is ordered after phase A, so it may overwrite
// the input; results are joined by api_fetch / api_events / api_records_copy.
template <class Backend>
int api_run(Context<Backend>* cx, const F2* d_flow, int64_t fstride, int B, int H, int W, const float persp[9],
            const float inv[9], const float inv_upper[27], const dofs_params* params,
            const unsigned char* allow = nullptr, const dofs_edge* d_edges = nullptr, int64_t n_edges = 0,
            int* d_acc = nullptr) {
    if (B <= 0 || H <= 0 || W <= 0 || !persp || !inv || !inv_upper) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    if (H > 32767 || W > 32767) return cx->fail(DOFS_ERR_INVALID_ARG, "H and W must be < 32768");
    if ((int64_t)H * W >= (1 << 26)) return cx->fail(DOFS_ERR_INVALID_ARG, "H*W must be < 2^26");
    // the dataflow replay's task words (frame * H*W + path, dofs_dataflow.h) must stay below its state words
    if ((int64_t)B * H * W > kMaxBatchPixels) return cx->fail(DOFS_ERR_INVALID_ARG, "B*H*W must be <= 2^30 - 16");
    dofs_params prm;
    if (params)
        prm = *params;
    else
        default_params(&prm);
    // segment.cpp:38-43: anything but 8 segments with the 4-neighbourhood (logged, not an error)
    const int nbr8 = prm.neighbor == 8 ? 1 : 0;
    Dims d = Pipeline<Backend>::dims_for(B, H, W, nbr8);
    Backend& be = cx->be;
    const int64_t id = cx->nbatch;
    const int s = cx->slot_of(id);
    Pipeline<Backend>& P = cx->pipe(s);
    if (P.snap_cap != cx->snap_cap) {
        P.snap_cap = cx->snap_cap;
        P.cap.B = 0;  // force a new layout
    }
    // the graph's arrays stay readable after the batch for dofs_events, and for a caller's edge list or
    // edge mask, whose graph may be a forest: dofs_final_roots reads the completion merges' KRT children
    const bool keep_graph = cx->keep_events || allow || d_edges || n_edges > 0;
    P.keep_graph = keep_graph;  // (fits() asks for a layout that keeps the graph when set)
    if (!P.fits(d) && cx->used[s]) be.event_sync(cx->evDone[s]);  // reallocation: batch id-2 must be done
    if (!P.reserve(d)) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    // the workspaces no batch has used yet take this shape now: their first batches then allocate
    // nothing (a hipMalloc of tens of GB takes seconds), whatever stream work follows
    for (int k = 0; k < cx->nslots; ++k) {
        Pipeline<Backend>& Q = cx->pipe(k);
        if (k == s || cx->used[k] || Q.fits(d)) continue;
        Q.snap_cap = cx->snap_cap;
        Q.keep_graph = keep_graph;
        if (!Q.reserve(d)) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    }
    P.set_params(prm, persp, inv, inv_upper);

    void* caller = be.cur_stream();
    // stage timing (and DOFS_SERIAL=1, for clean per-kernel profiles) runs the phases back to back
    const bool serial = be.profiling() || cx->serial;
    // the caller's own inputs beyond the flow (an edge list, an edge mask) are read past the blur: those
    // batches release the caller after the whole graph stage, on sA
    const bool own_in = allow || d_edges || n_edges > 0;
    void* sa = cx->sA;
    void* sb = serial ? cx->sA : cx->sB;
    be.record(cx->evIn, caller);
    be.wait(sa, cx->evIn);
    if (cx->used[s]) be.wait(sa, cx->evDone[s]);
    be.use(sa);
    P.w.allow = allow;
    int64_t mreal = d.M;
    if (d_edges || n_edges > 0) {  // segment_graph on the caller's edge list (one frame)
        mreal = P.run_a_edges(d_flow, d_edges, n_edges, d_acc, d_acc + n_edges);
        if (mreal < 0) return cx->fail(DOFS_ERR_INVALID_ARG, "too many edges");
    } else {
        P.ev_input = own_in ? nullptr : cx->evRead[s];  // recorded once the blur has read d_flow
        P.run_a(d_flow, fstride);
        P.ev_input = nullptr;
    }
    P.w.allow = nullptr;
    be.record(cx->evA[s], sa);
    if (sb != sa) be.wait(sb, cx->evA[s]);
    be.use(sb);
    // lean replay stores only the records the scoring reads; a forest (a caller's edge list that leaves
    // several components, mreal < M) runs full: dofs_final_roots reads the record of every component the
    // completion merges join, and a heavy child below min_size would not have one
    const bool lean = !cx->keep_events && mreal >= d.M;
    P.w.rv_lean = lean ? 1 : 0;
#ifdef DOFS_MEASURE
    if (be.kn.b_delay_us > 0) be.delay_us(be.kn.b_delay_us);  // (measurement: where stage B sits in the step)
#endif
    if (!cx->skip_b) P.run_b();
    be.record(cx->evDone[s], sb);
    be.wait(caller, own_in ? cx->evA[s] : cx->evRead[s]);
    be.use(caller);

    cx->used[s] = true;
    cx->nbatch = id + 1;
    auto& m = cx->meta[s];
    m.B = B;
    m.H = H;
    m.W = W;
    m.prm = prm;
    m.n_edges = (d_edges || n_edges > 0) ? n_edges : graph_edges(H, W, nbr8);
    m.mreal = mreal;
    m.lean = lean && Backend::kLeanReplay;
    return cx->check();
}

// One row band's minimum spanning forest (intra-frame sharding): flow rows
// [row0, row0 + rows) of an H x W frame must contain the band [r0, r1) and its blur halo.
// Synchronous on the caller's stream; uses a workspace of its own.
template <class Backend>
int api_band_msf(Context<Backend>* cx, const F2* d_rows, int row0, int rows, int H, int W, int r0, int r1,
                 const dofs_params* params, unsigned char* d_mask) {
    if (!d_rows || !d_mask || H <= 0 || W <= 0 || r0 < 0 || r1 > H || r0 >= r1 || rows <= 0)
        return cx->fail(DOFS_ERR_INVALID_ARG, "bad band");
    if ((int64_t)H * W >= (1 << 26) || H > 32767 || W > 32767) return cx->fail(DOFS_ERR_INVALID_ARG, "frame too large");
    dofs_params prm;
    if (params)
        prm = *params;
    else
        default_params(&prm);
    float taps[kMaxTaps];
    const int R = gaussian_taps(prm.blur_sigma, taps) / 2;
    const int need0 = r0 - R < 0 ? 0 : r0 - R, need1 = r1 + R > H ? H : r1 + R;
    if (row0 > need0 || row0 + rows < need1 || row0 < 0 || row0 + rows > H)
        return cx->fail(DOFS_ERR_INVALID_ARG, "flow rows must cover the band and its blur halo");
    const int nbr8 = prm.neighbor == 8 ? 1 : 0;
    Pipeline<Backend>& P = cx->pband;  // its own workspace: batches in flight are untouched
    if (!P.reserve(Pipeline<Backend>::dims_for(1, rows, W, nbr8))) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    const float z9[9] = {0};
    const float z27[27] = {0};
    P.set_params(prm, z9, z9, z27);
    P.run_band(d_rows, row0, rows, H, r0, r1, d_mask);
    cx->be.sync();
    return cx->check();
}

// Results of frame `frame` of batch id `batch` (one of the last nslots issued; -1 = the last).
template <class Backend>
int api_fetch(Context<Backend>* cx, int frame, dofs_result* out, int64_t batch = -1) {
    if (!cx->have_batch() || !out) return cx->fail(DOFS_ERR_INVALID_ARG, "no batch");
    if (batch < 0) batch = cx->nbatch - 1;
    if (!cx->live(batch)) return cx->fail(DOFS_ERR_INVALID_ARG, "batch no longer readable");
    const int slot = cx->slot_of(batch);
    const typename Context<Backend>::Meta& m = cx->meta[slot];
    if (frame < 0 || frame >= m.B) return cx->fail(DOFS_ERR_INVALID_ARG, "no frame");
    Backend& be = cx->be;
    cx->join(batch);
    const Ws& w = cx->pipe(slot).w;
    const Dims& d = w.d;
    int ctr[kCounters], ctr0[kCounters];
    be.d2h(ctr, w.ctr + (int64_t)frame * kCounters, sizeof(ctr));
    be.d2h(ctr0, w.ctr, sizeof(ctr0));
    be.sync();
    // the batch's results are invalid (a replay give-up or a refused record; never seen), reported rather than
    // returned
    if (ctr0[C_FLOWERR]) return fail_result(cx, ctr0[C_FLOWERR]);
    const int ns = ctr[C_SNAP];
    out->n_snapshots = ns;
    out->stats.n_edges = m.n_edges;
    out->stats.n_merges = m.mreal;
    out->stats.n_candidates = ctr[C_CAND];
    out->stats.n_scored = ctr[C_SCORED];
    out->stats.n_qualified = ctr[C_QUAL];
    out->stats.n_snapshots = ns;
    // labels, leaf order and blurred field are exact whatever the snapshot capacity (KPaint is per slot)
    if (out->labels) be.d2h(out->labels, w.labels + (int64_t)frame * d.N, sizeof(int) * (size_t)d.N);
    if (out->leaf_order) be.d2h(out->leaf_order, w.leaf_order + (int64_t)frame * d.N, sizeof(int) * (size_t)d.N);
    if (out->blurred) be.d2h(out->blurred, w.blur + (int64_t)frame * d.N, sizeof(F2) * (size_t)d.N);
    be.sync();
    if (ns > w.snap_cap || (out->snapshots && ns > out->snapshot_capacity))
        return cx->fail(DOFS_ERR_CAPACITY, "snapshot capacity");
    if (out->snapshots && ns) {
        be.d2h(out->snapshots, w.snaps + (int64_t)frame * w.snap_cap, sizeof(dofs_snapshot) * (size_t)ns);
        be.sync();
    }
    return cx->check();
}

// Forest::get_segment_best_score for every id (graph.cpp:386-389) of frame `frame` of batch id `batch`.
template <class Backend>
int api_segment_scores(Context<Backend>* cx, int64_t batch, int frame, double* out, int64_t capacity) {
    if (!cx->have_batch() || !out) return cx->fail(DOFS_ERR_INVALID_ARG, "no batch");
    if (batch < 0) batch = cx->nbatch - 1;
    if (!cx->live(batch)) return cx->fail(DOFS_ERR_INVALID_ARG, "batch no longer readable");
    const int slot = cx->slot_of(batch);
    if (frame < 0 || frame >= cx->meta[slot].B) return cx->fail(DOFS_ERR_INVALID_ARG, "no frame");
    Pipeline<Backend>& P = cx->pipe(slot);
    const int64_t N = P.w.d.N;
    if (capacity < N) return cx->fail(DOFS_ERR_CAPACITY, "score capacity (H*W doubles)");
    double* d = (double*)cx->scratch(sizeof(double) * (size_t)N);
    if (!d) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    Backend& be = cx->be;
    if (int e = result_err(cx, batch)) return fail_result(cx, e);
    cx->join(batch);
    if (P.w.d.M <= 0 || !P.pre)
        be.memset(d, 0, sizeof(double) * (size_t)N);
    else
        be.launch(1, N, KSegScores{P.w, P.pre, frame, d});
    be.d2h(out, d, sizeof(double) * (size_t)N);
    be.sync();
    return cx->check();
}

// Forest::get_bounding_box after the run (graph.cpp:446-452): the final union-find roots and their boxes,
// {root, xmin, ymin, xmax, ymax} ascending by root; *n = their number (min(n, capacity) written).
template <class Backend>
int api_final_roots(Context<Backend>* cx, int64_t batch, int frame, int32_t* out, int64_t capacity, int64_t* n) {
    if (!cx->have_batch() || (!out && capacity > 0)) return cx->fail(DOFS_ERR_INVALID_ARG, "no batch");
    if (batch < 0) batch = cx->nbatch - 1;
    if (!cx->live(batch)) return cx->fail(DOFS_ERR_INVALID_ARG, "batch no longer readable");
    const int slot = cx->slot_of(batch);
    if (frame < 0 || frame >= cx->meta[slot].B) return cx->fail(DOFS_ERR_INVALID_ARG, "no frame");
    Pipeline<Backend>& P = cx->pipe(slot);
    const Ws& w = P.w;
    const Dims& d = w.d;
    Backend& be = cx->be;
    if (int e = result_err(cx, batch)) return fail_result(cx, e);
    cx->join(batch);
    std::vector<int32_t> rec;
    if (d.M <= 0) {  // one pixel
        rec = {0, 0, 0, 0, 0};
    } else if (w.mreal >= d.M) {  // connected: the last merge's root keeps the frame's box
        int q = 0;
        RepVal r;
        be.d2h(&q, P.pre + (int64_t)frame * d.NL + d.N + d.M - 1, sizeof(int));
        be.sync();
        be.d2h(&r, w.Rv + (int64_t)frame * d.NL + q, sizeof(RepVal));
        be.sync();
        if ((unsigned)r.root >= (unsigned)d.N) return fail_result(cx, kErrRecord);
        rec = {r.root, r.bb.x0, r.bb.y0, r.bb.x1, r.bb.y1};
    } else {  // a forest: the components joined by the completion merges
        const int64_t k = d.M - w.mreal + 1;
        int32_t* dv = (int32_t*)cx->scratch(sizeof(int32_t) * 5 * (size_t)k);
        if (!dv) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
        be.launch(1, d.M - w.mreal, KFinalRoots{w, P.pre, frame, dv});
        rec.resize(5 * (size_t)k);
        be.d2h(rec.data(), dv, sizeof(int32_t) * rec.size());
        be.sync();
        if (int e = be.read_int(w.ctr + C_FLOWERR)) return fail_result(cx, e);  // (KFinalRoots checks every root)
        std::vector<int64_t> idx((size_t)k);
        for (int64_t i = 0; i < k; ++i) idx[(size_t)i] = i;
        std::sort(idx.begin(), idx.end(), [&](int64_t a, int64_t b) { return rec[5 * a] < rec[5 * b]; });
        std::vector<int32_t> sorted(rec.size());
        for (int64_t i = 0; i < k; ++i)
            for (int t = 0; t < 5; ++t) sorted[5 * i + t] = rec[5 * idx[(size_t)i] + t];
        rec.swap(sorted);
    }
    const int64_t cnt = (int64_t)rec.size() / 5;
    if (n) *n = cnt;
    for (int64_t i = 0; i < cnt && i < capacity; ++i) memcpy(out + 5 * i, rec.data() + 5 * i, 5 * sizeof(int32_t));
    return cx->check();
}

template <class Backend>
int api_events(Context<Backend>* cx, int frame, dofs_event* ev, int64_t capacity) {
    if (!cx->have_batch() || !ev) return cx->fail(DOFS_ERR_INVALID_ARG, "no batch");
    const int slot = cx->last_slot();
    if (frame < 0 || frame >= cx->meta[slot].B) return cx->fail(DOFS_ERR_INVALID_ARG, "no frame");
    if (cx->meta[slot].lean)
        return cx->fail(DOFS_ERR_INVALID_ARG, "the batch kept no event records: dofs_keep_events(ctx, 1) before it");
    if (int e = result_err(cx, cx->nbatch - 1)) return fail_result(cx, e);
    cx->join(cx->nbatch - 1);
    const Ws& w = cx->pipe(slot).w;
    const Dims& d = w.d;
    const int64_t M = cx->meta[slot].mreal;  // merges of the caller's graph (segment_graph: may be < H*W-1)
    if (capacity < M) return cx->fail(DOFS_ERR_CAPACITY, "event capacity");
    if (M <= 0) return DOFS_OK;
    Backend& be = cx->be;
    std::vector<int> eu((size_t)d.M), evv((size_t)d.M), pre((size_t)d.M), sz((size_t)d.M);
    std::vector<RepVal> rv((size_t)d.NL);
    std::vector<unsigned long long> key((size_t)d.M);
    const int64_t fo = (int64_t)frame * d.NL;
    be.d2h(eu.data(), w.EU + (int64_t)frame * d.M, 4 * (size_t)d.M);
    be.d2h(evv.data(), w.EV + (int64_t)frame * d.M, 4 * (size_t)d.M);
    const bool keys = cx->pipe(slot).keys_by_frame;
    std::vector<F2> bl(keys ? 0 : (size_t)d.N);
    if (keys)
        be.d2h(key.data(), w.key_out + (int64_t)frame * d.M, 8 * (size_t)d.M);
    else  // the batch-wide sort left the weights in global order: recompute them from the blurred field
        be.d2h(bl.data(), w.blur + (int64_t)frame * d.N, sizeof(F2) * (size_t)d.N);
    be.d2h(pre.data(), cx->pipe(slot).pre + fo + d.N, 4 * (size_t)d.M);
    be.d2h(rv.data(), w.Rv + fo, sizeof(RepVal) * (size_t)d.NL);
    be.d2h(sz.data(), w.SZ + fo + d.N, 4 * (size_t)d.M);
    be.sync();
    for (int64_t i = 0; i < M; ++i) {  // (the KRT sweep's singleton flags, Ws::single)
        eu[(size_t)i] &= kEndMask;
        evv[(size_t)i] &= kEndMask;
    }
    if (!keys)
        for (int64_t i = 0; i < M; ++i) {  // KMstEmit's edge_weight: float differences, double squares
            const F2 a = bl[(size_t)eu[i]], b = bl[(size_t)evv[i]];
            const double dx = a.x - b.x, dy = a.y - b.y;
            const double wt = sqrt(dx * dx + dy * dy);
            memcpy(&key[i], &wt, sizeof(double));
        }
    for (int64_t i = 0; i < M; ++i) {
        dofs_event& e = ev[i];
        const int q = pre[i];
        e.start = eu[i];
        e.end = evv[i];
        memcpy(&e.weight, &key[i], sizeof(double));
        const RepVal& r = rv[q];
        e.root = r.root;
        e.size = sz[i];
        e.rank = r.rank;
        e.bbox[0] = r.bb.x0;
        e.bbox[1] = r.bb.y0;
        e.bbox[2] = r.bb.x1;
        e.bbox[3] = r.bb.y1;
        e.mean[0] = r.mx;
        e.mean[1] = r.my;
    }
    return cx->check();
}

// The single-frame calls (dofs_segment, dofs_segment_graph) return every history slot: when the
// frame has more than the context's snapshot capacity, `rerun` runs it again with a capacity grown
// for this call only; the context's capacity (the batch API's, dofs_set_snapshot_capacity) is restored
// afterwards, so the next batch on that workspace re-lays it out at the caller's size.
template <class Backend, class Rerun>
int fetch_grown(Context<Backend>* cx, dofs_result* out, Rerun rerun) {
    int n = 0;
    cx->join(cx->nbatch - 1);
    cx->be.d2h(&n, cx->pipe(cx->last_slot()).w.ctr + C_SNAP, sizeof(int));
    cx->be.sync();
    if (n <= cx->snap_cap) return api_fetch(cx, 0, out);
    const int64_t keep = cx->snap_cap;
    while (cx->snap_cap < n) cx->snap_cap *= 2;
    int rc = rerun();
    if (!rc) rc = api_fetch(cx, 0, out);
    cx->snap_cap = keep;
    return rc;
}

template <class Backend>
int api_segment(Context<Backend>* cx, const float* flow, int H, int W, size_t stride, const float persp[9],
                const float inv[9], const float inv_upper[27], const dofs_params* params, dofs_result* out) {
    if (!flow || H <= 0 || W <= 0 || !out) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    const size_t row = (size_t)W * 2 * sizeof(float);
    if (stride == 0) stride = row;
    if (stride < row) return cx->fail(DOFS_ERR_INVALID_ARG, "row stride too small");
    const size_t bytes = row * (size_t)H;
    if (bytes > cx->d_in_bytes) {
        if (cx->d_in) cx->be.free(cx->d_in);
        cx->d_in = cx->be.alloc(bytes);
        cx->d_in_bytes = cx->d_in ? bytes : 0;
        if (!cx->d_in) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    }
    if (stride == row) {
        cx->be.h2d(cx->d_in, flow, bytes);
    } else {
        for (int y = 0; y < H; ++y)
            cx->be.h2d((char*)cx->d_in + row * y, (const char*)flow + stride * y, row);
    }
    int rc = api_run(cx, (const F2*)cx->d_in, (int64_t)H * W, 1, H, W, persp, inv, inv_upper, params);
    if (rc) return rc;
    // more history slots than the device snapshot capacity: run again with a capacity grown for this
    // call only (the batch API's capacity stays the one dofs_set_snapshot_capacity chose)
    return fetch_grown(cx, out, [&]() {
        return api_run(cx, (const F2*)cx->d_in, (int64_t)H * W, 1, H, W, persp, inv, inv_upper, params);
    });
}

// Upload a host flow field (row stride in bytes, 0 = packed) into the context's input buffer.
template <class Backend>
int upload_flow(Context<Backend>* cx, const float* flow, int H, int W, size_t stride) {
    const size_t row = (size_t)W * 2 * sizeof(float);
    if (stride == 0) stride = row;
    if (stride < row) return cx->fail(DOFS_ERR_INVALID_ARG, "row stride too small");
    const size_t bytes = row * (size_t)H;
    if (bytes > cx->d_in_bytes) {
        if (cx->d_in) {
            cx->be.sync();
            cx->be.free(cx->d_in);
        }
        cx->d_in = cx->be.alloc(bytes);
        cx->d_in_bytes = cx->d_in ? bytes : 0;
        if (!cx->d_in) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    }
    if (stride == row) {
        cx->be.h2d(cx->d_in, flow, bytes);
    } else {
        for (int y = 0; y < H; ++y) cx->be.h2d((char*)cx->d_in + row * y, (const char*)flow + stride * y, row);
    }
    return DOFS_OK;
}

// build_graph (graph.cpp:51-103) on a host field used as given: every edge of the 4- or 8-neighbourhood
// (neighborhood_8, graph.hpp:23) sorted stably by weight, i.e. by (weight, emission order) — the
// reference's multiset order. Writes min(E, capacity) edges; *n_edges = E; DOFS_ERR_CAPACITY if E > capacity.
template <class Backend>
int api_build_graph(Context<Backend>* cx, const float* flow, int H, int W, size_t stride, int nbr8, dofs_edge* edges,
                    int64_t capacity, int64_t* n_edges) {
    if (!flow || H <= 0 || W <= 0 || (!edges && capacity > 0)) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    if ((int64_t)H * W >= (1 << 26) || H > 32767 || W > 32767) return cx->fail(DOFS_ERR_INVALID_ARG, "frame too large");
    const Dims d = Pipeline<Backend>::dims_for(1, H, W, nbr8 ? 1 : 0);
    const int64_t E = graph_edges(H, W, nbr8 != 0), n4 = 4 * d.N;
    if (n_edges) *n_edges = E;
    if (E > capacity) return cx->fail(DOFS_ERR_CAPACITY, "edge capacity");
    cx->be.use_own();
    if (int rc = upload_flow(cx, flow, H, W, stride)) return rc;
    if (E == 0) return DOFS_OK;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_kout = al(8 * (size_t)n4), o_vin = o_kout + al(8 * (size_t)n4), o_vout = o_vin + al(4 * (size_t)n4),
                 o_edges = o_vout + al(4 * (size_t)n4), total = o_edges + al(sizeof(dofs_edge) * (size_t)E);
    char* g = (char*)cx->graph_buf(total);
    if (!g) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    Backend& be = cx->be;
    auto* kin = (unsigned long long*)g;
    auto* kout = (unsigned long long*)(g + o_kout);
    auto* vin = (unsigned*)(g + o_vin);
    auto* vout = (unsigned*)(g + o_vout);
    auto* de = (dofs_edge*)(g + o_edges);
    be.launch(1, n4, KGraphKeys{(const F2*)cx->d_in, d, kin, vin});
    be.sort_pairs(kin, kout, vin, vout, n4, 1, ceil_log2(n4));
    be.launch(1, E, KGraphEdges{kout, vout, d, de});
    be.d2h(edges, de, sizeof(dofs_edge) * (size_t)E);
    be.sync();
    return cx->check();
}

// segment_graph(flow, sorted_graph, ...) (graph.cpp:503-536) on a host field (used as given) and a host
// edge list taken in its order; results as dofs_segment (stats.n_merges = the unions performed).
template <class Backend>
int api_segment_graph(Context<Backend>* cx, const float* flow, int H, int W, size_t stride, const dofs_edge* edges,
                      int64_t E, const float persp[9], const float inv[9], const float inv_upper[27],
                      const dofs_params* params, dofs_result* out) {
    if (!flow || H <= 0 || W <= 0 || !out || E < 0 || (E > 0 && !edges))
        return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    if (E >= (int64_t)0x7FFFFFFF) return cx->fail(DOFS_ERR_INVALID_ARG, "too many edges");
    const int64_t N = (int64_t)H * W;
    for (int64_t i = 0; i < E; ++i)  // the reference would index out of its node vector
        if (edges[i].start < 0 || edges[i].start >= N || edges[i].end < 0 || edges[i].end >= N)
            return cx->fail(DOFS_ERR_INVALID_ARG, "edge endpoint outside the frame");
    cx->be.use_own();
    if (int rc = upload_flow(cx, flow, H, W, stride)) return rc;
    const size_t eb = (sizeof(dofs_edge) * (size_t)E + 255) & ~(size_t)255;
    char* g = (char*)cx->graph_buf(eb + 8 * (size_t)(E > 0 ? E : 1));
    if (!g) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    if (E > 0) cx->be.h2d(g, edges, sizeof(dofs_edge) * (size_t)E);
    const dofs_edge* de = (const dofs_edge*)g;
    int* acc = (int*)(g + eb);
    int rc = api_run(cx, (const F2*)cx->d_in, N, 1, H, W, persp, inv, inv_upper, params, nullptr, de, E, acc);
    if (rc) return rc;
    return fetch_grown(cx, out, [&]() {
        return api_run(cx, (const F2*)cx->d_in, N, 1, H, W, persp, inv, inv_upper, params, nullptr, de, E, acc);
    });
}

// Snapshot records beyond the per-frame capacity are not written (labels stay exact: KPaint works
// per slot). A batch that overflowed is reported, never copied silently: waits for the batch and
// returns DOFS_ERR_CAPACITY if any frame's count exceeded the capacity (C_OVF_ANY); the per-frame
// counts (C_OVF) say which. Grow it with dofs_set_snapshot_capacity and run the batch again.
template <class Backend>
int check_overflow(Context<Backend>* cx, int64_t batch) {
    const int slot = cx->slot_of(batch);
    cx->be.event_sync(cx->evDone[slot]);
    if (int e = cx->be.read_int(cx->pipe(slot).w.ctr + C_FLOWERR)) return fail_result(cx, e);
    const int ovf = cx->be.read_int(cx->pipe(slot).w.ctr + C_OVF_ANY);
    if (ovf) return cx->fail(DOFS_ERR_CAPACITY, "snapshot records overflowed the per-frame capacity");
    return cx->check();
}

// The first per_frame records of every frame are the first per_frame of its snapshots (slot order):
// KSnapshot writes the first snap_cap of them whatever the count, so with per_frame <= snap_cap every
// copied record exists — the counts say when a frame had more. A per_frame above the workspace's capacity
// is refused whatever the data (DOFS_ERR_CAPACITY), so ranks of one configuration all copy or all fail: a
// frame-parallel gather never sees one rank drop out.
// The copy waits for the batch (one host wait per collect; the pipelined caller collects batch k after
// submitting k + slots - 1, whose graph stage it then overlaps anyway) and reads the batch's replay flag:
// a batch whose results are invalid (C_FLOWERR: a replay give-up or a refused record) returns
// DOFS_ERR_INVALID_RESULT — after writing the block with every count DOFS_RECORDS_INVALID, so a collective
// gather that follows still moves equal blocks and every receiver sees which rank's frames are invalid. Any
// other failure (a HIP error: DOFS_ERR_DEVICE) leaves the block undefined, and the caller must not send it.
template <class Backend>
int api_records_copy(Context<Backend>* cx, int64_t batch, void* dst, int per_frame, void* stream) {
    if (!cx->live(batch) || !dst || per_frame < 0) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    const int slot = cx->slot_of(batch);
    const Ws& w = cx->pipe(slot).w;
    const int B = cx->meta[slot].B;
    if (per_frame > w.snap_cap)
        return cx->fail(DOFS_ERR_CAPACITY, "per_frame exceeds the snapshot capacity (dofs_set_snapshot_capacity)");
    cx->be.event_sync(cx->evDone[slot]);
    const int invalid = cx->be.read_int(w.ctr + C_FLOWERR);
    cx->be.set_stream(stream);
    cx->join(batch);
    cx->be.copy2d(dst, sizeof(int), w.ctr + C_SNAP, sizeof(int) * kCounters, sizeof(int), B);
    if (per_frame > 0)
        cx->be.copy2d((char*)dst + sizeof(int) * B, sizeof(dofs_box_record) * per_frame, w.recs,
                      sizeof(dofs_box_record) * w.snap_cap, sizeof(dofs_box_record) * per_frame, B);
    if (invalid) {
        static_assert(DOFS_RECORDS_INVALID == -1, "counts are filled with 0xFF bytes");
        cx->be.memset(dst, 0xFF, sizeof(int) * (size_t)B);
        if (int rc = cx->check()) return rc;
        return fail_result(cx, invalid);
    }
    return cx->check();
}

template <class Backend>
int api_lift_batch(Context<Backend>* cx, int n, const float* dirs, const int* boxes, const int* cls, const float mat[9],
                   const float inv[9], const float inv_upper[27], dofs_solution* out) {
    if (n <= 0 || !dirs || !boxes || !cls || !mat || !inv || !inv_upper || !out)
        return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    for (int i = 0; i < n; ++i)
        if (cls[i] < 0 || cls[i] > 2) return cx->fail(DOFS_ERR_INVALID_ARG, "cls must be 0..2");
    cx->be.use_own();
    const size_t b_dirs = sizeof(F2) * n, b_box = 16 * (size_t)n, b_cls = 4 * (size_t)n,
                 b_out = sizeof(dofs_solution) * n;
    const size_t o_box = (b_dirs + 255) & ~(size_t)255;
    const size_t o_cls = (o_box + b_box + 255) & ~(size_t)255;
    const size_t o_out = (o_cls + b_cls + 255) & ~(size_t)255;
    char* s = (char*)cx->scratch(o_out + b_out);
    if (!s) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    Backend& be = cx->be;
    be.h2d(s, dirs, b_dirs);
    be.h2d(s + o_box, boxes, b_box);
    be.h2d(s + o_cls, cls, b_cls);
    KLiftBatch k;
    k.dirs = (const F2*)s;
    k.boxes = (const int*)(s + o_box);
    k.cls = (const int*)(s + o_cls);
    k.out = (dofs_solution*)(s + o_out);
    memcpy(k.L.persp, mat, sizeof(k.L.persp));
    memcpy(k.L.inv, inv, sizeof(k.L.inv));
    memcpy(k.L.inv_upper, inv_upper, sizeof(k.L.inv_upper));
    dofs_params prm;
    default_params(&prm);
    for (int c = 0; c < 3; ++c) {
        k.L.obj_size[c][0] = prm.obj_size[c][0];
        k.L.obj_size[c][1] = prm.obj_size[c][1];
    }
    be.launch(1, n, k);
    be.d2h(out, s + o_out, b_out);
    be.sync();
    return cx->check();
}

// get_upper_face / get_upper_face_simple (lifting_3d.cpp:290-348 / :261-288) on the device, n boxes.
struct KUpperFaceBatch {
    const int* boxes;  // n x {xmin, ymin, xmax, ymax}
    const float* lf;   // n x 4 x (x, y)
    float* out;        // n x 4 x (x, y)
    int simple;
    DOFS_HD void operator()(int, int64_t i) const {
        P2 l[4], u[4];
        for (int k = 0; k < 4; ++k) l[k] = mk(lf[8 * i + 2 * k], lf[8 * i + 2 * k + 1]);
        if (simple)
            upper_face_simple(boxes + 4 * i, l, u);
        else
            upper_face(boxes + 4 * i, l, u);
        for (int k = 0; k < 4; ++k) {
            out[8 * i + 2 * k] = u[k].x;
            out[8 * i + 2 * k + 1] = u[k].y;
        }
    }
};

template <class Backend>
int api_upper_face_batch(Context<Backend>* cx, int n, const int* boxes, const float* lower, int simple, float* out) {
    if (n <= 0 || !boxes || !lower || !out) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    cx->be.use_own();
    const size_t b_box = 16 * (size_t)n, b_f = 32 * (size_t)n;
    const size_t o_lf = (b_box + 255) & ~(size_t)255, o_out = (o_lf + b_f + 255) & ~(size_t)255;
    char* s = (char*)cx->scratch(o_out + b_f);
    if (!s) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    Backend& be = cx->be;
    be.h2d(s, boxes, b_box);
    be.h2d(s + o_lf, lower, b_f);
    be.launch(1, n, KUpperFaceBatch{(const int*)s, (const float*)(s + o_lf), (float*)(s + o_out), simple});
    be.d2h(out, s + o_out, b_f);
    be.sync();
    return cx->check();
}

template <class Backend>
int api_set_snapshot_capacity(Context<Backend>* cx, int64_t cap) {
    if (cap < 1 || cap > (1 << 24)) return cx->fail(DOFS_ERR_INVALID_ARG, "capacity must be 1 .. 2^24");
    cx->snap_cap = cap;  // taken by each workspace at its next batch (re-layout)
    return DOFS_OK;
}

template <class Backend>
int api_intersect_batch(Context<Backend>* cx, int n, const float* pts, float* out) {
    if (n <= 0 || !pts || !out) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    cx->be.use_own();
    const size_t b_in = 32 * (size_t)n, o_out = (b_in + 255) & ~(size_t)255, b_out = 8 * (size_t)n;
    char* s = (char*)cx->scratch(o_out + b_out);
    if (!s) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    Backend& be = cx->be;
    be.h2d(s, pts, b_in);
    be.launch(1, n, KIntersectBatch{(const float*)s, (float*)(s + o_out)});
    be.d2h(out, s + o_out, b_out);
    be.sync();
    return cx->check();
}

// plot_best_segments_simple + draw_cube (draw.cpp:85-160) for the frames of batch `batch`:
// d_frames / d_out = B x H x W x 3 BGR (packed; d_out may equal d_frames). Ordered after the batch
// on the caller's stream; the edge map belongs to the batch's workspace, so overlays of one batch
// must be issued on one stream (or before the workspace is reused, batch + slots).
template <class Backend>
int api_overlay(Context<Backend>* cx, int64_t batch, const unsigned char* d_frames, unsigned char* d_out,
                bool check = true) {
    if (!cx->live(batch) || !d_frames || !d_out) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    const int slot = cx->slot_of(batch);
    const typename Context<Backend>::Meta& m = cx->meta[slot];
    const Ws& w = cx->pipe(slot).w;
    const int64_t N = (int64_t)m.H * m.W;
    const size_t lbytes = sizeof(int) * (size_t)m.B * (size_t)N;
    Backend& be = cx->be;
    if (lbytes > cx->d_lmap_bytes[slot]) {
        if (cx->d_lmap[slot]) {
            be.sync();  // an earlier overlay on this stream may still read it
            be.free(cx->d_lmap[slot]);
        }
        cx->d_lmap[slot] = (int*)be.alloc(lbytes);
        cx->d_lmap_bytes[slot] = cx->d_lmap[slot] ? lbytes : 0;
        if (!cx->d_lmap[slot]) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    }
    if (check)  // cubes are drawn from the snapshot records (the video loop reports counts instead)
        if (int rc = check_overflow(cx, batch)) return rc;
    OverlayWs o;
    o.frame = d_frames;
    o.out = d_out;
    o.lmap = cx->d_lmap[slot];
    o.labels = w.labels;
    o.snaps = w.snaps;
    o.ctr = w.ctr;
    o.snap_cap = w.snap_cap;
    o.H = m.H;
    o.W = m.W;
    o.N = N;
    o.min_score = m.prm.overlay_min_score;
    cx->join(batch);
    be.memset(o.lmap, 0xFF, lbytes);
    const int steps = (m.H > m.W ? m.H : m.W) + 1;
    be.launch(m.B, 12 * (int64_t)steps, KCubeLines{o, steps});
    be.launch(m.B, N, KOverlay{o});
    return cx->check();
}

// Host form for frame `frame` of the last batch (H2D of the frame, overlay, D2H).
template <class Backend>
int api_overlay_host(Context<Backend>* cx, int frame, const unsigned char* bgr, size_t stride, unsigned char* out) {
    if (!cx->have_batch() || !bgr || !out) return cx->fail(DOFS_ERR_INVALID_ARG, "bad args");
    const int64_t id = cx->nbatch - 1;
    const int slot = cx->slot_of(id);
    const typename Context<Backend>::Meta& m = cx->meta[slot];
    if (frame < 0 || frame >= m.B) return cx->fail(DOFS_ERR_INVALID_ARG, "no frame");
    const size_t row = (size_t)m.W * 3, bytes = row * (size_t)m.H;
    if (stride == 0) stride = row;
    if (stride < row) return cx->fail(DOFS_ERR_INVALID_ARG, "row stride too small");
    cx->be.event_sync(cx->evDone[slot]);
    if (cx->be.read_int(cx->pipe(slot).w.ctr + (int64_t)frame * kCounters + C_OVF))
        return cx->fail(DOFS_ERR_CAPACITY, "snapshot records overflowed the per-frame capacity");
    // a one-frame view of the batch: labels / snapshots / counters of `frame`
    unsigned char* d = (unsigned char*)cx->scratch(2 * bytes + 256);
    if (!d) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    Backend& be = cx->be;
    if (stride == row)
        be.h2d(d, bgr, bytes);
    else
        for (int y = 0; y < m.H; ++y) be.h2d(d + row * y, bgr + stride * y, row);
    const Ws& w = cx->pipe(slot).w;
    const int64_t N = (int64_t)m.H * m.W;
    if (sizeof(int) * (size_t)N > cx->d_lmap_bytes[slot]) {
        if (cx->d_lmap[slot]) be.free(cx->d_lmap[slot]);
        cx->d_lmap[slot] = (int*)be.alloc(sizeof(int) * (size_t)m.B * N);
        cx->d_lmap_bytes[slot] = cx->d_lmap[slot] ? sizeof(int) * (size_t)m.B * N : 0;
        if (!cx->d_lmap[slot]) return cx->fail(DOFS_ERR_OOM, "device allocation failed");
    }
    OverlayWs o;
    o.frame = d;
    o.out = d + bytes;
    o.lmap = cx->d_lmap[slot];
    o.labels = w.labels + (int64_t)frame * N;
    o.snaps = w.snaps + (int64_t)frame * w.snap_cap;
    o.ctr = w.ctr + (int64_t)frame * kCounters;
    o.snap_cap = w.snap_cap;
    o.H = m.H;
    o.W = m.W;
    o.N = N;
    o.min_score = m.prm.overlay_min_score;
    cx->join(id);
    be.memset(o.lmap, 0xFF, sizeof(int) * (size_t)N);
    const int steps = (m.H > m.W ? m.H : m.W) + 1;
    be.launch(1, 12 * (int64_t)steps, KCubeLines{o, steps});
    be.launch(1, N, KOverlay{o});
    be.d2h(out, d + bytes, bytes);
    be.sync();
    return cx->check();
}

}  // namespace dofs
