/*
 * dofs.h — C-ABI drop-in boundary for the dense-optical-flow clustering + 3D-lifting hot path.
 *
 * Reference interfaces replaced (DmitriyZhuravlev/DenseOpticalFlowSegmentation3D @ v1):
 *   dofs_segment / dofs_segment_batch_device
 *       ← Forest get_segmented_array(const cv::Mat& flow, const cv::Mat& bev,
 *                                     const cv::Matx33f& persp, const cv::Matx33f& inv,
 *                                     const std::vector<cv::Matx33f>& inv_upper, int neighbor=8)
 *         cpp/src/segment.cpp:34-72 (blur :52, build_graph :55, segment_graph :62)
 *         which in turn covers build_graph       cpp/inc/graph.hpp:22-23, cpp/src/graph.cpp:51-103
 *                              segment_graph     cpp/inc/graph.hpp:120-122, cpp/src/graph.cpp:503-536
 *                              Forest::new_merge cpp/src/graph.cpp:272-384
 *                              Forest::get_best_segments cpp/src/graph.cpp:391-429
 *         and the overlay's label semantics      cpp/src/draw.cpp:118-147 (score > 0.7, ascending slots)
 *   dofs_build_graph
 *       ← std::vector<Edge> build_graph(const cv::Mat& img, int width, int height, const DiffFunction& diff,
 *                                       bool neighborhood_8 = false)
 *         cpp/inc/graph.hpp:22-23, cpp/src/graph.cpp:51-103 (with diff = segment.cpp:20-32)
 *   dofs_segment_graph
 *       ← Forest segment_graph(const cv::Mat& flow, const std::vector<Edge>& sorted_graph, const cv::Mat& bev,
 *                              const cv::Matx33f& persp, const cv::Matx33f& inv,
 *                              const std::vector<cv::Matx33f>& inv_upper)
 *         cpp/inc/graph.hpp:120-122, cpp/src/graph.cpp:503-536
 *   dofs_lift / dofs_lift_batch
 *       ← Solution get_bottom_variants(const cv::Point2f& dir, const std::vector<cv::Point2i>& box,
 *                                      const cv::Matx33f& mat, const cv::Matx33f& inv,
 *                                      const cv::Matx33f& inv_upper, int cls)
 *         cpp/inc/lifting_3d.hpp:13-16, cpp/src/lifting_3d.cpp:350-439
 *   dofs_intersect ← cv::Point2f get_intersect(a1, a2, b1, b2)   cpp/inc/lifting_3d.hpp:26, lifting_3d.cpp:63-110
 *   dofs_calib     ← std::pair<Matx33f,Matx33f> get_mat()        cpp/inc/lifting_3d.hpp:17, lifting_3d.cpp:482-514
 *                    cv::Matx33f get_mat_upper(int cls)          cpp/inc/lifting_3d.hpp:18, lifting_3d.cpp:441-480
 *   dofs_upper_face        ← std::vector<cv::Point2f> get_upper_face(box_2d, lower_face)
 *                            cpp/inc/lifting_3d.hpp:21-22, lifting_3d.cpp:290-348
 *   dofs_upper_face_simple ← std::vector<cv::Point2f> get_upper_face_simple(box_2d, lower_face)
 *                            cpp/inc/lifting_3d.hpp:23-24, lifting_3d.cpp:261-288
 *   dofs_obj_size          ← std::pair<double,double> get_obj_size(int cls)
 *                            cpp/inc/lifting_3d.hpp:25, lifting_3d.cpp:524-528
 *   dofs_segment_scores    ← double Forest::get_segment_best_score(int node_id) const
 *                            cpp/inc/graph.hpp:96, graph.cpp:386-389 (segment_scores, :139, :326)
 *   dofs_final_roots       ← std::vector<cv::Point2i> Forest::get_bounding_box(int node_id) const after the run
 *                            cpp/inc/graph.hpp:103, graph.cpp:446-452 (bboxes cleared by merge, :208)
 *
 * Conventions
 *   - Plain C types only. Matrices are row-major float[9] (cv::Matx33f layout).
 *   - The flow field is H×W interleaved (u,v) float32 (cv::Mat CV_32FC2 layout).
 *   - Unlike the reference (which blurs the caller's Mat in place, segment.cpp:52), caller buffers
 *     are never mutated; the blurred field is returned on request (dofs_result.blurred).
 *   - Every entry point returns a dofs_status; no exceptions cross the ABI. An invalid `neighbor`
 *     falls back to the 4-neighbourhood exactly like segment.cpp:38-43 (not an error).
 *   - One dofs_ctx per host thread; each context owns one HIP stream unless a stream is passed.
 *     dofs_create may be called from several threads at once. Each context keeps the DOFS_* runtime knobs
 *      of the environment it was created in. dofs_last_error(NULL) reports the calling
 *     thread's last failed dofs_create; the string stays valid until that thread's next dofs_create.
 *   - The GPU library (libdofs_hip.so) requires a gfx950 device; there is no CPU fallback.
 */
#ifndef DOFS_H
#define DOFS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DOFS_ABI_VERSION 3

typedef enum dofs_status {
    DOFS_OK = 0,
    DOFS_ERR_INVALID_ARG = 1,
    DOFS_ERR_NO_DEVICE = 2,
    DOFS_ERR_DEVICE = 3,      /* a HIP runtime call failed; see dofs_last_error() */
    DOFS_ERR_CAPACITY = 4,    /* result capacity too small; n_snapshots holds the required count */
    DOFS_ERR_OOM = 5,
    DOFS_ERR_INVALID_RESULT = 6 /* the batch ran, but its results are invalid: its replay gave up a bounded
                                   wait, or a replay record held a root outside its frame (never seen; the
                                   device refused to use it) — dofs_last_error() says which. No HIP call
                                   failed. ABI version 3: version 2 returned DOFS_ERR_DEVICE here. */
} dofs_status;

/* Constants of the path; dofs_default_params() fills the reference values. */
typedef struct dofs_params {
    double blur_sigma;        /* 3.0   GaussianBlur(flow, flow, Size(0,0), 3.0)      segment.cpp:52 */
    int32_t neighbor;         /* 8     get_segmented_array(..., 8)                    segment.cpp:154 */
    int32_t min_size;         /* 500   Forest::new_merge default                      graph.hpp:93   */
    double score_threshold;   /* 0.3   Forest::new_merge default                      graph.hpp:93   */
    double overlay_min_score; /* 0.7   plot_best_segments_simple(..., 0.7)            segment.cpp:166 */
    double min_convexity[3];  /* 3/4, 1/2, 20/29 per class                            graph.cpp:328-339 */
    int32_t obj_size[3][2];   /* {258,84},{349,165},{370,180} BEV (l, w) per class     lifting_3d.cpp:257 */
} dofs_params;

/* Solution (graph.hpp:25-46). valid == 0 <=> Solution::rectangle is empty. */
typedef struct dofs_solution {
    int32_t cls;
    int32_t valid;
    float ps_bev[4][2];
    float lower_face[4][2];
    float upper_face[4][2];
    float rectangle[4][2];
    double w_error;
    double h_error;
    double orient;
} dofs_solution;

/* One non-empty slot of Forest::segment_history (graph.hpp:48-57, graph.cpp:348-356).
 * slot  = history index = union-find root pixel id at the winning merge.
 * event = index of the winning merge in Kruskal order (0 .. H*W-2).
 * Member pixels (SegmentData::seg) = leaf_order[seg_begin .. seg_begin + size). */
typedef struct dofs_snapshot {
    int32_t slot;
    int32_t event;
    int32_t size;
    int32_t seg_begin;
    int32_t bbox[4];          /* xmin, ymin, xmax, ymax (inclusive), graph.cpp:197-207 */
    double score;
    double move;
    dofs_solution sol;
} dofs_snapshot;

typedef struct dofs_stats {
    int64_t n_edges;          /* graph edges (build_graph size) */
    int64_t n_merges;         /* unions performed = H*W-1 */
    int64_t n_candidates;     /* merges passing the size / row / move filters (graph.cpp:280-300) */
    int64_t n_scored;         /* candidates with get_score != -1 */
    int64_t n_qualified;      /* candidates passing convexity and score > threshold */
    int64_t n_snapshots;      /* non-empty history slots */
} dofs_stats;

/* Caller-owned result buffers. Optional pointers may be NULL. */
typedef struct dofs_result {
    dofs_snapshot* snapshots; /* sorted by slot ascending */
    int32_t snapshot_capacity;
    int32_t n_snapshots;
    int32_t* labels;          /* [H*W] overlay label: max slot among snapshots with score > overlay_min_score, else -1 */
    int32_t* leaf_order;      /* [H*W] pixel ids in dendrogram leaf order */
    float* blurred;           /* [H*W*2] blurred flow */
    dofs_stats stats;
} dofs_result;

/* Edge (graph.hpp:13-17): same layout as the reference's struct {int start; int end; double weight;}
 * (16 bytes), so a std::vector<Edge>'s data() can be passed as is. */
typedef struct dofs_edge {
    int32_t start;
    int32_t end;
    double weight;
} dofs_edge;

/* Per-merge record (debug / parity of the order-dependent replay): state of the merged set
 * right after Forest::merge (graph.cpp:170-218) for merge k in Kruskal order. */
typedef struct dofs_event {
    int32_t start;            /* Edge::start (pixel id) */
    int32_t end;              /* Edge::end */
    double weight;            /* Edge::weight */
    int32_t root;             /* parent_b returned by merge */
    int32_t size;
    int32_t rank;
    int32_t bbox[4];
    float mean[2];            /* Node::flow_value of the root */
} dofs_event;

/* Fixed-size 3D-box record for the frame-parallel gather (one per snapshot, 96 bytes). score and move
 * keep the reference's double (SegmentData::score, graph.hpp:30-31; the move norm, graph.cpp:349-354);
 * the faces are Solution's float corners (lifting_3d.hpp, get_bottom_variants lifting_3d.cpp:412-438).
 * ABI version 2: version 1 narrowed score and move to float (88 bytes). */
typedef struct dofs_box_record {
    int32_t frame;
    int32_t slot;
    int32_t cls;
    int32_t size;
    double score;
    double move;
    float lower_face[4][2];
    float upper_face[4][2];
} dofs_box_record;

typedef struct dofs_ctx dofs_ctx;

int32_t dofs_abi_version(void);
void dofs_default_params(dofs_params* p);

/* get_mat() + get_mat_upper(0..2): persp = image→BEV, inv = BEV→image, inv_upper[cls] (host code). */
int32_t dofs_calib(float persp[9], float inv[9], float inv_upper[27]);

dofs_ctx* dofs_create(int32_t device);
void dofs_destroy(dofs_ctx* ctx);
const char* dofs_last_error(dofs_ctx* ctx);

/* get_segmented_array on host buffers (H2D, run, D2H). row_stride_bytes = 0 → packed (W*8). */
int32_t dofs_segment(dofs_ctx* ctx, const float* flow_uv, int32_t H, int32_t W, size_t row_stride_bytes,
                     const float persp[9], const float inv[9], const float inv_upper[27],
                     const dofs_params* params, dofs_result* out);

/* build_graph on a host field used AS GIVEN (get_segmented_array blurs first, segment.cpp:52-55): every
 * edge of the 4-neighbourhood (neighborhood_8 == 0, the reference's default) or 8-neighbourhood, emitted
 * per pixel in raster order as left, up, up-left, down-left (graph.cpp:62-93) with weight = diff
 * (segment.cpp:20-32), sorted stably by weight (the std::multiset order, graph.cpp:55-60). Writes the
 * sorted list to `edges` (host); *n_edges = E = build_graph's size; DOFS_ERR_CAPACITY (nothing written)
 * if capacity < E. Synchronous. */
int32_t dofs_build_graph(dofs_ctx* ctx, const float* flow_uv, int32_t H, int32_t W, size_t row_stride_bytes,
                         int32_t neighborhood_8, dofs_edge* edges, int64_t capacity, int64_t* n_edges);

/* segment_graph on a host field used AS GIVEN (the Forest's node flows, graph.cpp:129-148) and a host edge
 * list processed in its order (graph.cpp:519-531: find both ends, new_merge if they differ) — any list,
 * sorted or not, connected or not. Results as dofs_segment; stats.n_edges = n_edges, stats.n_merges =
 * the unions performed (H*W-1 when the edges connect the frame); dofs_events then returns those merges.
 * params: blur_sigma and neighbor are unused. An endpoint outside [0, H*W) is DOFS_ERR_INVALID_ARG. */
int32_t dofs_segment_graph(dofs_ctx* ctx, const float* flow_uv, int32_t H, int32_t W, size_t row_stride_bytes,
                           const dofs_edge* edges, int64_t n_edges, const float persp[9], const float inv[9],
                           const float inv_upper[27], const dofs_params* params, dofs_result* out);

/* Per-merge event stream of the last frame segmented by `ctx` (frame index within the last batch).
 * events must hold H*W-1 records (dofs_segment_graph: stats.n_merges). */
int32_t dofs_events(dofs_ctx* ctx, int32_t frame, dofs_event* events, int64_t capacity);

/* Frame-parallel batch on device-resident input: d_flow = B×H×W×2 float32 (device pointer),
 * stream = hipStream_t or NULL (the default stream, as in HIP). Asynchronous: the batch is ordered after the
 * work already queued on `stream`, and `stream` is ordered after the batch has consumed d_flow.
 * Batches use three device workspaces in turn and run as a two-stage pipeline (graph stage,
 * then replay + scoring stage), so consecutive calls overlap. Batch ids count calls from 0; the
 * results of the last three batches stay readable (dofs_batch_records_copy_id); dofs_batch_fetch,
 * dofs_events and dofs_batch_records_* read the last one. */
int32_t dofs_segment_batch_device(dofs_ctx* ctx, const float* d_flow, int32_t B, int32_t H, int32_t W,
                                  const float persp[9], const float inv[9], const float inv_upper[27],
                                  const dofs_params* params, void* stream);
int32_t dofs_batch_fetch(dofs_ctx* ctx, int32_t frame, dofs_result* out);
/* dofs_batch_fetch for batch id `batch` (one of the last dofs_batch_slots() issued). Waits for it. */
int32_t dofs_batch_fetch_id(dofs_ctx* ctx, int64_t batch, int32_t frame, dofs_result* out);

/* Forest::get_segment_best_score(id) for every id of frame `frame` of batch id `batch` (-1 = the last
 * batch; dofs_segment / dofs_segment_graph run as one-frame batches): scores[id] = segment_scores[id],
 * which new_merge writes for EVERY scored candidate (get_score != -1) of root id, before the convexity
 * and score-threshold tests (graph.cpp:326) — the root's last scored candidate's score, not its best
 * (that is the snapshot's score) — and 0.0, the vector's initial value (graph.cpp:139), where none.
 * capacity >= H*W doubles (host). Waits for the batch. */
int32_t dofs_segment_scores(dofs_ctx* ctx, int64_t batch, int32_t frame, double* scores, int64_t capacity);

/* Forest::get_bounding_box(id) AFTER the Kruskal loop (graph.cpp:446-452): merge clears the non-root
 * side's box (graph.cpp:208), so only the final union-find roots still have one — one per connected
 * component of the processed edges (one for get_segmented_array's grid, with the whole frame's box).
 * Writes min(n, capacity) records {root, xmin, ymin, xmax, ymax} (inclusive) ascending by root;
 * *n_roots = n. Every other id's box is the empty vector. (A snapshot's box at its winning merge is
 * dofs_snapshot.bbox.) batch = -1: the last batch. Waits for the batch. */
int32_t dofs_final_roots(dofs_ctx* ctx, int64_t batch, int32_t frame, int32_t* roots_bbox, int64_t capacity,
                         int64_t* n_roots);

/* Intra-frame sharding of the MST stage (BASELINE config 5: one large frame split
 * into row bands across GPUs). The global MST (graph.cpp:519-531 accepts exactly it) is contained in
 * the union of every row band's minimum spanning forest and the edges crossing band boundaries.
 *
 * dofs_band_msf_device: the minimum spanning forest of band rows [band_r0, band_r1) of an H x W
 * frame (edges with both endpoints in the band), from device flow rows [row0, row0 + rows) that
 * cover the band plus the blur halo (blur radius rows each side, clamped to the frame); writes
 * d_mask[(y - band_r0) * W + x] = bit k set for each forest edge emitted by pixel (x, y) (k: 0 left,
 * 1 up, 2 up-left, 3 down-left). Synchronous on `stream`.
 *
 * dofs_segment_masked_device: get_segmented_array on one device frame whose MST search is limited
 * to the edges allowed by d_allowed (H x W bytes, same bit layout) — the OR of the band forests and
 * every band-crossing edge gives results identical to dofs_segment_batch_device. Asynchronous, as a
 * one-frame batch (read with dofs_batch_fetch / dofs_events / dofs_batch_records_*). */
int32_t dofs_band_msf_device(dofs_ctx* ctx, const float* d_flow_rows, int32_t row0, int32_t rows, int32_t H,
                             int32_t W, int32_t band_r0, int32_t band_r1, const dofs_params* params,
                             uint8_t* d_mask, void* stream);
int32_t dofs_segment_masked_device(dofs_ctx* ctx, const float* d_flow, int32_t H, int32_t W,
                                   const uint8_t* d_allowed, const float persp[9], const float inv[9],
                                   const float inv_upper[27], const dofs_params* params, void* stream);
/* Device pointers to the last batch's fixed-capacity box records (B × capacity records, frame-major;
 * unused records have slot == -1) and per-frame counters (device int32, 64 per frame, the snapshot
 * count at index 4). Waits for the batch; valid until three more batches are issued. */
int32_t dofs_batch_records_device(dofs_ctx* ctx, void** d_records, void** d_counts, int32_t* capacity);

/* Copy the batch's box records to a caller device buffer on `stream`: int32 counts[B] (snapshots per
 * frame, the full count), then B × per_frame dofs_box_record (the first per_frame records of each
 * frame, slot order; entries past a frame's count have slot == -1). A frame with count > per_frame
 * was truncated by the caller's per_frame, which the counts show. Each frame keeps its first
 * dofs_snapshot_capacity() records (default 4096), so per_frame must not exceed that capacity:
 * DOFS_ERR_CAPACITY (nothing copied) otherwise, whatever the data — ranks of one configuration
 * therefore all copy or all fail. The labels are exact in every case.
 * Waits on the host for the batch (one wait per copy) and checks its results: a batch whose results are
 * invalid (DOFS_ERR_INVALID_RESULT: its replay gave up a bounded wait, or a replay record held an
 * out-of-range root; never seen) is copied with every count = DOFS_RECORDS_INVALID and the
 * call returns DOFS_ERR_INVALID_RESULT, so a gather that follows still moves equal blocks and every receiver
 * can tell which frames are invalid. Any other error (DOFS_ERR_DEVICE: a HIP call failed) leaves the block
 * undefined: do not send it. */
#define DOFS_RECORDS_INVALID (-1)
int32_t dofs_batch_records_copy(dofs_ctx* ctx, void* d_dst, int32_t per_frame, void* stream);
/* Same for batch id `batch` (one of the last three issued); ordered after that batch on `stream`. */
int32_t dofs_batch_records_copy_id(dofs_ctx* ctx, int64_t batch, void* d_dst, int32_t per_frame,
                                   void* stream);
/* Per-frame snapshot-record capacity of the batch API (taken by each workspace at its next batch). */
int32_t dofs_set_snapshot_capacity(dofs_ctx* ctx, int32_t per_frame);
int32_t dofs_snapshot_capacity(dofs_ctx* ctx);
/* Per-merge event records (dofs_events) for the batches issued afterwards: on = 1 keeps every merge's
 * replay record; 0 (the default) keeps only those the results read — path tops, merges of at least
 * min_size pixels — and dofs_events on such a batch fails with DOFS_ERR_INVALID_ARG. The reference's
 * segment() keeps no per-merge records either; its boxes, scores and labels are the same in both modes. */
int32_t dofs_keep_events(dofs_ctx* ctx, int32_t on);
/* Number of batches issued on ctx (the last batch id + 1). */
int64_t dofs_batch_count(dofs_ctx* ctx);
/* Frames (B) of the last batch issued on ctx (0 if none). */
int32_t dofs_batch_frames(dofs_ctx* ctx);
/* Number of batch workspaces (batches whose results stay readable; a caller that reads batch k's
 * results after submitting batch k + slots - 1 keeps every stage of the pipeline busy). */
int32_t dofs_batch_slots(dofs_ctx* ctx);
/* Device bytes of the last batch's workspace (one of dofs_batch_slots() such workspaces). */
int64_t dofs_workspace_bytes(dofs_ctx* ctx);

/* The last batch's per-frame counter blocks (B x 64 int32: candidates, snapshots, MST edges, ... and
 * at 16 + r the flag "Borůvka round r found a cross-component edge"), copied to host; waits for the
 * batch. Diagnostics and the bench's roofline model. capacity = ints available at out.
 * Also: [14] snapshot count of a frame whose records overflowed (else 0), [56] (frame 0) any overflow,
 * [57] merges on long heavy paths (the wave-per-path replay's work). */
int32_t dofs_batch_counters(dofs_ctx* ctx, int32_t* out, int64_t capacity);

/* Stage timing with device events (0 = off). Stages: 0 blur, 1 MST (Borůvka), 2 MST sort, 3 KRT,
 * 4 preorder, 5 replay, 6 lift + slots, 7 labels. dofs_profile_read returns the accumulated
 * milliseconds per stage and the number of profiled batches, then resets. */
int32_t dofs_profile(dofs_ctx* ctx, int32_t enable);
int32_t dofs_profile_read(dofs_ctx* ctx, double ms[8], int32_t* batches);

/* Kernel probe: device events around every launch of the per-element kernel named `kernel` (its
 * functor name in dofs_kernels.h, e.g. "KDncCompress"; NULL or "" = off), on the stream it runs on.
 * dofs_probe_read returns the accumulated milliseconds and the launch count, then resets. */
int32_t dofs_probe(dofs_ctx* ctx, const char* kernel);
int32_t dofs_probe_read(dofs_ctx* ctx, double* ms, int64_t* launches);
/* Several kernels at once: dofs_probe(ctx, "k_boruvka_min,k_krt_fused,...") then per name (in that order,
 * at most n) the accumulated milliseconds and launch count; returns the number of probed names
 * (negative status on error) and resets. */
int32_t dofs_probe_read_n(dofs_ctx* ctx, int32_t n, double* ms, int64_t* launches);

/* The last batch's Borůvka tile census (B x 40 int32): entry [f][m] = pixels of frame f's 32x8 tiles
 * that round m's minimum search found done (m >= 1; m = 0: never), so k_boruvka_min processed them in
 * pass 0 of rounds 1..m and pass 1 of rounds 1..m-1 (bench.py's roofline unit count). */
int32_t dofs_batch_tile_pixels(dofs_ctx* ctx, int32_t* out, int64_t capacity);

/* The last batch's Borůvka record census (B x 40 int32): entry [f][r] = (tile, component) records
 * that round r's k_boruvka_min4 wrote for frame f (0 where the frame took the pixel-candidate kernel
 * k_boruvka_min). With the tile census it gives the record kernels' roofline units (bench.py). */
int32_t dofs_batch_records(dofs_ctx* ctx, int32_t* out, int64_t capacity);

/* get_bottom_variants on the GPU (one candidate, or n candidates with per-candidate class). */
int32_t dofs_lift(dofs_ctx* ctx, const float dir[2], const int32_t box[4], const float mat[9],
                  const float inv[9], const float inv_upper[9], int32_t cls, dofs_solution* out);
int32_t dofs_lift_batch(dofs_ctx* ctx, int32_t n, const float* dirs, const int32_t* boxes,
                        const int32_t* cls, const float mat[9], const float inv[9],
                        const float inv_upper[27], dofs_solution* out);

/* get_upper_face (lifting_3d.cpp:290-348; the path's own upper face, :418) and get_upper_face_simple
 * (:261-288), host code: box = {xmin, ymin, xmax, ymax} (box_2d[0], box_2d[1]), lower_face / upper_face =
 * 4 corners x (x, y). Exact float / double semantics of the reference (cv::Point2f arithmetic, no FMA). */
void dofs_upper_face(const int32_t box[4], const float lower_face[8], float upper_face[8]);
void dofs_upper_face_simple(const int32_t box[4], const float lower_face[8], float upper_face[8]);
/* The same on the device for n boxes (simple = 0: get_upper_face, 1: get_upper_face_simple); boxes =
 * n x 4 int32, lower_faces / upper_faces = n x 8 floats. Synchronous. */
int32_t dofs_upper_face_batch(dofs_ctx* ctx, int32_t n, const int32_t* boxes, const float* lower_faces,
                              int32_t simple, float* upper_faces);
/* get_obj_size(cls) (lifting_3d.cpp:524-528): the class's BEV (length, width); cls outside 0..2 is
 * DOFS_ERR_INVALID_ARG (the reference indexes its 3-entry vector unchecked). */
int32_t dofs_obj_size(int32_t cls, double out[2]);

/* get_intersect (host code, exact float semantics of lifting_3d.cpp:63-89). */
void dofs_intersect(const float a1[2], const float a2[2], const float b1[2], const float b2[2], float out[2]);
/* The same on the device (the intersect() the lifting kernels use): pts = n x {a1, a2, b1, b2} x {x, y}
 * (8 floats per query), out = n x 2. Synchronous. */
int32_t dofs_intersect_batch(dofs_ctx* ctx, int32_t n, const float* pts, float* out);

/* ---- Upstream of the path: dense optical flow --------------------------------
 * dofs_farneback ← cv::calcOpticalFlowFarneback(prev, next, flow, pyr_scale, levels, winsize,
 *                   iterations, poly_n, poly_sigma, flags)   as called at cpp/src/segment.cpp:101,226
 *                   (0.5, 3, 15, 3, 5, 1.2, 0); OpenCV 4.x optflowgf.cpp algorithm, flags 0 only
 *                   (box-filter update, no initial flow). Frames are 8-bit single channel.
 * dofs_bgr_to_gray ← cv::cvtColor(im, gray, COLOR_BGR2GRAY)   cpp/src/segment.cpp:97-98,222-223 */
typedef struct dofs_flow_params {
    double pyr_scale;   /* 0.5 */
    int32_t levels;     /* 3   */
    int32_t winsize;    /* 15  */
    int32_t iterations; /* 3   */
    int32_t poly_n;     /* 5   */
    double poly_sigma;  /* 1.2 */
    int32_t flags;      /* 0 (OPTFLOW_USE_INITIAL_FLOW / OPTFLOW_FARNEBACK_GAUSSIAN unsupported) */
} dofs_flow_params;
void dofs_default_flow_params(dofs_flow_params* p);
/* Host frames (row stride in bytes, 0 = packed) -> host flow H x W x 2 float32. Synchronous. */
int32_t dofs_farneback(dofs_ctx* ctx, const uint8_t* prev, const uint8_t* next, int32_t H, int32_t W,
                       size_t row_stride_bytes, const dofs_flow_params* params, float* flow_uv);
/* Device batch: d_prev, d_next = B x H x W uint8 (packed), d_flow = B x H x W x 2 float32 — the layout
 * dofs_segment_batch_device consumes. Asynchronous on `stream` (NULL = the default stream). */
int32_t dofs_farneback_batch_device(dofs_ctx* ctx, const uint8_t* d_prev, const uint8_t* d_next, int32_t B,
                                    int32_t H, int32_t W, const dofs_flow_params* params, float* d_flow,
                                    void* stream);
/* BGR (3 bytes per pixel, packed rows) -> gray: host, and device (n_pixels, asynchronous on stream). */
void dofs_bgr_to_gray(const uint8_t* bgr, int32_t H, int32_t W, size_t row_stride_bytes, uint8_t* gray);
int32_t dofs_bgr_to_gray_device(const uint8_t* d_bgr, int64_t n_pixels, uint8_t* d_gray, void* stream);

/* ---- The video loop around the path --------------------------------------------
 * dofs_video_clip_device ← int main1() (cpp/src/segment.cpp:174-275): for each consecutive frame pair
 *   of a clip, cvtColor(BGR2GRAY) (:222-223), calcOpticalFlowFarneback(gray1, gray2, flow, 0.5, 3, 15,
 *   3, 5, 1.2, 0) (:226), get_segmented_array(flow, ...) (:251) and plot_best_segments_simple(frame,
 *   bev, forest, 0.7) (:258) — decode and display are the caller's. d_bgr = n_frames x H x W x 3 BGR
 *   uint8 (device). Pair p = (frame p, frame p + 1) writes, for frame p + 1:
 *     d_overlay + p*H*W*3     the overlay (H x W x 3; NULL = skip),
 *     d_counts[p]             its snapshot count (NULL = skip; a count above the snapshot capacity
 *                             means its records and cubes were truncated — the loop does not wait to check),
 *     d_records + p*per_frame its first per_frame 3D-box records (NULL = skip).
 *   Pairs run in chunks of `batch` through dofs_farneback_batch_device and the two-stage segment
 *   pipeline, the Farneback of one chunk overlapping the segmentation of the previous one. Asynchronous
 *   on `stream`; uses dofs_segment_batch_device batches (results of the last chunks stay readable). */
int32_t dofs_video_clip_device(dofs_ctx* ctx, const uint8_t* d_bgr, int32_t n_frames, int32_t H, int32_t W,
                               int32_t batch, const float persp[9], const float inv[9], const float inv_upper[27],
                               const dofs_params* params, const dofs_flow_params* flow_params, uint8_t* d_overlay,
                               int32_t* d_counts, dofs_box_record* d_records, int32_t per_frame, void* stream);

/* ---- Downstream of the path: the overlay -------------------------------------
 * dofs_overlay_batch_device ← cv::Mat plot_best_segments_simple(cv::Mat frame, cv::Mat bev, Forest&,
 *                              double min_score)   cpp/src/draw.cpp:101-160, with
 *                              draw_cube(im, lower_face, upper_face, Vec3b(255,0,0), 1)  draw.cpp:85-99
 *                              as called at cpp/src/segment.cpp:166 and :258 (min_score 0.7 =
 *                              dofs_params.overlay_min_score of the batch).
 *   Members of every snapshot with score > min_score painted in its class colour, its 3D box drawn
 *   (cv::line, thickness 1, 8-connected) into frame and painted copy, then
 *   addWeighted(frame, 0.6, seg, 0.4, 0). d_frames / d_out = B x H x W x 3 BGR uint8 (packed) of
 *   batch id `batch` (one of the last dofs_batch_slots issued); d_out may equal d_frames (the
 *   reference draws into `frame`). Asynchronous on `stream`, ordered after the batch; waits on the host
 *   for the batch and returns DOFS_ERR_CAPACITY if a frame's snapshots overflowed the capacity.
 * dofs_overlay: the same for frame `frame` of the last batch, host buffers (row stride in bytes,
 *   0 = packed W*3; out is packed). Synchronous. */
int32_t dofs_overlay_batch_device(dofs_ctx* ctx, int64_t batch, const uint8_t* d_frames, uint8_t* d_out,
                                  void* stream);
int32_t dofs_overlay(dofs_ctx* ctx, int32_t frame, const uint8_t* frame_bgr, size_t row_stride_bytes,
                     uint8_t* out_bgr);

/* Synthetic flow fields of the benchmark spec (DESIGN.md §Synthetic input), generated on device:
 * frame b uses seed0 + b. d_out = B×H×W×2 float32. */
int32_t dofs_synth_flow_device(float* d_out, int32_t B, int32_t H, int32_t W, uint64_t seed0, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DOFS_H */
