// dofs_cabi.inc.h — extern "C" entry points of include/dofs.h. Included once by a translation unit
// that has defined `using DofsBackend = <backend>;` (dofs_hip.hip: the HIP backend).
#pragma once

#include <memory>

#include "dofs_api.h"

struct dofs_ctx : dofs::Context<DofsBackend> {
    dofs_ctx(int device, const dofs::Knobs& kn) : dofs::Context<DofsBackend>(device, kn) {}
    std::shared_ptr<void> flow_engine;  // the optical-flow stage (HIP build; created on first use)
    std::shared_ptr<void> video;        // the clip pipeline's buffers and streams (HIP build)
};

extern "C" {

int32_t dofs_abi_version(void) { return DOFS_ABI_VERSION; }

void dofs_default_params(dofs_params* p) {
    if (p) dofs::default_params(p);
}

int32_t dofs_calib(float persp[9], float inv[9], float inv_upper[27]) {
    if (!persp || !inv || !inv_upper) return DOFS_ERR_INVALID_ARG;
    dofs::calib(persp, inv, inv_upper);
    return DOFS_OK;
}

void dofs_intersect(const float a1[2], const float a2[2], const float b1[2], const float b2[2], float out[2]) {
    dofs::P2 r = dofs::intersect(dofs::mk(a1[0], a1[1]), dofs::mk(a2[0], a2[1]), dofs::mk(b1[0], b1[1]),
                                 dofs::mk(b2[0], b2[1]));
    out[0] = r.x;
    out[1] = r.y;
}

void dofs_upper_face(const int32_t box[4], const float lower_face[8], float upper_face[8]) {
    dofs::P2 l[4], u[4];
    for (int k = 0; k < 4; ++k) l[k] = dofs::mk(lower_face[2 * k], lower_face[2 * k + 1]);
    dofs::upper_face(box, l, u);
    for (int k = 0; k < 4; ++k) {
        upper_face[2 * k] = u[k].x;
        upper_face[2 * k + 1] = u[k].y;
    }
}

void dofs_upper_face_simple(const int32_t box[4], const float lower_face[8], float upper_face[8]) {
    dofs::P2 l[4], u[4];
    for (int k = 0; k < 4; ++k) l[k] = dofs::mk(lower_face[2 * k], lower_face[2 * k + 1]);
    dofs::upper_face_simple(box, l, u);
    for (int k = 0; k < 4; ++k) {
        upper_face[2 * k] = u[k].x;
        upper_face[2 * k + 1] = u[k].y;
    }
}

int32_t dofs_obj_size(int32_t cls, double out[2]) {
    int sz[2];
    if (!out || !dofs::obj_size_of(cls, sz)) return DOFS_ERR_INVALID_ARG;
    out[0] = sz[0];
    out[1] = sz[1];
    return DOFS_OK;
}

// why this thread's last dofs_create returned NULL (dofs_last_error(NULL)); per thread, so concurrent
// dofs_create calls neither race on it nor invalidate each other's strings
static thread_local std::string g_create_err = "null context";

dofs_ctx* dofs_create(int32_t device) {
    dofs::Knobs kn;  // the context's own knobs (dofs_knobs.h)
    if (!dofs::knobs_load(&kn, &g_create_err)) return nullptr;  // an unknown DOFS_* knob or an invalid value
    if (!DofsBackend::device_ok(device)) {
        g_create_err = "no gfx950 device " + std::to_string(device);
        return nullptr;
    }
    dofs_ctx* c = new dofs_ctx(device, kn);
    if (!c->be.ok()) {
        g_create_err = c->be.error();
        delete c;
        return nullptr;
    }
    g_create_err = "null context";
    return c;
}

void dofs_destroy(dofs_ctx* ctx) { delete ctx; }

// Test entry (not in dofs.h): the knobs this context was created with (dofs_knobs.h) — {serial, flow_long,
// long_path, krt_dnc, pre_jump}; 0 for flow_long / long_path = the backend's default
int32_t dofs_debug_knobs(dofs_ctx* ctx, int32_t out[5]) {
    if (!ctx || !out) return DOFS_ERR_INVALID_ARG;
    const dofs::Knobs& k = ctx->be.kn;
    out[0] = k.serial;
    out[1] = k.flow_long;
    out[2] = k.long_path;
    out[3] = k.krt_dnc;
    out[4] = k.pre_jump;
    return DOFS_OK;
}

const char* dofs_last_error(dofs_ctx* ctx) { return ctx ? ctx->err.c_str() : g_create_err.c_str(); }

int32_t dofs_segment(dofs_ctx* ctx, const float* flow_uv, int32_t H, int32_t W, size_t row_stride_bytes,
                     const float persp[9], const float inv[9], const float inv_upper[27], const dofs_params* params,
                     dofs_result* out) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.use_own();
    return dofs::api_segment(ctx, flow_uv, H, W, row_stride_bytes, persp, inv, inv_upper, params, out);
}

int32_t dofs_build_graph(dofs_ctx* ctx, const float* flow_uv, int32_t H, int32_t W, size_t row_stride_bytes,
                         int32_t neighborhood_8, dofs_edge* edges, int64_t capacity, int64_t* n_edges) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_build_graph(ctx, flow_uv, H, W, row_stride_bytes, neighborhood_8, edges, capacity, n_edges);
}

int32_t dofs_segment_graph(dofs_ctx* ctx, const float* flow_uv, int32_t H, int32_t W, size_t row_stride_bytes,
                           const dofs_edge* edges, int64_t n_edges, const float persp[9], const float inv[9],
                           const float inv_upper[27], const dofs_params* params, dofs_result* out) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_segment_graph(ctx, flow_uv, H, W, row_stride_bytes, edges, n_edges, persp, inv, inv_upper,
                                   params, out);
}

int32_t dofs_events(dofs_ctx* ctx, int32_t frame, dofs_event* events, int64_t capacity) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_events(ctx, frame, events, capacity);
}

int32_t dofs_segment_batch_device(dofs_ctx* ctx, const float* d_flow, int32_t B, int32_t H, int32_t W,
                                  const float persp[9], const float inv[9], const float inv_upper[27],
                                  const dofs_params* params, void* stream) {
    if (!ctx || !d_flow) return DOFS_ERR_INVALID_ARG;
    ctx->be.set_stream(stream);
    return dofs::api_run(ctx, (const dofs::F2*)d_flow, (int64_t)H * W, B, H, W, persp, inv, inv_upper, params);
}

int32_t dofs_band_msf_device(dofs_ctx* ctx, const float* d_flow_rows, int32_t row0, int32_t rows, int32_t H,
                             int32_t W, int32_t band_r0, int32_t band_r1, const dofs_params* params,
                             uint8_t* d_mask, void* stream) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.set_stream(stream);
    return dofs::api_band_msf(ctx, (const dofs::F2*)d_flow_rows, row0, rows, H, W, band_r0, band_r1, params, d_mask);
}

int32_t dofs_segment_masked_device(dofs_ctx* ctx, const float* d_flow, int32_t H, int32_t W,
                                   const uint8_t* d_allowed, const float persp[9], const float inv[9],
                                   const float inv_upper[27], const dofs_params* params, void* stream) {
    if (!ctx || !d_flow || !d_allowed) return DOFS_ERR_INVALID_ARG;
    ctx->be.set_stream(stream);
    return dofs::api_run(ctx, (const dofs::F2*)d_flow, (int64_t)H * W, 1, H, W, persp, inv, inv_upper, params,
                         d_allowed);
}

int32_t dofs_batch_fetch(dofs_ctx* ctx, int32_t frame, dofs_result* out) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_fetch(ctx, frame, out);
}

int32_t dofs_batch_fetch_id(dofs_ctx* ctx, int64_t batch, int32_t frame, dofs_result* out) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.use_own();
    return dofs::api_fetch(ctx, frame, out, batch);
}

int32_t dofs_segment_scores(dofs_ctx* ctx, int64_t batch, int32_t frame, double* scores, int64_t capacity) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.use_own();
    return dofs::api_segment_scores(ctx, batch, frame, scores, capacity);
}

int32_t dofs_final_roots(dofs_ctx* ctx, int64_t batch, int32_t frame, int32_t* roots_bbox, int64_t capacity,
                         int64_t* n_roots) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.use_own();
    return dofs::api_final_roots(ctx, batch, frame, roots_bbox, capacity, n_roots);
}

int32_t dofs_batch_records_device(dofs_ctx* ctx, void** d_records, void** d_counts, int32_t* capacity) {
    if (!ctx || !ctx->have_batch()) return DOFS_ERR_INVALID_ARG;
    ctx->be.event_sync(ctx->evDone[ctx->last_slot()]);  // the pointers are read after the batch ended
    const dofs::Ws& w = ctx->pipe(ctx->last_slot()).w;
    if (d_records) *d_records = w.recs;
    if (d_counts) *d_counts = w.ctr;  // int32 counters, stride kCounters, count at C_SNAP
    if (capacity) *capacity = w.snap_cap;
    return ctx->check();
}

int32_t dofs_batch_records_copy(dofs_ctx* ctx, void* d_dst, int32_t per_frame, void* stream) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_records_copy(ctx, ctx->nbatch - 1, d_dst, per_frame, stream);
}

int32_t dofs_batch_records_copy_id(dofs_ctx* ctx, int64_t batch, void* d_dst, int32_t per_frame, void* stream) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_records_copy(ctx, batch, d_dst, per_frame, stream);
}

int32_t dofs_batch_counters(dofs_ctx* ctx, int32_t* out, int64_t capacity) {
    if (!ctx || !out || !ctx->have_batch()) return DOFS_ERR_INVALID_ARG;
    const int slot = ctx->last_slot();
    const int64_t n = (int64_t)ctx->meta[slot].B * dofs::kCounters;
    if (capacity < n) return DOFS_ERR_CAPACITY;
    ctx->be.use_own();
    ctx->join(ctx->nbatch - 1);
    ctx->be.d2h(out, ctx->pipe(slot).w.ctr, sizeof(int32_t) * (size_t)n);
    ctx->be.sync();
    return ctx->check();
}

int32_t dofs_set_snapshot_capacity(dofs_ctx* ctx, int32_t per_frame) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_set_snapshot_capacity(ctx, per_frame);
}

int32_t dofs_snapshot_capacity(dofs_ctx* ctx) { return ctx ? (int32_t)ctx->snap_cap : -1; }

int32_t dofs_keep_events(dofs_ctx* ctx, int32_t on) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->keep_events = on != 0;
    return DOFS_OK;
}

int64_t dofs_batch_count(dofs_ctx* ctx) { return ctx ? ctx->nbatch : -1; }

int32_t dofs_batch_frames(dofs_ctx* ctx) {
    if (!ctx || !ctx->have_batch()) return 0;
    return ctx->meta[ctx->last_slot()].B;
}

int32_t dofs_batch_slots(dofs_ctx* ctx) { return ctx ? ctx->nslots : -1; }

int64_t dofs_workspace_bytes(dofs_ctx* ctx) {
    if (!ctx || !ctx->have_batch()) return 0;
    return (int64_t)ctx->pipe(ctx->last_slot()).base_bytes;
}

int32_t dofs_profile(dofs_ctx* ctx, int32_t enable) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.profile(enable != 0);
    return DOFS_OK;
}

int32_t dofs_profile_read(dofs_ctx* ctx, double ms[8], int32_t* batches) {
    if (!ctx || !ms) return DOFS_ERR_INVALID_ARG;
    ctx->drain();
    int n = ctx->be.profile_read(ms);
    if (batches) *batches = n;
    return ctx->check();
}

int32_t dofs_probe(dofs_ctx* ctx, const char* kernel) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.probe(kernel);
    return DOFS_OK;
}

int32_t dofs_probe_read(dofs_ctx* ctx, double* ms, int64_t* launches) {
    if (!ctx || !ms) return DOFS_ERR_INVALID_ARG;
    ctx->drain();
    const int64_t n = ctx->be.probe_read(ms);
    if (launches) *launches = n;
    return ctx->check();
}

int32_t dofs_probe_read_n(dofs_ctx* ctx, int32_t n, double* ms, int64_t* launches) {
    if (!ctx || !ms || n < 0) return -DOFS_ERR_INVALID_ARG;
    ctx->drain();
    const int k = ctx->be.probe_read_n(n, ms, launches);
    return ctx->check() == DOFS_OK ? k : -DOFS_ERR_DEVICE;
}

int32_t dofs_batch_tile_pixels(dofs_ctx* ctx, int32_t* out, int64_t capacity) {
    if (!ctx || !out || !ctx->have_batch()) return DOFS_ERR_INVALID_ARG;
    const int slot = ctx->last_slot();
    const int64_t n = (int64_t)ctx->meta[slot].B * dofs::kRoundsMax;
    if (capacity < n) return DOFS_ERR_CAPACITY;
    ctx->be.use_own();
    ctx->join(ctx->nbatch - 1);
    ctx->be.d2h(out, ctx->pipe(slot).w.tpx, sizeof(int32_t) * (size_t)n);
    ctx->be.sync();
    return ctx->check();
}

int32_t dofs_batch_records(dofs_ctx* ctx, int32_t* out, int64_t capacity) {
    if (!ctx || !out || !ctx->have_batch()) return DOFS_ERR_INVALID_ARG;
    const int slot = ctx->last_slot();
    const int64_t n = (int64_t)ctx->meta[slot].B * dofs::kRoundsMax;
    if (capacity < n) return DOFS_ERR_CAPACITY;
    ctx->be.use_own();
    ctx->join(ctx->nbatch - 1);
    ctx->be.d2h(out, ctx->pipe(slot).w.trec, sizeof(int32_t) * (size_t)n);
    ctx->be.sync();
    return ctx->check();
}

int32_t dofs_lift(dofs_ctx* ctx, const float dir[2], const int32_t box[4], const float mat[9], const float inv[9],
                  const float inv_upper[9], int32_t cls, dofs_solution* out) {
    if (!ctx || cls < 0 || cls > 2 || !inv_upper) return DOFS_ERR_INVALID_ARG;
    float up[27] = {0};
    for (int i = 0; i < 9; ++i) up[9 * cls + i] = inv_upper[i];
    return dofs::api_lift_batch(ctx, 1, dir, box, &cls, mat, inv, up, out);
}

int32_t dofs_lift_batch(dofs_ctx* ctx, int32_t n, const float* dirs, const int32_t* boxes, const int32_t* cls,
                        const float mat[9], const float inv[9], const float inv_upper[27], dofs_solution* out) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_lift_batch(ctx, n, dirs, boxes, cls, mat, inv, inv_upper, out);
}

int32_t dofs_upper_face_batch(dofs_ctx* ctx, int32_t n, const int32_t* boxes, const float* lower_faces,
                              int32_t simple, float* upper_faces) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_upper_face_batch(ctx, n, boxes, lower_faces, simple, upper_faces);
}

int32_t dofs_intersect_batch(dofs_ctx* ctx, int32_t n, const float* pts, float* out) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    return dofs::api_intersect_batch(ctx, n, pts, out);
}

int32_t dofs_synth_flow_device(float* d_out, int32_t B, int32_t H, int32_t W, uint64_t seed0, void* stream) {
    if (!d_out || B <= 0 || H <= 0 || W <= 0) return DOFS_ERR_INVALID_ARG;
    dofs::KSynth k{(dofs::F2*)d_out, H, W, (unsigned long long)seed0};
    return DofsBackend::launch_static(stream, B, (int64_t)H * W, k);
}

int32_t dofs_overlay_batch_device(dofs_ctx* ctx, int64_t batch, const uint8_t* d_frames, uint8_t* d_out,
                                  void* stream) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.set_stream(stream);
    return dofs::api_overlay(ctx, batch, d_frames, d_out);
}

int32_t dofs_overlay(dofs_ctx* ctx, int32_t frame, const uint8_t* frame_bgr, size_t row_stride_bytes,
                     uint8_t* out_bgr) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    ctx->be.use_own();
    return dofs::api_overlay_host(ctx, frame, frame_bgr, row_stride_bytes, out_bgr);
}

}  // extern "C"
