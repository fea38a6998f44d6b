// dofs_pipeline.h — orchestration of one batch of frames through the kernels of dofs_kernels.h.
// Templated on the execution backend: dofs_hip.hip instantiates it with the HIP backend (the
// product); tests/emu instantiates it with a sequential host backend to model the algorithm.
#pragma once

#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "dofs_kernels.h"

namespace dofs {

inline int ceil_log2(int64_t n) {
    int k = 0;
    while (((int64_t)1 << k) < n) ++k;
    return k;
}

// OpenCV 4.x getGaussianKernel (bit-exact variant: double arithmetic, float result) for float input:
// ksize = cvRound(sigma*4*2+1)|1 (segment.cpp:52 → cv::GaussianBlur(..., Size(0,0), 3.0)).
inline int gaussian_taps(double sigma, float* k) {
    int n = ((int)nearbyint(sigma * 4 * 2 + 1)) | 1;
    if (n > kMaxTaps - 1) n = (kMaxTaps - 1) | 1;
    std::vector<double> v((size_t)(n / 2 + 1));
    const double sx = sigma > 0 ? sigma : n * 0.15 + 0.35;
    const double scale2X = (-0.5 * 0.25) / (sx * sx);
    const int n2 = (n - 1) / 2;
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; ++i, x += 2) {
        v[i] = exp((double)(x * x) * scale2X);
        sum += v[i];
    }
    sum = sum * 2 + 1;
    const double mul1 = 1.0 / sum;
    double sum2 = 0;
    for (int i = 0; i < n2; ++i) {
        v[i] *= mul1;
        sum2 += v[i];
    }
    v[n2] = 1.0 - sum2 * 2;
    for (int i = 0; i <= n2; ++i) k[i] = k[n - 1 - i] = (float)v[i];
    return n;
}

template <class Backend>
struct Pipeline {
    Backend& be;
    Ws w;
    void* base = nullptr;
    size_t base_bytes = 0;
    Dims cap{};  // allocated shape
    int* pre = nullptr;
    int64_t snap_cap = 4096;
    // block-start labels of the KRT: the top-down global depths (DNC) or the per-frame sweep. The sweep's
    // time is one frame's sequence of blocks (≈ 40 ms at 1080p, 111 ms at 4K, whatever the batch); the
    // DNC's is proportional to the batch's merges (≈ 1.45 ms per million): DNC wins below ≈ 9 frames a
    // batch at any frame size (4K, one frame: KRT 111 → 12 ms). krt_mode: -1 auto (DNC for batches of at
    // most kDncFrames frames on a backend that selects it), 0 sweep, 1 DNC (DOFS_KRT_DNC=0 / 1)
    int krt_mode = -1;
    static constexpr int kDncFrames = 8;
    // Auto mode never forces a re-layout: a small (tail) batch on a workspace laid out for a large batch
    // without the DNC's arrays runs the sweep instead (a re-layout would free and re-allocate the
    // multi-GB workspace twice: down to the small shape, then up again for the next full batch).
    bool use_dnc(const Dims& d) const {
        if (krt_mode >= 0) return krt_mode == 1;
        return Backend::kDncAuto && d.B <= kDncFrames && (layout_words || !base || cap.B <= kDncFrames);
    }
    int skip_mask = 0;          // measurement only (DOFS_SKIPMASK): 1 short replay, 2 long replay, 4 lift
    void* ev_input = nullptr;   // run_a records it once the input flow has been read (the caller's release)
    bool keys_by_frame = true;  // key_out holds each frame's sorted weights (else: recomputed for events)
    unsigned vmask = ~0u;       // emission index bits of val_out
    int long_path = kLongPath;

    explicit Pipeline(Backend& b) : be(b) { memset(&w, 0, sizeof(w)); }
    ~Pipeline() {
        if (base) be.free(base);
    }

    static Dims dims_for(int B, int H, int W, int nbr8) {
        Dims d;
        d.H = H;
        d.W = W;
        d.N = (int64_t)H * W;
        d.M = d.N - 1;
        d.NL = d.N + d.M;
        d.P2 = 1;
        while (d.P2 < d.N) d.P2 <<= 1;
        d.B = B;
        d.nbr8 = nbr8;
        return d;
    }

    bool layout_packed = false;  // the layout treats key_out as dead (batch-wide sort): batches must sort packed
    bool layout_words = false;   // the layout holds the global-kernel KRT's arrays (P, CS, MX, own)
    // keep_graph (the context's keep_events): phase A's outputs stay readable after phase B (dofs_events
    // reads EU / EV; tools/krt_race.py the KRT's); else phase B's arrays reuse them (layout)
    bool keep_graph = false;
    bool layout_keep = false;
    bool fits(const Dims& d) const {
        const bool packed = Backend::mst_packed(std::max<int64_t>(d.M, 1), d.B, ceil_log2(4 * d.N));
        return base && cap.B >= d.B && cap.N == d.N && cap.W == d.W && (packed || !layout_packed) &&
               (layout_words || !(use_dnc(d) || Backend::kKrtLabelWords)) && (layout_keep || !keep_graph);
    }

    // Carve every buffer from one allocation (grow-only). Returns false on allocation failure.
    bool reserve(const Dims& d) {
        if (!fits(d)) {
            if (base) be.free(base);
            base = nullptr;
            size_t bytes = layout(d, nullptr);
            base = be.alloc(bytes);
            if (!base) return false;
            base_bytes = bytes;
            cap = d;
            layout(d, (char*)base);
            // the dataflow replay's queue slots (w.bw) accept a word only with this launch's tag, and
            // every launch's tag is new within the process; a fresh allocation may hold another
            // process's words, tags included, so it starts all ones (no tag) — once, synchronously
            be.memset(w.bw, 0xFF, sizeof(unsigned long long) * (size_t)d.B * (size_t)d.N);
            be.sync();
        }
        w.d = d;
        return true;
    }

    // One allocation per workspace. Phase A (graph) runs before phase B (replay + scoring) of the same
    // batch and the next batch on this workspace starts only after both, so the phase-B arrays live in
    // regions phase A is done with (first fit; a fresh block when nothing fits), and the arrays of the
    // global-kernel KRT (P, CS, MX, own) exist only where that KRT runs (DOFS_KRT_DNC, the emulator).
    // The arrays live across the stage boundary come first; then, in one run, those that die inside
    // phase A and (unless the context keeps the graph: keep_events) phase A's own outputs that only
    // phase A reads — adjacent dead regions merge, so the replay records (B·NL·32 bytes) fit there.
    // DESIGN.md §3 tables every array and its life.
    size_t layout(const Dims& d, char* p) {
        size_t off = 0;
        auto take = [&](size_t bytes) {
            off = (off + 255) & ~(size_t)255;
            char* r = p ? p + off : nullptr;
            off += bytes;
            return r;
        };
        const int64_t B = d.B, N = d.N, M = std::max<int64_t>(d.M, 1), NL = d.NL;
        const bool words = use_dnc(d) || Backend::kKrtLabelWords;
        layout_words = words;
        layout_keep = keep_graph;
        struct Region {  // [o, o + n) of the allocation, free for phase B
            size_t o, n;
        };
        std::vector<Region> dead;
        auto take_dead = [&](size_t bytes) {
            const size_t start = (off + 255) & ~(size_t)255;
            char* r = take(bytes);
            if (!dead.empty() && ((dead.back().o + dead.back().n + 255) & ~(size_t)255) == start)
                dead.back().n = off - dead.back().o;  // adjacent: one region
            else
                dead.push_back(Region{start, bytes});
            return r;
        };
        // a phase-B array: first fit in a dead region, below `limit` (the replay records: memory no kernel of
        // phase B reads once KPathInit, which writes their state words, starts)
        auto take_b = [&](size_t bytes, size_t limit = ~(size_t)0) {
            for (Region& g : dead) {
                const size_t a = (g.o + 255) & ~(size_t)255;
                if (a + bytes <= g.o + g.n && a + bytes <= limit) {
                    g.n = g.o + g.n - (a + bytes);
                    g.o = a + bytes;
                    return p ? p + a : nullptr;
                }
            }
            return take(bytes);
        };
        // phase A's outputs that phase B does not read: dead after phase A (keep_events keeps them for
        // dofs_events and the diagnosis tools)
        const bool zone = !keep_graph;
        auto take_a = [&](size_t bytes) { return zone ? take_dead(bytes) : take(bytes); };
        // the sorted weights: per frame (read by dofs_events) unless the whole batch is sorted at once
        // (run_a: the same predicate), when they are in global order and dead after the sort
        const bool packed = Backend::mst_packed(M, (int)B, ceil_log2(4 * N));
        layout_packed = packed;

        // ---- live across the stage boundary: read by phase B or by the result accessors
        w.blur = (F2*)take(sizeof(F2) * B * N);           // KBlur*; dofs_fetch's blurred field
        w.bw = (unsigned long long*)take(8 * B * N);      // Borůvka minima; the dataflow replay's queue
        w.SZ = (int*)take(4 * B * NL);                    // KRT node sizes (scoring)
        w.pre = (int*)take(4 * B * NL);
        w.ord = (int*)take(4 * B * NL);
        w.lscan = (int*)take(4 * B * NL);
        w.In = (StepIn*)take(sizeof(StepIn) * B * NL);    // (the KRT sweep's union-find records before)
        const Region in_region{(size_t)(off - sizeof(StepIn) * B * NL), sizeof(StepIn) * (size_t)B * (size_t)NL};
        w.leaf_order = (int*)take(4 * B * N);
        w.cur = (int*)take(4 * B * N);
        w.slast = w.cur;  // the replay's cursors are dead when KSlotInit fills it
        w.ptop = (int*)take(4 * B * N);
        w.list_short = (int*)take(4 * B * N);
        w.list_long = (int*)take(4 * B * N);
        if (!packed) w.key_out = (unsigned long long*)take(8 * B * M);
        if (!Backend::kReplayFlow) {  // the emulator's round-based replay's park lists
            w.comp = (int*)take(4 * B * N);
            w.off = (int*)take(4 * B * N);
        }
        w.own = words ? (int*)take(4 * B * M) : nullptr;
        w.P = words ? (unsigned long long*)take(8 * B * NL) : nullptr;
        w.CS = words ? (int*)take(4 * B * NL) : nullptr;
        w.MX = words ? (int*)take(4 * B * NL) : nullptr;
        // ---- dead inside phase A (one run of adjacent regions)
        w.tmp = (F2*)take_dead(sizeof(F2) * B * N);  // row blur, Borůvka records
        if (Backend::kReplayFlow) {
            w.comp = (int*)take_dead(4 * B * N);  // Borůvka labels
            w.off = (int*)take_dead(4 * B * N);   // MST offsets
        }
        w.bi = (unsigned*)take_dead(4 * B * N);
        w.mstbits = (int*)take_dead(4 * B * N);
        w.cnt = (int*)take_dead(4 * B * N);
        w.val_in = (unsigned*)take_dead(4 * B * M);
        if (packed) w.key_out = (unsigned long long*)take_dead(8 * B * M);
        w.val_out = (unsigned*)take_dead(4 * B * M);
        w.J = (unsigned long long*)take_dead(8 * B * NL);  // preorder jump words
        // ---- phase A's own outputs, read by phase A only (the same run, when dead after it): first those the
        // preorder and KPathInit do not read
        w.EU = (int*)take_a(4 * B * M);  // (dofs_events reads them: keep_events keeps them)
        w.EV = (int*)take_a(4 * B * M);
        const size_t rv_limit = off;
        w.uf = (int*)take_a(4 * B * N);
        w.lposr = w.uf;  // the MST's union-find is dead once the KRT starts
        w.key_in = (unsigned long long*)take_a(8 * B * M);
        w.hls = w.key_in;  // the KRT's children sizes for KPathInit: the sort input is dead by then
        w.lu = (int*)take_a(4 * B * M);
        w.lv = (int*)take_a(4 * B * M);
        w.hlB = (unsigned char*)take_a(B * M);
        w.lite = (unsigned char*)take_a(B * NL);
        // ---- phase B only: the replay records and path-top state words (state_at: KPathInit writes the
        // states, the replay the records; read by the scoring and the result accessors), then the scoring's
        // arrays (KFilter .. KLabel), largest first — those also in the replay inputs (StepIn), dead once the
        // replay ends (kept with the graph: tools/flow_dump.py reads them)
        w.Rv = (RepVal*)take_b(sizeof(RepVal) * B * NL, rv_limit);
        if (zone) dead.insert(dead.begin(), in_region);
        w.seg = (int*)take_b(4 * B * 2 * d.P2);
        w.sbest = (unsigned long long*)take_b(8 * B * N);
        w.cscore = (double*)take_b(8 * B * M);
        w.sevent = (int*)take_b(4 * B * N);
        w.sflag = (int*)take_b(4 * B * N);
        w.soff = (int*)take_b(4 * B * N);
        w.labels = (int*)take_b(4 * B * N);
        w.cand = (int*)take_b(4 * B * M);
        w.snaps = (dofs_snapshot*)take(sizeof(dofs_snapshot) * B * snap_cap);
        w.recs = (dofs_box_record*)take(sizeof(dofs_box_record) * B * snap_cap);
        w.ctr = (int*)take(4 * B * kCounters);
        w.tpx = (int*)take(4 * B * kRoundsMax);
        w.trec = (int*)take(4 * B * kRoundsMax);
        w.snap_cap = (int)snap_cap;
        return off + 256;
    }

    void set_params(const dofs_params& prm, const float persp[9], const float inv[9], const float inv_upper[27]) {
        w.bn = gaussian_taps(prm.blur_sigma, w.bk);
        memcpy(w.L.persp, persp, sizeof(w.L.persp));
        memcpy(w.L.inv, inv, sizeof(w.L.inv));
        memcpy(w.L.inv_upper, inv_upper, sizeof(w.L.inv_upper));
        for (int c = 0; c < 3; ++c) {
            w.L.obj_size[c][0] = prm.obj_size[c][0];
            w.L.obj_size[c][1] = prm.obj_size[c][1];
            w.min_convexity[c] = prm.min_convexity[c];
        }
        w.min_size = prm.min_size;
        w.score_threshold = prm.score_threshold;
        w.overlay_min_score = prm.overlay_min_score;
        w.long_path = long_path;
    }

    // K2 Borůvka MST under (weight, emission index) of the frames in w (edges limited to w.allow)
    void boruvka() {
        const Dims& d = w.d;
        const int B = d.B;
        const int64_t N = d.N;
        const bool first_done = be.boruvka_first(w);  // (HIP: init + round 0's minimum edges per LDS tile)
        if (!first_done) be.launch(B, N, KBoruvkaInit{w});
        const int R = std::min(ceil_log2(N) + 2, kRoundsMax - 1);
        for (int r = 0; r < R; ++r) {
            if (r == 0) {  // every pixel hooks along its minimum edge (a forest of pointers)
                if (!first_done) be.launch(B, N, KBoruvkaFirst{w});
                if (!be.pairs_in_relabel(w)) be.launch(B, N, KBoruvkaPairs{w});  // (HIP: k_boruvka_tile0)
            } else {
                be.boruvka_min(w, r, 0);  // KBoruvkaMinW (HIP: workgroup-aggregated per tile)
                be.boruvka_min(w, r, 1);  // KBoruvkaMinI
                be.boruvka_hook(w, r);    // KBoruvkaHook (also clears the roots' minima for round r + 1)
            }
            be.boruvka_relabel(w, r);  // KBoruvkaRelabelFind
        }
        be.boruvka_tiles(w);  // HIP: pixels per tile-done round (the roofline's processed-pixel count)
    }

    // Minimum spanning forest of the row band [r0, r1) of an H x W frame (edges with both ends in the
    // band), from device flow rows [row0, row0 + rows) that include the blur halo; writes the
    // forest's edges as per-pixel emitted-edge bits (mask[(y - r0) * W + x]). The caller reserved
    // dims_for(1, rows, W, nbr8).
    void run_band(const F2* flow_rows, int row0, int rows, int H, int r0, int r1, unsigned char* mask) {
        const int nbr8 = w.d.nbr8;
        w.single = 0;
        Ws wr = w;
        wr.d = dims_for(1, rows, w.d.W, nbr8);
        wr.flow = flow_rows;
        wr.flow_fstride = (int64_t)rows * w.d.W;
        be.launch(1, wr.d.N, KBlurRow{wr});
        w.d = dims_for(1, r1 - r0, w.d.W, nbr8);
        w.allow = nullptr;
        be.launch(1, w.d.N, KBlurColBand{w, H, row0, r0});
        be.memset(w.ctr, 0, sizeof(int) * kCounters);
        if (w.d.N > 1) {
            boruvka();
        } else {
            be.memset(w.mstbits, 0, sizeof(int));
        }
        be.launch(1, w.d.N, KMaskOut{w, mask});
    }

    // Phase A (graph): blur, MST, Kruskal order, KRT, preorder, replay inputs — on B frames of
    // device-resident flow (frame stride fstride F2 elements). Throughput-bound.
    void run_a(const F2* flow, int64_t fstride) {
        const Dims& d = w.d;
        const int B = d.B;
        const int64_t N = d.N, M = d.M;
        w.mreal = M;
        w.flow = flow;
        w.flow_fstride = fstride;
        {  // singleton flags ride in the two top value bits: only when the index and frame bits leave them
            const int vb = ceil_log2(4 * N);
            int fb = 0;
            if (be.mst_packed(std::max<int64_t>(M, 1), B, vb))
                while ((1 << fb) < B) ++fb;
            w.single = Backend::kSingleFlags && vb + fb <= 30 ? 1 : 0;
        }
        be.memset(w.ctr, 0, sizeof(int) * (size_t)B * kCounters);

        be.mark(0);
        // K1 blur (segment.cpp:52): KBlurRow + KBlurCol (HIP: LDS-tiled) — the only reader of the input
        be.blur(w);
        if (ev_input) be.record(ev_input, be.cur_stream());
        be.ord_mark(w);  // (HIP: stage B's merge marks in ord, off its chain)
        if (M <= 0) {  // single pixel: no edge, no merge
            be.launch(B, N, KLabelInit{w, true});
            be.launch(B, 1, KSingle{w});
            pre = nullptr;
            be.mark(8);
            return;
        }

        be.mark(1);
        boruvka();
        be.mark(2);
        be.launch(B, N, KMstCount{w});
        // each frame's MST spans its connected grid: N - 1 edges (not so under an edge mask: a forest)
        be.scan_excl_total(w.cnt, w.off, N, B, w.allow ? -1 : (int)(N - 1));
        // Kruskal order: val_out holds each frame's MST edges by (weight, index); when the backend sorts
        // the whole batch at once the frame id rides above the index bits and key_out is not per frame
        const int vb = ceil_log2(4 * N);
        const bool packed = be.mst_packed(M, B, vb);
        KMstEmit em{w, packed ? vb : 0};
        em.k32m = packed ? Backend::sort_k32() : 0;  // 32-bit sort keys (HIP batch sort, dofs_sortfix.h)
        em.k32b = Backend::sort_k32_bits();
        be.launch(B, N, em);
        be.sort_mst(w, M, B, vb, packed);
        keys_by_frame = !packed;
        vmask = vb >= 32 ? ~0u : (1u << vb) - 1u;
        krt(false);
    }

    // Phase A of segment_graph (graph.cpp:503-536) on a caller's edge list of one frame (device
    // `edges`, E of them, in Kruskal order): the flow is used as given; Borůvka under the list order
    // finds the accepted edges, which become the merges (a forest is completed by extra merges that
    // are never scored). acc / off: E ints of scratch. Returns the number of accepted edges (waits
    // for the device), or -1 if E is too large for 32-bit positions.
    int64_t run_a_edges(const F2* flow, const dofs_edge* edges, int64_t E, int* acc, int* off) {
        const Dims& d = w.d;
        const int64_t N = d.N, M = d.M;
        if (E >= (int64_t)0x7FFFFFFF) return -1;  // positions and the scan are 32-bit
        w.flow = flow;
        w.flow_fstride = N;
        w.single = 0;  // the caller's edge list: no minimum-edge slots
        be.memset(w.ctr, 0, sizeof(int) * kCounters);
        be.mark(0);
        be.launch(1, N, KCopyFlow{w});
        be.ord_mark(w);
        if (M <= 0) {
            be.launch(1, N, KLabelInit{w, true});
            be.launch(1, 1, KSingle{w});
            pre = nullptr;
            w.mreal = 0;
            be.mark(8);
            return 0;
        }
        be.mark(1);
        be.launch(1, N, KElInit{w});
        int64_t m = 0;
        if (E > 0) {
            be.memset(acc, 0, sizeof(int) * (size_t)E);
            const int R = std::min(ceil_log2(N) + 1, kRoundsMax - 1);
            for (int r = 0; r < R; ++r) {
                be.launch(1, E, KElMin{w, edges, r});
                be.launch(1, N, KElHook{w, edges, acc, r});
                be.launch(1, N, KElRelabel{w, r});
            }
            be.scan_excl(acc, off, E, 1);
            be.sync();
            m = (int64_t)be.read_int(off + E - 1) + be.read_int(acc + E - 1);
            be.launch(1, E, KElEmit{w, edges, acc, off});
        }
        w.mreal = m;
        keys_by_frame = true;
        if (m < M) {  // a forest: chain its roots after the caller's merges
            be.launch(1, N, KElRootFlag{w});
            be.scan_excl(w.cnt, w.off, N, 1);
            be.launch(1, N, KElRootList{w});
            be.launch(1, M - m, KElChain{w});
        }
        be.mark(2);
        krt(true);
        return m;
    }

    // K3 Kruskal reconstruction tree of the merges EU / EV (given: already there; else decoded from the
    // sorted MST edges), then the preorder unless it runs at the start of phase B
    void krt(bool given) {
        const Dims& d = w.d;
        const int B = d.B;
        const int64_t N = d.N, M = d.M, NL = d.NL;
        be.mark(3);
        w.jscatter = be.pre_jump(d) ? 1 : 0;
        const bool dnc = use_dnc(d);
        KEdgeInit ei{w, dnc};
        ei.given = given;
        ei.vmask = vmask;
        if (!given || dnc) be.launch(B, M, ei);
        const bool words = dnc || Backend::kKrtLabelWords;  // the global-kernel KRT reads them
        be.launch(B, words ? NL : N, KLabelInit{w, words});
        const int64_t deep = Backend::deep_block();  // levels with block size <= deep run per block
        if (dnc) {  // the top-down global depths (small batches; DOFS_KRT_DNC=1)
            for (int64_t S = (int64_t)1 << ceil_log2(M); S > deep; S >>= 1) {
                const int ep = dnc_epoch(M, S);
                be.launch(B, M, KDncUnion{w, S, ep});
                be.dnc_compress(w, S, ep);  // KDncCompress (HIP: workgroup-aggregated atomics)
                be.launch(B, M, KDncLRootRelabel{w, S, ep});
            }
        } else {  // labels at every deep block's start by one sweep over the blocks in rank order
            be.krt_seq(w);
        }
        be.dnc_deep(w);
        be.dnc_parent(w);  // KDncParent (HIP: k_dnc_deep's epilogue)
    }

    // K4 heavy-first preorder (pointer jumping) and the replay's per-position inputs. It runs at the start of
    // phase B: phase A bounds the step and phase B has slack (round 4, B = 112, same box: in phase A
    // 1,736-1,746 Mpix/s, in phase B 1,758-1,761)
    void preorder_pos() {
        const Dims& d = w.d;
        const int B = d.B;
        const int64_t N = d.N, NL = d.NL;
        be.mark(4);
        // merge nodes only (the leaves hang off them): two hops per launch at least triple every
        // node's jump distance (the second hop may read an ancestor word not yet advanced in this
        // launch), so 3^launches >= M reaches every root
        // (the HIP backend instead sweeps each frame's KRT blocks top-down once, k_pre_sweep, and
        // writes every node's position itself)
        const bool swept = be.pre_sweep(w);
        if (!swept) {
            int launches = 0;
            const int64_t chain = std::min<int64_t>(d.M, Backend::jump_chain_bound(d.M));
            for (int64_t span = 1; span < chain; span *= 3) ++launches;
            for (int t = 0; t < launches; ++t) be.launch(B, d.M, KJump{w.J, NL, 2, N});
        }
        pre = w.pre;
        if (!swept) be.launch(B, NL, KOrd{w});  // the sweep writes every position itself
        be.scan_excl_leaf(w.ord, w.lscan, NL, B, N);
        be.launch(B, NL, KLeafOrder{w, pre});
    }
    void path_init() { be.launch(w.d.B, w.d.M, KPathInit{w, w.pre}); }

    // Phase B (replay + scoring): the order-dependent replay is latency-bound (a few waves per
    // frame), so the HIP backend overlaps it with the next batch's phase A on a second stream.
    void run_b() {
        if (w.d.M <= 0) return;
        preorder_pos();
#ifdef DOFS_POISON_RV
        // check build: every replay record starts as zeros (in-range indices), so a read of a record the replay did not write
        // in this batch shows (results or an index fault) instead of reading an earlier batch's value
        be.memset(w.Rv, 0, sizeof(RepVal) * (size_t)w.d.B * (size_t)w.d.NL);
#endif
        path_init();
        be.mark(5);
        // K5 bottom-up replay of Forest::merge along heavy paths: one dataflow launch (HIP), else rounds
        if constexpr (Backend::kReplayFlow) {
            if (!(skip_mask & 3))
                be.replay_flow(w);
            else  // (measurement: the scoring then reads zeros, in-range indices, not whatever shares the memory)
                be.memset(w.Rv, 0, sizeof(RepVal) * (size_t)w.d.B * (size_t)w.d.NL);
        } else {
            replay_rounds();
        }
        score();
    }

    // K5 in rounds (the emulator): round r advances the short paths parked in round r - 1 and the long paths
    void replay_rounds() {
        const Dims& d = w.d;
        const int B = d.B;
        const int64_t N = d.N;
        const int RR = ceil_log2(N) + 2;
        // short paths: round r advances the paths parked in round r - 1 (lists ping-pong between two
        // pixel-sized buffers whose owners, the MST passes, are done)
        int* park[2] = {w.off, w.comp};
        const int* in = w.list_short;
        int inc = C_SHORT;
        for (int r = 0; r < RR; ++r) {
            if (!(skip_mask & 1)) {
                // round r appends to counter (r + 1) % 3 (zero: the batch's counter reset, or round
                // r - 1) and zeroes (r + 2) % 3 for round r + 1 (last read by round r - 1)
                const int oc = C_SQ + (r + 1) % 3;
                if (r == 0)  // the tiny short paths first, then the rest of list_short
                    be.launch_counted(B, N, KReplay{w, 0, w.list_short, C_TINY, park[0], oc, true}, C_TINY);
                be.launch_counted(B, N, KReplay{w, 2 * r, in, inc, park[r & 1], oc}, inc, C_SQ + (r + 2) % 3);
                in = park[r & 1];
                inc = oc;
            }
            if (!(skip_mask & 2)) be.replay_long(w, r);
        }
    }

    void score() {
        const Dims& d = w.d;
        const int B = d.B;
        const int64_t N = d.N, M = d.M;
        be.mark(6);
        // K6 new_merge filters, lifting, per-slot arg-max, snapshots
        be.launch(B, M, KFilter{w, pre});
        be.launch(B, N, KSlotInit{w});
        // the candidate list launches cover [0, C_CAND) of each frame (read on the device), not all M
        if (!(skip_mask & 4)) be.launch_counted(B, M, KLift{w, pre}, C_CAND);
        be.launch_counted(B, M, KSlotEvent{w, pre}, C_CAND);
        be.launch(B, N, KSlotFlag{w});
        be.scan_excl(w.sflag, w.soff, N, B);
        be.launch(B, 1, KSnapCount{w});
        be.launch(B, snap_cap, KRecClear{w});
        be.launch(B, N, KSnapshot{w, pre});

        be.mark(7);
        // K7 overlay labels
        be.launch(B, 2 * d.P2, KSegInit{w});
        be.launch(B, N, KPaint{w, pre});
        be.launch(B, N, KLabel{w});
        be.mark(8);
    }
};

}  // namespace dofs
