// dofs_kernels.h — per-element bodies of every kernel of the pipeline.
//
// Each functor's operator()(f, i) handles element i of frame f. The HIP translation unit wraps them
// in grid-stride __global__ launchers; the test-only host emulator loops over (f, i).
//
// Stages (reference → kernel):
//   segment.cpp:52 GaussianBlur            KBlurRow, KBlurCol
//   segment.cpp:20-32 diff + graph.cpp:51-103 build_graph (implicit: weights computed on the fly)
//                                          KBoruvka* : minimum spanning tree under the strict order
//                                          (weight, emission index) = Kruskal's order (multiset
//                                          upper-bound insertion == stable sort)
//   graph.cpp:519-531 Kruskal loop         KMst* + radix sort of the N-1 MST edges
//                                          KDnc* : Kruskal reconstruction tree (KRT) by top-down
//                                          divide and conquer over rank blocks
//   graph.cpp:170-218 Forest::merge        KTree*, KJump, KOrd, KPathInit, KReplay: bottom-up replay
//                                          of union-by-rank roots, ranks, float running means, bboxes
//                                          along heavy paths of the KRT
//   graph.cpp:272-356 Forest::new_merge    KFilter, KLift (get_score x3 classes), KSlot*, KSnapshot
//   draw.cpp:118-147 overlay labels        KSeg*, KLabel
#pragma once

#include "dofs_common.h"
#include "dofs_lift.h"

namespace dofs {

// Inputs of the merge at preorder position q (node x, heavy child h, light child l), precomputed in
// parallel; the replay then only carries the order-dependent state (mean, rank, root). Stored packed, 16 B
// per position (StepIn, written by KPathInit at random positions and read by the replay in position order);
// the replay decodes it (step_v) into
//   fs = (float)size(h)      r = 1 / (double)size(x)
//   wb = float(mean(l) * (float)size(l))  — static when l is a pixel (la = its x | y << 16,
//        lb = its id: rank 0, root = itself); when l is a merge node (kStepDyn) its mean, rank,
//        root and bbox are produced by the replay itself: la holds size(l) and lb its preorder
//        position, and they are read once l's path has completed.
// Round 5: the record was these 32 bytes as stored; everything but the pixel's flow and id derives from the
// two children's sizes and the position (heavy-first preorder: the light child follows the heavy subtree,
// at q + 2 size(h)), so 16 bytes hold it — half the random stores of KPathInit and the replay's reads.
struct StepIn {
    unsigned hs;     // size(h) (bits 0-25, H*W < 2^26) | the kStep* flags << 26
    int lt;          // a merge light child (kStepDyn): size(l); a pixel: its id
    float wbx, wby;  // a pixel light child's blurred flow (· size 1); 0 for a merge
};
static_assert(sizeof(StepIn) == 16, "StepIn is one 16-byte record");
struct StepV {  // a decoded StepIn (step_v)
    float fs;
    float wbx, wby;
    int meta;
    double r;
    int la;
    int lb;
};
constexpr int kStepB = 1;    // light child is the end side (B) of the merge
constexpr int kStepTop = 2;  // x is the top of its heavy path
constexpr int kStepDyn = 4;  // light child is a merge node (value produced by the replay)
constexpr int kStepKeep = 16;  // (8: kLongOk, dofs_hip.hip) size(x) >= min_size: scoring may read x's replay record (Ws::rv_lean)
constexpr int kStepShift = 26;  // StepIn::hs: the flags above size(h)
constexpr unsigned kStepSizeMask = (1u << kStepShift) - 1u;
DOFS_HD inline int step_meta(const StepIn& in) { return (int)(in.hs >> kStepShift); }
// a merge light child's preorder position (kStepDyn only)
DOFS_HD inline int step_lq(const StepIn& in, int64_t q) { return (int)(q + 2 * (int64_t)(in.hs & kStepSizeMask)); }
// decode the record at position q of a frame W pixels wide: the same values the 32-byte record held
DOFS_HD inline StepV step_v(const StepIn& in, int64_t q, int W) {
    StepV v;
    const int sh = (int)(in.hs & kStepSizeMask);
    v.meta = step_meta(in);
    v.fs = (float)sh;
    if (v.meta & kStepDyn) {
        const int sl = in.lt;
        v.r = 1. / (double)(sh + sl);  // size(x)
        v.wbx = v.wby = 0.f;
        v.la = sl;
        v.lb = (int)(q + 2 * (int64_t)sh);
    } else {
        const int lt = in.lt;
        v.r = 1. / (double)(sh + 1);
        v.wbx = in.wbx;
        v.wby = in.wby;
        v.la = (lt % W) | ((lt / W) << 16);
        v.lb = lt;
    }
    return v;
}

// Workspace: device pointers (frame-major; per-frame strides by size class) + constants.
struct Ws {
    Dims d;
    // inputs
    const F2* flow;
    int64_t flow_fstride;          // F2 elements between frames of the input
    const unsigned char* allow;    // optional: bit k of allow[p] = edge (p, k) may be in the MST
    // blur
    F2* tmp;
    F2* blur;
    float bk[kMaxTaps];
    int bn;
    // Borůvka (per pixel, stride N)
    int* comp;
    unsigned long long* bw;
    unsigned* bi;
    int* uf;
    int* mstbits;  // per pixel: byte k != 0 <=> its emitted edge k is an MST edge (plain byte stores; the
                   // HIP record hook sets its byte by an atomic OR on the word)
    int* cnt;
    int* off;
    // MST edges (stride M)
    unsigned long long* key_in;
    unsigned* val_in;
    unsigned long long* key_out;
    unsigned* val_out;
    int* EU;
    int* EV;
    int* lu;
    int* lv;
    int* own;
    unsigned char* hlB;  // merge i's light child is its end side B
    // label / node space (stride NL)
    unsigned long long* P;  // KRT label words (link | size << 32)
    int* CS;
    int* MX;
    int* SZ;
    unsigned long long* J;  // pointer jumping: (ancestor, offset sum) packed (jump_pack)
    unsigned char* lite;    // node is a light child (or the root): the top of a heavy path
    int* pre;               // heavy-first preorder position
    int* ord;
    int* lscan;
    StepIn* In;
    RepVal* Rv;  // replay outputs by preorder position
    // per pixel (stride N)
    int* leaf_order;
    int* lposr;  // per frame (stride N): preorder position of the leaf of each leaf rank (aliases uf,
                 // dead after the MST); KPathInit's path bottoms
    int* cur;
    int* slast;  // per slot: the last scored candidate merge (Forest::segment_scores, graph.cpp:326); aliases
                 // cur, the replay's path cursors, dead once the replay ended
    int* ptop;
    int* list_short;
    int* list_long;
    int* sevent;
    unsigned long long* sbest;
    int* sflag;
    int* soff;
    int* labels;
    // per edge (stride M)
    int* cand;
    double* cscore;
    // per merge (stride M): size of its heavy child | size of its light child << 32, written by the
    // KRT's parent pass for KPathInit (coalesced instead of gathered); aliases cscore, which KLift
    // fills only after the replay inputs are built
    unsigned long long* hls;
    // segment tree (stride 2*P2)
    int* seg;
    // outputs (stride snap_cap)
    dofs_snapshot* snaps;
    dofs_box_record* recs;
    int snap_cap;
    // counters (stride kCounters)
    int* ctr;
    // pixels of the Borůvka tiles by the round that found them done (stride kRoundsMax; 0: never)
    int* tpx;
    // records written by round r's k_boruvka_min4 (stride kRoundsMax; HIP record path only)
    int* trec;
    // parameters
    LiftMats L;
    int min_size;
    double score_threshold;
    double overlay_min_score;
    int long_path;  // heavy paths at least this long run on the wave-cooperative replay
    int jscatter;   // HIP: the LDS KRT's epilogue writes its block's outside children's jump words and
                    // path-top flags (the chip-wide jumping preorder of small batches), else k_pre_sweep
    int deep_wave;  // HIP: the LDS KRT's depths below 32 merges by one register pass per 16-merge window
    // HIP dataflow replay: a short path stores a merge's replay record only where something reads it — its
    // path top (the parent's light child), a parked state, a merge of >= min_size pixels (kStepKeep: the
    // scoring's candidates) — not the records of the other merges (dofs_events needs them all)
    int rv_lean;
    int single;     // HIP: EU / EV carry bit kSingleBit — the endpoint is a single pixel at this merge (the
                    // merge is its minimum incident edge, so its first in Kruskal order): the KRT sweep
                    // takes its label without a find
    int64_t mreal;  // merges of the caller's graph (scored); later ones only complete a forest (< M)
    double min_convexity[3];

    DOFS_HD int* C(int f) const { return ctr + (int64_t)f * kCounters; }
};

// The replay state word of the path top at preorder position pos (graph.cpp:184-190's dependency, made
// explicit): the first pad word of the top's replay record. One 32-byte sector holds both, so a waiting
// path's state poll and record fetch read one sector and the completer's publish and state exchange write
// one (a separate state array cost a second random sector per light child: round 5). Only path tops have
// a state; the other positions' pads are free (their plain 32-byte stores write zeros there).
DOFS_HD inline int* state_at(const Ws& w, int64_t pos) { return &w.Rv[pos].pad0; }

// The batch's sticky result error, C_FLOWERR of frame 0 (bits; every result accessor reports it as
// DOFS_ERR_INVALID_RESULT): kErrGiveUp, the dataflow replay gave up a bounded wait; kErrRecord, a replay
// record's union-find root used as an index (the scoring's slot arrays) lay outside its frame. A lane that
// finds such a root skips the access, so a wrong record can cost the batch its results but never an
// out-of-range atomic or gather.
constexpr int kErrGiveUp = 1;
constexpr int kErrRecord = 2;
constexpr int kErrMst = 4;  // a frame's MST without N - 1 edges where its offsets assumed them (KMstEmit)
DOFS_HD inline bool root_ok(const Ws& w, int root) {
    if ((unsigned)root < (unsigned)w.d.N) return true;
    dofs_aor(w.C(0) + C_FLOWERR, kErrRecord);
    return false;
}

// ---------------------------------------------------------------------------------------------
// Implicit 8-neighbour grid graph (graph.cpp:62-93): pixel p emits edge k∈{0:left, 1:up,
// 2:up-left, 3:down-left}; emission index idx = 4p + k orders edges exactly like the reference's
// sequential emission. start = p, end = neighbour.
// ---------------------------------------------------------------------------------------------
DOFS_HD inline bool edge_exists(const Dims& d, int x, int y, int k) {
    switch (k) {
        case 0: return x > 0;
        case 1: return y > 0;
        case 2: return d.nbr8 && x > 0 && y > 0;
        default: return d.nbr8 && x > 0 && y < d.H - 1;
    }
}
DOFS_HD inline int64_t edge_end(const Dims& d, int64_t p, int k) {
    switch (k) {
        case 0: return p - 1;
        case 1: return p - d.W;
        case 2: return p - d.W - 1;
        default: return p + d.W - 1;
    }
}
// dx * dx + dy * dy for dx, dy converted from floats, bit for bit with one rounding less to issue: a
// float's square is exact in double (24 + 24 significant bits <= 53, no overflow or underflow for any
// float), so fma(dx, dx, dy * dy) rounds the same exact sum the separate multiply and add round once
DOFS_HD inline double sq_len(double dx, double dy) { return fma(dx, dx, dy * dy); }
// diff (segment.cpp:20-32): float subtraction, double squares/sum/sqrt (correctly rounded).
DOFS_HD inline double edge_weight(const F2* b, int64_t p, int64_t q) {
    double dx = b[p].x - b[q].x;
    double dy = b[p].y - b[q].y;
    return sqrt(sq_len(dx, dy));
}
DOFS_HD inline unsigned long long dbits(double w) {
    union {
        double d;
        unsigned long long u;
    } c;
    c.d = w;
    return c.u;
}
// The 32-bit Kruskal sort key of a weight key (HIP batch sort, dofs_sortfix.h): m mantissa bits below a
// (32 - m)-bit exponent offset inside the window of 2^(32 - m) binades that ends at etop, the biased
// double exponent bound of every weight of the frame. Monotone non-decreasing in the 64-bit key read as
// unsigned: below the window (zero included) 0; above it, or a set sign bit, the largest key.
// tb: the key's width in bits (m mantissa bits, tb - m exponent bits; the largest key is 2^tb - 1)
DOFS_HD inline unsigned key32_of(unsigned long long k, int etop, int m, int tb = 32) {
    const unsigned top = tb >= 32 ? 0xFFFFFFFFu : (1u << tb) - 1u;
    if (k >> 63) return top;
    const int e = (int)((k >> 52) & 0x7FF), lo = etop - ((1 << (tb - m)) - 1);
    if (e > etop) return top;
    if (e < lo) return 0u;
    return ((unsigned)(e - lo) << m) | (unsigned)((k >> (52 - m)) & ((1ull << m) - 1));
}
// etop from a frame's largest |blurred component| M (float bits, C_BMAX): |dx|, |dy| <= 2M after the float
// subtraction, so a weight is at most 2 sqrt(2) M < 4 M: its double exponent is at most M's + 2
DOFS_HD inline int key32_etop(int mbits) {
    const int fe = (mbits >> 23) & 0xFF;
    return (fe > 0 ? fe : 1) - 127 + 1023 + 2;
}
DOFS_HD inline double bitsd(unsigned long long u) {
    union {
        double d;
        unsigned long long u;
    } c;
    c.u = u;
    return c.d;
}

// Edge (s, k) is a candidate of the MST search (all edges, or the allowed subset of a sharded frame)
DOFS_HD inline bool edge_allowed(const Ws& w, int f, int64_t s, int k) {
    return !w.allow || ((w.allow[f * w.d.N + s] >> k) & 1);
}

// cv::borderInterpolate(p, len, BORDER_REFLECT_101)
DOFS_HD inline int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p;
        else
            p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// ---------------------------------------------------------------------------------------------
// K1 — separable Gaussian blur (segment.cpp:52), OpenCV RowFilter then SymmColumnFilter order.
// ---------------------------------------------------------------------------------------------
struct KBlurRow {
    Ws w;
    DOFS_HD void operator()(int f, int64_t i) const {
        const int W = w.d.W;
        const int y = (int)(i / W), x = (int)(i % W);
        const F2* row = w.flow + f * w.flow_fstride + (int64_t)y * W;
        const int r = w.bn / 2;
        F2 s0 = row[reflect101(x - r, W)];
        float sx = w.bk[0] * s0.x, sy = w.bk[0] * s0.y;
        for (int t = 1; t < w.bn; ++t) {
            F2 v = row[reflect101(x - r + t, W)];
            sx += w.bk[t] * v.x;
            sy += w.bk[t] * v.y;
        }
        F2 o;
        o.x = sx;
        o.y = sy;
        w.tmp[f * w.d.N + i] = o;
    }
};

struct KBlurCol {
    Ws w;
    DOFS_HD void operator()(int f, int64_t i) const {
        const int W = w.d.W, H = w.d.H;
        const int y = (int)(i / W), x = (int)(i % W);
        const F2* t = w.tmp + f * w.d.N;
        const int r = w.bn / 2;
        F2 c = t[i];
        float sx = w.bk[r] * c.x + 0.0f, sy = w.bk[r] * c.y + 0.0f;
        for (int j = 1; j <= r; ++j) {
            F2 a = t[(int64_t)reflect101(y + j, H) * W + x];
            F2 b = t[(int64_t)reflect101(y - j, H) * W + x];
            sx += w.bk[r + j] * (a.x + b.x);
            sy += w.bk[r + j] * (a.y + b.y);
        }
        F2 o;
        o.x = sx;
        o.y = sy;
        w.blur[f * w.d.N + i] = o;
    }
};

// Column pass of a row band [r0, r0 + d.H) of an image of height Himg, from row-filtered rows
// [row0, row0 + rows) that include the blur halo: identical to KBlurCol on the whole image.
struct KBlurColBand {
    Ws w;
    int Himg, row0, r0;
    DOFS_HD void operator()(int f, int64_t i) const {
        const int W = w.d.W;
        const int y = r0 + (int)(i / W), x = (int)(i % W);
        const F2* t = w.tmp;
        const int r = w.bn / 2;
        F2 c = t[(int64_t)(y - row0) * W + x];
        float sx = w.bk[r] * c.x + 0.0f, sy = w.bk[r] * c.y + 0.0f;
        for (int j = 1; j <= r; ++j) {
            F2 a = t[(int64_t)(reflect101(y + j, Himg) - row0) * W + x];
            F2 b = t[(int64_t)(reflect101(y - j, Himg) - row0) * W + x];
            sx += w.bk[r + j] * (a.x + b.x);
            sy += w.bk[r + j] * (a.y + b.y);
        }
        F2 o;
        o.x = sx;
        o.y = sy;
        w.blur[i] = o;
    }
};

// ---------------------------------------------------------------------------------------------
// Lock-free union-find on an int parent array.
// ---------------------------------------------------------------------------------------------
DOFS_HD inline int uf_find(int* P, int x) {
    for (;;) {
        int p = dofs_ld(P + x);
        if (p == x) return x;
        int gp = dofs_ld(P + p);
        if (gp == p) return p;
        dofs_st(P + x, gp);  // path halving (x is not a root; P[x] only ever moves toward its root)
        x = gp;
    }
}
// Randomised linking: the root with the larger hash priority is hooked onto the other, so trees
// stay O(log n) deep in expectation even when unions arrive in monotone (chain) order.
DOFS_HD inline unsigned uf_prio(int x) {
    unsigned h = (unsigned)x * 0x9E3779B1u;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    return h;
}
DOFS_HD inline bool uf_above(int a, int b) {  // a is hooked below b
    const unsigned pa = uf_prio(a), pb = uf_prio(b);
    return pa > pb || (pa == pb && a > b);
}
DOFS_HD inline void uf_union(int* P, int a, int b) {
    for (;;) {
        a = uf_find(P, a);
        b = uf_find(P, b);
        if (a == b) return;
        if (!uf_above(a, b)) {
            int t = a;
            a = b;
            b = t;
        }
        if (dofs_cas(P + a, a, b) == a) return;
    }
}
DOFS_HD inline int uf_root_ro(const int* P, int x) {  // read-only walk (no writer in this kernel)
    int p = P[x];
    while (p != x) {
        x = p;
        p = P[x];
    }
    return x;
}

// ---------------------------------------------------------------------------------------------
// K2 — Borůvka MST on the implicit grid graph, strict order (weight bits, idx).
// ---------------------------------------------------------------------------------------------
struct KBoruvkaInit {
    Ws w;
    DOFS_HD void operator()(int f, int64_t p) const {
        const int64_t o = f * w.d.N + p;
        w.comp[o] = (int)p;
        w.uf[o] = (int)p;
        w.mstbits[o] = 0;
    }
};

// The minimum incident edge of pixel p in round 0 (every pixel its own component), as its slot 0-7 (0xFF:
// none) and emission index: slots 0-3 the edges p emits (left, up, up-left, down-left), 4-7 the edges its
// right, lower, lower-right and upper-right neighbours q[4..7] emit towards it; bq[j] the neighbours'
// blurred flows, ok[j] the slot's edge exists, allow_bits the edges the MST may use. The lexicographic
// minimum (weight, index): edge_weight(b, s, e) = sqrt(sq) with s the emitting pixel (float differences,
// double squares). sqrt is monotone and correctly rounded, so the minimum weight is sqrt of the minimum
// sq, and only edges whose sq lies within 2^-48 (relative) of it can tie with it (a weight's rounding
// interval is 2^-52 wide): one sqrt per pixel, not eight (as k_boruvka_min4 does in the later rounds).
// (KBoruvkaFirst, and k_boruvka_first_t's tile of LDS-staged flows in the HIP build.)
DOFS_HD inline int first_min_slot(F2 bp, const F2* bq, const bool* ok, unsigned allow_bits, int64_t p,
                                  const int64_t* q, unsigned* bidx_out) {
    unsigned long long sqb[8];
    unsigned long long msq = ~0ull;  // bits of non-negative doubles order like the values
DOFS_UNROLL
    for (int j = 0; j < 8; ++j) {
        const F2 bs = j < 4 ? bp : bq[j], be = j < 4 ? bq[j] : bp;
        const double dx = bs.x - be.x, dy = bs.y - be.y;
        sqb[j] = (ok[j] && ((allow_bits >> j) & 1)) ? dbits(sq_len(dx, dy)) : ~0ull;
        msq = sqb[j] < msq ? sqb[j] : msq;
    }
    unsigned bidx = kNoEdge;
    int jb = 0xFF;
    if (msq != ~0ull) {
        const double mv = bitsd(msq);
        const unsigned long long best = dbits(sqrt(mv));
        const unsigned long long thr = dbits(mv * 1.0000000000000036);  // (1 + 2^-48) mv
DOFS_UNROLL
        for (int j = 0; j < 8; ++j) {
            if (sqb[j] > thr) continue;  // also the non-candidates (~0)
            const bool tie = sqb[j] == msq || dbits(sqrt(bitsd(sqb[j]))) == best;
            const unsigned idx = (unsigned)(4 * (j < 4 ? p : q[j]) + (j & 3));
            if (tie && idx < bidx) {
                bidx = idx;
                jb = j;
            }
        }
    }
    *bidx_out = bidx;
    return jb;
}

// Round 0: every pixel is its own component, so its minimum edge is the min over its <= 8 incident
// edges (4 it emits, 4 its right/lower neighbours emit towards it) — no atomics. The minimum edges
// form a forest whose only cycles are the mutual pairs (a unique minimum per component under the
// strict order): each pixel points at the far end of its minimum edge (uf) and marks the edge;
// KBoruvkaPairs then roots each pair at its smaller pixel, and the relabel's finds (path halving)
// give every pixel its component — no unions, no CAS. The minima words start round 1 as "none".
struct KBoruvkaFirst {
    Ws w;
    DOFS_HD void operator()(int f, int64_t p) const {
        const Dims& d = w.d;
        const int x = (int)(p % d.W), y = (int)(p / d.W);
        const F2* b = w.blur + f * d.N;
        // all loads first (in-frame addresses; an absent neighbour reads the pixel itself and is
        // masked), as in k_boruvka_min's pass 0: slots 0-3 the edges p emits (left, up, up-left,
        // down-left), 4-7 the edges its right, lower, lower-right and upper-right neighbours emit
        const int64_t W = d.W;
        const bool xl = x > 0, xr = x + 1 < d.W, yu = y > 0, yd = y + 1 < d.H;
        const bool ok[8] = {xl, yu, d.nbr8 && xl && yu, d.nbr8 && xl && yd,
                            xr, yd, d.nbr8 && xr && yd, d.nbr8 && xr && yu};
        const int64_t nb[8] = {p - 1, p - W, p - W - 1, p + W - 1, p + 1, p + W, p + W + 1, p - W + 1};
        int64_t q[8];
        F2 bq[8];
DOFS_UNROLL
        for (int j = 0; j < 8; ++j) q[j] = ok[j] ? nb[j] : p;
        const F2 bp = b[p];
DOFS_UNROLL
        for (int j = 0; j < 8; ++j) bq[j] = b[q[j]];
        unsigned allow_bits = 0xff;  // bit j: slot j's edge may be in the MST
        if (w.allow) {
            const unsigned char* al = w.allow + f * d.N;
            allow_bits = al[p] & 0xfu;
            for (int j = 4; j < 8; ++j) allow_bits |= ((al[q[j]] >> (j - 4)) & 1u) << j;
        }
        unsigned bidx;
        const int jb = first_min_slot(bp, bq, ok, allow_bits, p, q, &bidx);
        const int64_t far = jb == 0xFF ? p : q[jb];
        // the pixel's minimum incident edge as its slot 0..7 (0xFF: none), in the leaf part of lite (free:
        // path-top flags are written and read for merge nodes only) until KMstEmit reads it
        if (w.single) w.lite[f * d.NL + p] = (unsigned char)jb;
        const int64_t o = f * d.N + p;
        w.bw[o] = ~0ull;
        w.bi[o] = kNoEdge;
        w.uf[o] = (int)far;
        if (bidx != kNoEdge) {
            reinterpret_cast<unsigned char*>(w.mstbits + f * d.N + (bidx >> 2))[bidx & 3] = 1;
            if (p == 0) w.C(f)[C_ACT + 0] = 1;
        }
    }
};
struct KBoruvkaPairs {  // a mutual pair of minimum edges: the smaller pixel becomes the root
    Ws w;
    DOFS_HD void operator()(int f, int64_t p) const {
        int* uf = w.uf + f * w.d.N;
        const int q = uf[p];
        if (q > (int)p && uf[q] == (int)p) uf[p] = (int)p;
    }
};

struct KBoruvkaReset {  // clear the per-component minima (measurement / fallback path; Hook clears them)
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t c) const {
        if (r > 0 && !w.C(f)[C_ACT + r - 1]) return;
        const int64_t o = f * w.d.N + c;
        w.bw[o] = ~0ull;
        w.bi[o] = kNoEdge;
    }
};

struct KBoruvkaMinW {
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t p) const {
        if (r > 0 && !w.C(f)[C_ACT + r - 1]) return;
        const Dims& d = w.d;
        const int x = (int)(p % d.W), y = (int)(p / d.W);
        const int* comp = w.comp + f * d.N;
        const F2* b = w.blur + f * d.N;
        unsigned long long* bw = w.bw + f * d.N;
        const int cp = comp[p];
        bool any = false;
        for (int k = 0; k < 4; ++k) {
            if (!edge_exists(d, x, y, k) || !edge_allowed(w, f, p, k)) continue;
            const int64_t q = edge_end(d, p, k);
            const int cq = comp[q];
            if (cp == cq) continue;
            const unsigned long long wb = dbits(edge_weight(b, p, q));
            if (wb < bw[cp]) dofs_amin_u64(bw + cp, wb);  // plain read first: bw only decreases
            if (wb < bw[cq]) dofs_amin_u64(bw + cq, wb);
            any = true;
        }
        if (any) w.C(f)[C_ACT + r] = 1;
    }
};

struct KBoruvkaMinI {
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t p) const {
        if (!w.C(f)[C_ACT + r]) return;
        const Dims& d = w.d;
        const int x = (int)(p % d.W), y = (int)(p / d.W);
        const int* comp = w.comp + f * d.N;
        const F2* b = w.blur + f * d.N;
        const unsigned long long* bw = w.bw + f * d.N;
        unsigned* bi = w.bi + f * d.N;
        const int cp = comp[p];
        for (int k = 0; k < 4; ++k) {
            if (!edge_exists(d, x, y, k) || !edge_allowed(w, f, p, k)) continue;
            const int64_t q = edge_end(d, p, k);
            const int cq = comp[q];
            if (cp == cq) continue;
            const unsigned long long wb = dbits(edge_weight(b, p, q));
            const unsigned idx = (unsigned)(4 * p + k);
            if (wb == bw[cp] && idx < bi[cp]) dofs_amin_u32(bi + cp, idx);
            if (wb == bw[cq] && idx < bi[cq]) dofs_amin_u32(bi + cq, idx);
        }
    }
};

// root c hooks along its minimum edge and clears its minima: the next round's minima of a root start
// from "none" (every root of round r + 1 is a root of round r, and only roots are keys of the minima)
DOFS_HD inline void boruvka_hook_root(const Ws& w, int f, int64_t c) {
    const Dims& d = w.d;
    const int* comp = w.comp + f * d.N;
    const int64_t o = f * d.N + c;
    const unsigned idx = w.bi[o];
    w.bw[o] = ~0ull;
    w.bi[o] = kNoEdge;
    if (idx == kNoEdge) return;
    const int64_t p = idx >> 2;
    const int k = idx & 3;
    const int64_t q = edge_end(d, p, k);
    reinterpret_cast<unsigned char*>(w.mstbits + f * d.N + p)[k] = 1;  // no atomic: one byte per edge
    uf_union(w.uf + f * d.N, comp[p], comp[q]);
}
struct KBoruvkaHook {  // every component root (HIP: k_boruvka_hook4, four pixels per lane)
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t c) const {
        if (!w.C(f)[C_ACT + r]) return;
        if (w.comp[f * w.d.N + c] == (int)c) boruvka_hook_root(w, f, c);
    }
};

struct KBoruvkaCompress {  // uf[c] = root
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t c) const {
        if (!w.C(f)[C_ACT + r]) return;
        int* uf = w.uf + f * w.d.N;
        int x = (int)c;
        int p = uf[x];
        if (p == x) return;
        while (true) {
            int gp = uf[p];
            if (gp == p) break;
            p = gp;
        }
        uf[c] = p;
    }
};

struct KBoruvkaRelabelFind {  // comp[p] = the root of its component (finds with path halving)
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t p) const {
        if (!w.C(f)[C_ACT + r]) return;
        int* comp = w.comp + f * w.d.N;
        const int c = comp[p];
        const int root = uf_find(w.uf + f * w.d.N, c);
        if (root != c) comp[p] = root;
    }
};

struct KBoruvkaRelabel {
    Ws w;
    int r;
    DOFS_HD void operator()(int f, int64_t p) const {
        if (!w.C(f)[C_ACT + r]) return;
        int* comp = w.comp + f * w.d.N;
        comp[p] = w.uf[f * w.d.N + comp[p]];
    }
};

// ---------------------------------------------------------------------------------------------
// MST edge list in emission order, then (after the radix sort) in Kruskal order.
// ---------------------------------------------------------------------------------------------
// the four edge bytes of a pixel's MST word as bits 0..3
DOFS_HD inline unsigned mst_bits(int word) {
    const unsigned v = (unsigned)word;
    return (v & 1u) | ((v >> 7) & 2u) | ((v >> 14) & 4u) | ((v >> 21) & 8u);
}

struct KMaskOut {  // a band's minimum spanning forest as per-pixel emitted-edge bits
    Ws w;
    unsigned char* mask;
    DOFS_HD void operator()(int, int64_t p) const { mask[p] = (unsigned char)mst_bits(w.mstbits[p]); }
};

struct KMstCount {
    Ws w;
    DOFS_HD void operator()(int f, int64_t p) const {
        w.cnt[f * w.d.N + p] = __builtin_popcount(mst_bits(w.mstbits[f * w.d.N + p]));
    }
};

// singleton flags (Ws::single): in the sorted values' two top bits (KMstEmit; the sort fix-up compares
// values below them), then in EU / EV bit kSingleBit (KEdgeInit; pixel ids are < 2^26)
constexpr unsigned kValSingleS = 1u << 30, kValSingleE = 1u << 31;
constexpr int kSingleBit = 30;
constexpr int kEndMask = (1 << kSingleBit) - 1;
struct KMstEmit {
    Ws w;
    int fshift;  // > 0: the frame id rides above the emission index (one batch-wide frame sort, HIP)
    int k32m = 0;  // > 0: 32-bit keys (key32_of, this many mantissa bits) into key_in's first half (HIP)
    int k32b = 32;  // their width in bits (key32_of's tb)
    DOFS_HD void operator()(int f, int64_t p) const {
        const Dims& d = w.d;
        const int bits = (int)mst_bits(w.mstbits[f * d.N + p]);
        if (!bits) return;
        const int etop = k32m ? key32_etop(w.C(f)[C_BMAX]) : 0;
        int64_t j = w.off[f * d.N + p];
        const F2* b = w.blur + f * d.N;
        // the flow of p and of its MST edges' far ends read together (an unused slot re-reads p)
        const F2 bp = b[p];
        F2 bq[4];
        DOFS_UNROLL
        for (int k = 0; k < 4; ++k) bq[k] = b[(bits >> k) & 1 ? edge_end(d, p, k) : p];
        unsigned ms = 0xFF, mq[4] = {0xFF, 0xFF, 0xFF, 0xFF};  // minimum-edge slots of p and of the far ends
        if (w.single) {
            const unsigned char* lt = w.lite + f * d.NL;
            ms = lt[p];
            DOFS_UNROLL
            for (int k = 0; k < 4; ++k) mq[k] = (bits >> k) & 1 ? lt[edge_end(d, p, k)] : 0xFF;
        }
        DOFS_UNROLL
        for (int k = 0; k < 4; ++k) {
            if (!(bits & (1 << k))) continue;
            if (j < d.M) {
                const double dx = bp.x - bq[k].x, dy = bp.y - bq[k].y;  // edge_weight(b, p, q)
                const unsigned long long key = dbits(sqrt(sq_len(dx, dy)));
                if (k32m)
                    reinterpret_cast<unsigned*>(w.key_in)[f * d.M + j] = key32_of(key, etop, k32m, k32b);
                else
                    w.key_in[f * d.M + j] = key;
                // p's first merge is its minimum edge (slot k); the far end receives this edge in its slot 4 + k
                const unsigned sg = (ms == (unsigned)k ? kValSingleS : 0u) | (mq[k] == (unsigned)(4 + k) ? kValSingleE : 0u);
                w.val_in[f * d.M + j] = (unsigned)(4 * p + k) | (fshift ? (unsigned)f << fshift : 0u) | sg;
            }
            ++j;
        }
        if (p == d.N - 1) {
            w.C(f)[C_MST] = (int)j;
            // the offsets' scan took N - 1 edges per unmasked frame (scan_excl_total): a frame that ends
            // elsewhere (never, for a connected grid) has shifted every later frame's edges — fail loudly
            if (!w.allow && j != d.M) dofs_aor(w.C(0) + C_FLOWERR, kErrMst);
        }
    }
};

struct KEdgeInit {  // endpoints by rank; labels = the endpoints (global-kernel KRT only: `labels`)
    Ws w;
    bool labels;
    bool given = false;   // EU / EV already hold the merges (segment_graph on a caller's edge list)
    unsigned vmask = ~0u;  // the emission index bits of val_out (a frame id may sit above them)
    DOFS_HD void operator()(int f, int64_t i) const {
        const Dims& d = w.d;
        const int64_t o = f * d.M + i;
        int64_t p, q;
        if (given) {
            p = w.EU[o];
            q = w.EV[o];
        } else {
            const unsigned val = w.val_out[o];
            const unsigned idx = val & vmask;
            p = idx >> 2;
            q = edge_end(d, p, idx & 3);
            const int su = w.single && (val & kValSingleS) ? 1 << kSingleBit : 0;
            const int sv = w.single && (val & kValSingleE) ? 1 << kSingleBit : 0;
            w.EU[o] = (int)p | su;
            w.EV[o] = (int)q | sv;
        }
        if (!labels) return;  // the sweep writes every merge's block-start labels
        w.lu[o] = (int)p;
        w.lv[o] = (int)q;
        w.own[o] = 0;
    }
};

// ---------------------------------------------------------------------------------------------
// build_graph (graph.cpp:51-103) as a sorted edge list: every emitted edge's weight bits and emission
// index, radix-sorted (stable) — the reference's multiset order (weight, emission order).
// ---------------------------------------------------------------------------------------------
struct KGraphKeys {
    const F2* flow;
    Dims d;
    unsigned long long* key;
    unsigned* val;
    DOFS_HD void operator()(int, int64_t i) const {  // i = 4 p + k over all pixels
        const int64_t p = i >> 2;
        const int k = (int)(i & 3);
        const int x = (int)(p % d.W), y = (int)(p / d.W);
        if (edge_exists(d, x, y, k)) {
            key[i] = dbits(edge_weight(flow, p, edge_end(d, p, k)));
            val[i] = (unsigned)i;
        } else {  // sorts behind every edge (weights are >= +0, NaN bits below ~0)
            key[i] = ~0ull;
            val[i] = kNoEdge;
        }
    }
};
struct KGraphEdges {  // Edge {start, end, weight} (graph.hpp:13-17, create_edge graph.cpp:43-49)
    const unsigned long long* key;
    const unsigned* val;
    Dims d;
    dofs_edge* out;
    DOFS_HD void operator()(int, int64_t i) const {
        const unsigned idx = val[i];
        const int64_t p = idx >> 2;
        dofs_edge e;
        e.start = (int32_t)p;
        e.end = (int32_t)edge_end(d, p, idx & 3);
        e.weight = bitsd(key[i]);
        out[i] = e;
    }
};

// ---------------------------------------------------------------------------------------------
// segment_graph on a caller's edge list (graph.cpp:503-536): Kruskal over the list in its order
// accepts exactly the minimum spanning forest under the strict order "position in the list", which
// Borůvka finds in O(log N) rounds (per component the incident cross edge of least position; hooks
// follow strictly decreasing positions except mutual pairs, rooted at the smaller id). Accepted edges
// in list order are the merges; if they form a forest, the component roots are chained by extra
// merges after them (Ws::mreal says where the caller's merges end; those are never scored).
// Per-vertex arrays: comp (component root label), uf (hooks), bi (least incident position).
// Round flags: counters C_ACT + r of frame 0.
// ---------------------------------------------------------------------------------------------
struct KElInit {
    Ws w;
    DOFS_HD void operator()(int, int64_t v) const {
        w.comp[v] = (int)v;
        w.uf[v] = (int)v;
        w.bi[v] = kNoEdge;
    }
};
struct KElMin {
    Ws w;
    const dofs_edge* e;
    int r;
    DOFS_HD void operator()(int, int64_t i) const {
        if (r > 0 && !w.ctr[C_ACT + r - 1]) return;
        const int a = w.comp[e[i].start], b = w.comp[e[i].end];
        if (a == b) return;
        dofs_amin_u32(w.bi + a, (unsigned)i);
        dofs_amin_u32(w.bi + b, (unsigned)i);
        if (!w.ctr[C_ACT + r]) dofs_st(w.ctr + C_ACT + r, 1);
    }
};
struct KElHook {
    Ws w;
    const dofs_edge* e;
    int* acc;  // per edge: accepted (an MSF edge)
    int r;
    DOFS_HD void operator()(int, int64_t c) const {
        if (!w.ctr[C_ACT + r] || w.comp[c] != (int)c) return;
        const unsigned m = w.bi[c];
        if (m == kNoEdge) return;
        const int a = w.comp[e[m].start], b = w.comp[e[m].end];
        const int o = a == (int)c ? b : a;
        acc[m] = 1;
        if (w.bi[o] == m && (int)c < o) return;  // mutual pair: the smaller root stays a root
        w.uf[c] = o;
    }
};
struct KElRelabel {
    Ws w;
    int r;
    DOFS_HD void operator()(int, int64_t p) const {
        if (!w.ctr[C_ACT + r]) return;
        const int c = w.comp[p];
        const int root = uf_find(w.uf, c);
        if (root != c) w.comp[p] = root;
        w.bi[p] = kNoEdge;  // the hook has read every minimum of this round
    }
};
struct KElEmit {  // accepted edges in list order: merge j = the j-th accepted edge
    Ws w;
    const dofs_edge* e;
    const int* acc;
    const int* off;
    DOFS_HD void operator()(int, int64_t i) const {
        if (!acc[i]) return;
        const int j = off[i];
        w.EU[j] = e[i].start;
        w.EV[j] = e[i].end;
        w.key_out[j] = dbits(e[i].weight);
    }
};
struct KElRootFlag {
    Ws w;
    DOFS_HD void operator()(int, int64_t v) const { w.cnt[v] = w.comp[v] == (int)v ? 1 : 0; }
};
struct KElRootList {  // the forest's roots in ascending id
    Ws w;
    DOFS_HD void operator()(int, int64_t v) const {
        if (w.comp[v] == (int)v) w.cur[w.off[v]] = (int)v;
    }
};
struct KElChain {  // merge mreal + j joins the components of roots j and j + 1 (after every real merge)
    Ws w;
    DOFS_HD void operator()(int, int64_t j) const {
        w.EU[w.mreal + j] = w.cur[j];
        w.EV[w.mreal + j] = w.cur[j + 1];
        w.key_out[w.mreal + j] = 0x7FF0000000000000ull;  // +inf: not an edge of the caller's graph
    }
};
struct KCopyFlow {  // the flow as given (segment_graph does not blur)
    Ws w;
    DOFS_HD void operator()(int f, int64_t p) const { w.blur[f * w.d.N + p] = w.flow[f * w.flow_fstride + p]; }
};

// ---------------------------------------------------------------------------------------------
// K3 block-start labels by one sequential sweep over rank blocks: a pixel
// union-find holds the forest of all merges before the current block; a block's endpoint labels
// are read from it (the component's max merge rank, or the pixel itself while it is alone), then
// the block's merges are united into it and each resulting component records its new max rank and
// size. Replaces the top-down global depths: one union per merge instead of one per depth.
// Arrays (per frame, stride N): kpar = parent, ksz = size at roots, klab = max merge rank at roots
// (-1: a single pixel).
// ---------------------------------------------------------------------------------------------
struct KSeqInit {
    int* kpar;
    int* ksz;
    int* klab;
    int64_t N;
    DOFS_HD void operator()(int f, int64_t x) const {
        const int64_t o = f * N + x;
        kpar[o] = (int)x;
        ksz[o] = 1;
        klab[o] = -1;
    }
};
// label of pixel x whose component root is r
DOFS_HD inline int seq_label(const int* klab, int r, int x, int64_t N) {
    const int j = dofs_ld((int*)klab + r);
    return j < 0 ? x : (int)(N + j);
}
// union returning the root it hooked (-1: already one component)
DOFS_HD inline int uf_union_hooked(int* P, int a, int b) {
    for (;;) {
        a = uf_find(P, a);
        b = uf_find(P, b);
        if (a == b) return -1;
        if (!uf_above(a, b)) {
            const int t = a;
            a = b;
            b = t;
        }
        if (dofs_cas(P + a, a, b) == a) return a;
    }
}
// size of KRT node N + j (label size for the deep kernel: SZ; and the high half of its label word
// for the global-kernel form of the deep depths)
DOFS_HD inline void seq_set_size(const Ws& w, int f, int j, int sz) {
    const int64_t o = f * w.d.NL + w.d.N + j;
    w.SZ[o] = sz;
    if (w.P) ((int*)(w.P + o))[1] = sz;
}

// pointer-jumping word: (ancestor, offset sum) packed
DOFS_HD inline unsigned long long jump_pack(int anc, int sum) {
    return (unsigned long long)(unsigned)anc | ((unsigned long long)(unsigned)sum << 32);
}
DOFS_HD inline int jump_anc(unsigned long long v) { return (int)(unsigned)(v & 0xffffffffu); }
DOFS_HD inline int jump_sum(unsigned long long v) { return (int)(unsigned)(v >> 32); }

struct KLabelInit {  // pixel sizes, the root's size / jump word / path-top flag; full: also the
    Ws w;           // global-kernel KRT's words (untagged label words, zero counters) over NL
    bool full;      // (launched over NL when full, over N otherwise)
    DOFS_HD void operator()(int f, int64_t x) const {
        const Dims& d = w.d;
        const int64_t o = f * d.NL + x;
        if (!full) {
            w.SZ[o] = 1;
            if (x == 0) {  // KRT root = last merge: the whole frame (preorder 0, a path top)
                const int64_t r = f * d.NL + d.NL - 1;
                w.SZ[r] = (int)d.N;
                w.J[r] = jump_pack(-1, 0);
                w.lite[r] = 1;
            }
            return;
        }
        if (w.MX) w.MX[o] = 0;  // (the global-kernel KRT's arrays exist only where it runs)
        if (w.CS) w.CS[o] = 0;
        int sz = 0;
        if (x < d.N) {
            sz = 1;
            w.SZ[o] = 1;
        } else if (x == d.NL - 1) {
            sz = (int)d.N;
            w.SZ[o] = sz;
            w.J[o] = jump_pack(-1, 0);
            w.lite[o] = 1;
        }
        if (w.P) w.P[o] = (unsigned long long)(unsigned)sz << 32;  // link word epoch 0: a root at every depth
    }
};

// ---------------------------------------------------------------------------------------------
// K3 — KRT by top-down divide and conquer over rank blocks. At depth d with
// block size S: L = first S/2 ranks of a block, R = the rest. Labels of every edge endpoint are the
// components at the start of its block (pixel id, or N + max edge rank of the component). The
// L-edges of all blocks form a forest over a collision-free label space; its components get the
// label N + (max L rank). After the last depth (S = 2) every edge's endpoint labels are the
// components it merges at its own rank — its two KRT children (KDncParent).
// ---------------------------------------------------------------------------------------------
DOFS_HD inline bool dnc_is_L(const Dims& d, int64_t i, int64_t S) {
    const int64_t h = S >> 1;
    const int64_t s = i & ~(S - 1);
    return (i - s) < h && (s + h) < d.M;  // L edge of a block whose R half is non-empty
}
DOFS_HD inline bool dnc_is_R(int64_t i, int64_t S) { return (i & (S - 1)) >= (S >> 1); }

// Union-find over the label space of one depth, linking by component size (big components stay
// roots, so the many small components touching one big component hook onto it without CAS
// contention on its root), ties by hash. Returns the label whose parent pointer this union set:
// in a forest every edge hooks exactly one label and every non-root label is hooked by exactly one
// edge, which gives each label a unique owner without atomics.
//
// Depth tags instead of cleanup passes: parent words are (tag | parent) and max-rank words
// (tag | rank) with tag = the depth's epoch (1, 2, ... from the top depth down, above the label
// bits). A word with another depth's tag reads as "root" / "untouched", so nothing a depth writes
// needs restoring; the one counter (CS) is re-zeroed by the single L-root lane that consumes it.
constexpr int kLabBits = 27;  // labels < N + M < 2^27 (H*W < 2^26)
constexpr unsigned kLabMask = (1u << kLabBits) - 1;
constexpr int kRankBits = 26;  // ranks < M < 2^26; epochs <= 31 keep (epoch << 26 | rank) >= 0
constexpr int kRankMask = (1 << kRankBits) - 1;
DOFS_HDM inline int dnc_epoch(int64_t M, int64_t S) {  // 1 at the top depth, +1 per halving
    int top = 0, s = 0;
    while (((int64_t)1 << top) < M) ++top;
    while (((int64_t)1 << s) < S) ++s;
    return top - s + 1;
}
// Label word (64-bit): low half = link (tag | parent), high half = the label's component size, so
// a find step reads a label's parent and size in one access (the union's size comparison and the
// compress pass's size sum need no separate load).
DOFS_HD inline unsigned lab_link(unsigned long long v) { return (unsigned)v; }
DOFS_HD inline int lab_size(unsigned long long v) { return (int)(v >> 32); }
DOFS_HD inline void lab_set_link(unsigned long long* P, int x, unsigned link) {  // low half only
    dofs_st((int*)(P + x), (int)link);
}
DOFS_HD inline int dnc_find(unsigned long long* P, int x, unsigned tag, unsigned long long* word) {
    for (;;) {
        const unsigned long long v = dofs_ld64(P + x);
        if ((lab_link(v) & ~kLabMask) != tag) {
            *word = v;
            return x;
        }
        const int p = (int)(lab_link(v) & kLabMask);
        const unsigned long long vp = dofs_ld64(P + p);
        if ((lab_link(vp) & ~kLabMask) != tag) {
            *word = vp;
            return p;
        }
        const int gp = (int)(lab_link(vp) & kLabMask);
        lab_set_link(P, x, tag | (unsigned)gp);  // path halving
        x = gp;
    }
}
DOFS_HD inline int dnc_union(unsigned long long* P, int a, int b, unsigned tag) {
    for (;;) {
        unsigned long long va, vb;
        a = dnc_find(P, a, tag, &va);
        b = dnc_find(P, b, tag, &vb);
        if (a == b) return -1;  // unreachable: L-edges form a forest over the labels
        const int sa = lab_size(va), sb = lab_size(vb);
        if (!(sa != sb ? sa < sb : uf_above(a, b))) {  // a is hooked below b
            const int t = a;
            a = b;
            b = t;
            va = vb;
        }
        const unsigned long long nv = (va & 0xFFFFFFFF00000000ull) | (tag | (unsigned)b);
        if (dofs_cas64(P + a, va, nv) == va) return a;
    }
}
DOFS_HD inline int walk_compress(unsigned long long* P, int x, unsigned tag, int* size_x) {
    unsigned long long v = P[x];  // no union runs concurrently: plain loads
    *size_x = lab_size(v);
    int r = x;
    while ((lab_link(v) & ~kLabMask) == tag) {
        r = (int)(lab_link(v) & kLabMask);
        v = P[r];
    }
    for (int y = x; y != r;) {
        const int p = (int)(lab_link(P[y]) & kLabMask);
        if (p != r) ((unsigned*)(P + y))[0] = tag | (unsigned)r;
        y = p;
    }
    return r;
}
DOFS_HD inline int dnc_root(const unsigned long long* P, int x, unsigned tag) {  // after compress: one hop
    const unsigned v = lab_link(P[x]);
    return (v & ~kLabMask) == tag ? (int)(v & kLabMask) : x;
}

struct KDncUnion {
    Ws w;
    int64_t S;
    int ep;
    DOFS_HD void operator()(int f, int64_t i) const {
        const Dims& d = w.d;
        if (!dnc_is_L(d, i, S)) return;
        const int64_t o = f * d.M + i;
        const int64_t lb = f * d.NL;
        w.own[o] = dnc_union(w.P + lb, w.lu[o], w.lv[o], (unsigned)ep << kLabBits);
    }
};

struct KDncCompress {
    Ws w;
    int64_t S;
    int ep;
    DOFS_HD void operator()(int f, int64_t i) const {
        const Dims& d = w.d;
        if (!dnc_is_L(d, i, S)) return;  // uniform per wave while S/2 >= 64 (aggregation below)
        const int64_t o = f * d.M + i;
        const int64_t lb = f * d.NL;
        const int h = w.own[o];
        int szh;
        const int r = walk_compress(w.P + lb, h, (unsigned)ep << kLabBits, &szh);
        // component size over the labels hooked in it (the root label is added by the L-root
        // edge) and the max L-edge rank (depth-tagged); wave-aggregated: a big component's root is
        // the key of most lanes at the top levels
        dofs_agg_add(w.CS + lb, r, szh, true);
        dofs_agg_max(w.MX + lb, r, (ep << kRankBits) | (int)i, true);
        w.own[o] = r;  // L-root candidate: its component's root (the HIP pass keeps per-workgroup maxima only)
    }
};

// After KDncCompress (roots final, hooked labels point at them): an L edge whose rank is its
// component's max (an L-root) gets the component size; an R edge relabels its endpoints to the
// components' new labels.
struct KDncLRootRelabel {
    Ws w;
    int64_t S;
    int ep;
    DOFS_HD void operator()(int f, int64_t i) const {
        const Dims& d = w.d;
        const int64_t o = f * d.M + i;
        const int64_t lb = f * d.NL;
        const unsigned tag = (unsigned)ep << kLabBits;
        const int mtag = ep << kRankBits;
        if (dnc_is_L(d, i, S)) {
            const int r = w.own[o];  // candidate's root (-1: not the max rank of its component)
            if (r < 0 || w.MX[lb + r] != (mtag | (int)i)) return;
            const int sz = w.CS[lb + r] + lab_size(w.P[lb + r]);
            w.CS[lb + r] = 0;  // the only reader of this component's counter
            ((int*)(w.P + lb + d.N + i))[1] = sz;  // the new label's size (high half of its word)
            w.SZ[lb + d.N + i] = sz;
            return;
        }
        if (!dnc_is_R(i, S)) return;
        for (int side = 0; side < 2; ++side) {
            int* lp = side ? (w.lv + o) : (w.lu + o);
            const int x = *lp;
            const int r = dnc_root(w.P + lb, x, tag);
            // x is a label of this block's L forest <=> hooked this depth or a touched root
            const int m = w.MX[lb + r];
            if (r != x || (m & ~kRankMask) == mtag) *lp = (int)(d.N + (m & kRankMask));
        }
    }
};

// Final labels (lu, lv) of edge i = its KRT children (start side A, end side B): every node gets
// its parent from the one edge whose final label it is. Here each merge also splits its children
// into heavy (larger subtree; ties → A) and light, and seeds the heavy-first preorder's pointer
// jumping (K4): a heavy child sits right after its parent (offset 1), the light one after the
// parent's whole heavy subtree (offset 1 + 2*size(heavy) - 1). The light child starts a heavy path.
DOFS_HD inline unsigned long long hl_pack(int sh, int sl) {
    return (unsigned long long)(unsigned)sh | ((unsigned long long)(unsigned)sl << 32);
}
struct KDncParent {
    Ws w;
    DOFS_HD void operator()(int f, int64_t i) const {
        const Dims& d = w.d;
        const int64_t o = f * d.M + i, lb = f * d.NL;
        const int a = w.lu[o], b = w.lv[o];
        const int sa = w.SZ[lb + a], sb = w.SZ[lb + b];
        const bool lightB = sa >= sb;
        const int h = lightB ? a : b, l = lightB ? b : a;
        const int x = (int)(d.N + i);
        w.J[lb + h] = jump_pack(x, 1);
        w.J[lb + l] = jump_pack(x, 2 * (lightB ? sa : sb));
        w.lite[lb + h] = 0;
        w.lite[lb + l] = 1;
        w.hlB[o] = lightB ? 1 : 0;
        w.hls[o] = hl_pack(lightB ? sa : sb, lightB ? sb : sa);
    }
};

// ---------------------------------------------------------------------------------------------
// K4 — heavy-first preorder of the KRT (every heavy path becomes a contiguous range) via
// pointer jumping over parent links with accumulated offsets (seeded by KDncParent).
// ---------------------------------------------------------------------------------------------
// heavy child of internal node y (light side recorded by KDncParent)
DOFS_HD inline int heavy_child(const Ws& w, int f, int y, int* light, int* light_is_B) {
    const int64_t e = f * w.d.M + (y - w.d.N);
    const int a = w.lu[e], b = w.lv[e];  // final labels = children
    if (w.hlB[e]) {
        *light = b;
        *light_is_B = 1;
        return a;
    }
    *light = a;
    *light_is_B = 0;
    return b;
}

// In-place asynchronous pointer jumping. Invariant: J[x] = (a, s) with s = the sum of the offsets
// from x (inclusive) up to its ancestor a (exclusive); a = -1 once s reaches the root. Every
// 64-bit snapshot of J[a] satisfies it too, so x may jump over a with whatever value of J[a] it
// reads, in any order: each round at least halves every remaining distance, as the synchronous
// double-buffered form does, at half the traffic (one array, converged nodes idle).
struct KJump {  // `hops` jumps per launch (each on the freshest ancestor word it reads)
    unsigned long long* J;
    int64_t NL;
    int hops;
    int64_t first;  // node range [first, NL): the merge nodes (leaves are resolved by KJumpLeaf)
    DOFS_HD void operator()(int f, int64_t k) const {
        const int64_t x = first + k;
        const int64_t o = f * NL + x;
        unsigned long long v = dofs_ld64(J + o);
        if (jump_anc(v) < 0) return;
        for (int h = 0; h < hops; ++h) {
            const int a = jump_anc(v);
            if (a < 0) break;
            const unsigned long long u = dofs_ld64(J + f * NL + a);
            v = jump_pack(jump_anc(u), jump_sum(v) + jump_sum(u));
        }
        dofs_st64(J + o, v);
    }
};

struct KJumpLeaf {  // a pixel (leaf) hangs off a merge: one jump once the merges have converged
    unsigned long long* J;
    int64_t NL;
    DOFS_HD void operator()(int f, int64_t x) const {
        const int64_t o = f * NL + x;
        const unsigned long long v = J[o];
        const int a = jump_anc(v);
        if (a < 0) return;
        J[o] = jump_pack(-1, jump_sum(v) + jump_sum(J[f * NL + a]));
    }
};

struct KOrd {  // preorder positions; a leaf (x < N) takes its last jump here (KJumpLeaf's, not stored)
    Ws w;
    DOFS_HD void operator()(int f, int64_t x) const {
        const Dims& d = w.d;
        const unsigned long long v = w.J[f * d.NL + x];
        const int a = jump_anc(v);
        const int q = jump_sum(v) + (x < d.N && a >= 0 ? jump_sum(w.J[f * d.NL + a]) : 0);
        w.pre[f * d.NL + x] = q;
        w.ord[f * d.NL + q] = (int)x;  // leaf ranks: scan of (ord < N)
    }
};

struct KLeafOrder {  // one lane per preorder position: leaf ranks rise with the position, so both the
    Ws w;           // reads (ord, lscan) and the leaves' stores (leaf_order) are coalesced
    const int* pre;
    DOFS_HD void operator()(int f, int64_t q) const {
        const Dims& d = w.d;
        const int v = w.ord[f * d.NL + q];
        if (v >= d.N) return;  // a merge
        const int r = w.lscan[f * d.NL + q];
        w.leaf_order[f * d.N + r] = v;
        w.lposr[f * d.N + r] = (int)q;
    }
};

constexpr int kTinyPath = 8;    // short heavy paths of at most this many merges form round 0's first list
constexpr int kLongPath = 256;  // default: heavy paths at least this long go to the wave-cooperative replay
// state_at() at a heavy-path top: the replay phase its path completed in, or one of these pending
// states (all compare >= any phase, i.e. "not ready")
constexpr int kPendLong = kIntMax - 1;  // long path, not complete
constexpr int kParkBase = kIntMax - 2;  // long path stopped in round r: kParkBase - r


// The replay's inputs of the merge at preorder position q (Forest::merge, graph.cpp:170-218): heavy and
// light child sizes hl (sh | sl << 32), the light child lt (its side lB), whether q tops a heavy path
DOFS_HD inline StepIn step_in(const Ws& w, int f, int q, bool top, int lt, int lB, unsigned long long hl) {
    const Dims& d = w.d;
    const int sh = (int)(unsigned)(hl & 0xffffffffu), sl = (int)(unsigned)(hl >> 32);
    (void)q;
    int meta = (lB ? kStepB : 0) | (top ? kStepTop : 0) | (sh + sl >= w.min_size ? kStepKeep : 0);
    StepIn in;
    if (lt < d.N) {
        const F2 v = w.blur[f * d.N + lt];
        in.wbx = v.x * (float)1;
        in.wby = v.y * (float)1;
        in.lt = lt;
    } else {
        meta |= kStepDyn;  // (the light child's position q + 2 sh follows from the record's own)
        in.wbx = in.wby = 0.f;
        in.lt = sl;
    }
    in.hs = (unsigned)sh | ((unsigned)meta << kStepShift);
    return in;
}

struct KPathInit {  // one lane per merge node x = N + k; path ids and lists through the list taker
    Ws w;
    const int* pre;
    static constexpr bool kBlockTake = true;
    template <class T>
    DOFS_HD void operator()(int f, int64_t k, bool valid, T& t) const {
        const Dims& d = w.d;
        const int64_t x = d.N + k;
        const int64_t lb = f * d.NL;
        bool top = false, islong = false;
        int q = 0, qb = 0;
        if (valid) {
            q = pre[lb + x];
            top = w.lite[lb + x] != 0;
            {
                int lt, lB;
                heavy_child(w, f, (int)x, &lt, &lB);
                const unsigned long long hl = w.hls[f * d.M + k];  // children's sizes (the KRT's parent pass)
                w.In[lb + q] = step_in(w, f, q, top, lt, lB, hl);
            }
            if (top) {  // heavy path [q, bottom): its bottom leaf is the first leaf after q in preorder
                qb = w.lposr[f * d.N + w.lscan[lb + q]];
                islong = qb - q >= w.long_path;
            }
            if (top) *state_at(w, lb + q) = islong ? kPendLong : kIntMax;  // read at path tops only
            if (islong) dofs_aadd(w.C(f) + C_LONGM, qb - q);
        }
        // short paths in two lists by length, so round 0's waves hold paths of like length (a wave
        // runs as long as its longest path): tiny ones from the back of list_short, the rest from
        // its front (together at most one per merge < N: the two never meet)
        const bool tiny = top && !islong && qb - q <= kTinyPath;
        // merges whose replay record the lean replay stores (the replay's byte census, bench.py)
        (void)t.take(w.C(f) + C_KEEP, valid && w.SZ[lb + x] >= w.min_size);
        int j, jl, js;
        t.take3(w.C(f) + C_PATHS, top, w.C(f) + C_LONG, islong, w.C(f) + C_SHORT, top && !islong && !tiny, &j, &jl,
                &js);
        const int jt = t.take(w.C(f) + C_TINY, tiny);
        if (top) {
            w.cur[f * d.N + j] = qb - 1;
            w.ptop[f * d.N + j] = q;
            if (islong) {
                w.list_long[f * d.N + jl] = j;
                if (q == 0) w.C(f)[C_ROOTL] = jl + 1;  // the KRT root's path: the frame's longest chain
            }
            else if (tiny)
                w.list_short[f * d.N + d.N - 1 - jt] = j;
            else
                w.list_short[f * d.N + js] = j;
        }
        // leaves: nothing — a path's bottom leaf state is read from the flow by the replay itself
        // (path_start), a light leaf's inputs are in its parent's StepIn
    }
};

// Forest::merge (graph.cpp:170-218) of the running (heavy) set with a light child:
//   mean = ((m_h * (float)s_h) + (m_l * (float)s_l)) * (1. / (s_h + s_l))  [float, float, double→float]
//   root = rank(A) > rank(B) ? root(A) : root(B), A = start side;  rank += (rank(A) == rank(B))
struct RunState {
    float mx, my;
    int rank, root;
    B4 bb;
};
DOFS_HD inline void step_merge(RunState& s, float fs, float wbx, float wby, double r, int meta, int lrank,
                               int lroot, B4 lbb) {
    const float tx = s.mx * fs, ty = s.my * fs;
    s.mx = (float)((double)(tx + wbx) * r);
    s.my = (float)((double)(ty + wby) * r);
    const int nroot = (meta & kStepB) ? (s.rank > lrank ? s.root : lroot) : (lrank > s.rank ? lroot : s.root);
    s.rank = (s.rank == lrank) ? s.rank + 1 : (s.rank > lrank ? s.rank : lrank);
    s.root = nroot;
    s.bb.x0 = lbb.x0 < s.bb.x0 ? lbb.x0 : s.bb.x0;  // graph.cpp:197-207
    s.bb.y0 = lbb.y0 < s.bb.y0 ? lbb.y0 : s.bb.y0;
    s.bb.x1 = lbb.x1 > s.bb.x1 ? lbb.x1 : s.bb.x1;
    s.bb.y1 = lbb.y1 > s.bb.y1 ? lbb.y1 : s.bb.y1;
}

// K5 — sequential replay along one heavy path (bottom-up), round `round`: advances until a light
// child not completed in an earlier round is met (resumed next round) or the path top is done.
// `list`/`count` select the short-path or the long-path list (the HIP build replays long paths
// with the two-wave kernel of dofs_hip.hip instead; same state, same results).
// State at preorder position qb (just below a path cursor): a leaf's singleton set (its blurred
// flow, rank 0, root = itself, its pixel as bbox), or a merge's replay outputs.
DOFS_HD inline void path_start(const Ws& w, int f, int64_t qb, float* mx, float* my, int* rank, int* root, B4* bb) {
    const Dims& d = w.d;
    const int64_t lb = f * d.NL;
    const int x = w.ord[lb + qb];
    if (x < d.N) {
        const F2 v = w.blur[f * d.N + x];
        *mx = v.x;
        *my = v.y;
        *rank = 0;
        *root = x;
        bb->x0 = bb->x1 = (int16_t)(x % d.W);
        bb->y0 = bb->y1 = (int16_t)(x / d.W);
        return;
    }
    const RepVal v = w.Rv[lb + qb];
    *mx = v.mx;
    *my = v.my;
    *rank = v.rank;
    *root = v.root;
    *bb = v.bb;
}

// Replay kernels run in phases: round r's short-path pass is phase 2r, its long-path pass 2r+1
// (a path top's state word, state_at(), = the phase it completed in). A pass sees completions of earlier phases.
// Advances heavy paths bottom-up until they complete or block on a light child whose path has not
// completed yet. A parked path is appended to `out` (the next round's list; one block-aggregated
// counter atomic per block), so later rounds only visit the paths still pending. out == nullptr:
// the list is rescanned every round (the emulator's long paths).
struct KReplay {
    Ws w;
    int phase;
    const int* list;
    int count;  // counter index of list's length (the launch is bounded by it)
    int* out;
    int outc;          // counter index of out's length
    bool rev = false;  // list is filled from the back (the tiny short paths)
    static constexpr bool kBlockTake = true;
    template <class T>
    DOFS_HD void operator()(int f, int64_t jj, bool valid, T& t) const {
        int j = 0;
        const bool park = valid && advance(f, jj, &j);
        if (out) {
            const int s = t.take(w.C(f) + outc, park);
            if (park) out[f * w.d.N + s] = j;
        }
    }
    DOFS_HD bool advance(int f, int64_t jj, int* jo) const {  // true: parked
        const Dims& d = w.d;
        const int j = list[f * d.N + (rev ? d.N - 1 - jj : jj)];
        *jo = j;
        int* curp = w.cur + f * d.N + j;
        int q = *curp;
        if (q < 0) return false;
        const int64_t lb = f * d.NL;
        RunState s;
        path_start(w, f, q + 1, &s.mx, &s.my, &s.rank, &s.root, &s.bb);
        for (;;) {
            const StepV in = step_v(w.In[lb + q], q, d.W);
            float wbx = in.wbx, wby = in.wby;
            int lrank = 0, lroot = in.lb;
            B4 lbb;
            if (in.meta & kStepDyn) {
                const int lq = in.lb;
                if (*state_at(w, lb + lq) >= phase) {
                    *curp = q;
                    return true;
                }
                const RepVal lv = w.Rv[lb + lq];
                wbx = lv.mx * (float)in.la;
                wby = lv.my * (float)in.la;
                lrank = lv.rank;
                lroot = lv.root;
                lbb = lv.bb;
            } else {
                lbb.x0 = lbb.x1 = (int16_t)(in.la & 0xffff);
                lbb.y0 = lbb.y1 = (int16_t)(in.la >> 16);
            }
            step_merge(s, in.fs, wbx, wby, in.r, in.meta, lrank, lroot, lbb);
            RepVal o;
            o.mx = s.mx;
            o.my = s.my;
            o.rank = s.rank;
            o.root = s.root;
            o.bb = s.bb;
            o.pad0 = o.pad1 = 0;
            w.Rv[lb + q] = o;
            if (in.meta & kStepTop) {
                *state_at(w, lb + q) = phase;
                *curp = -1;
                return false;
            }
            --q;
        }
    }
};

// State of merge node x after its merge: replay outputs (by preorder position) + size/bbox (KRT).
DOFS_HD inline NodeVal node_val(const Ws& w, const int* pre, int f, int64_t x) {
    const Dims& d = w.d;
    const int64_t lb = f * d.NL;
    const int q = pre[lb + x];
    NodeVal v;
    const RepVal r = w.Rv[lb + q];
    v.mx = r.mx;
    v.my = r.my;
    v.rank = r.rank;
    v.root = r.root;
    v.size = w.SZ[lb + x];
    const B4 b = r.bb;
    v.x0 = b.x0;
    v.y0 = b.y0;
    v.x1 = b.x1;
    v.y1 = b.y1;
    v.pad = 0;
    return v;
}

// ---------------------------------------------------------------------------------------------
// K6 — new_merge filters + lifting (graph.cpp:280-356) and the per-slot arg-max.
// ---------------------------------------------------------------------------------------------
DOFS_HD inline double vec_norm(float x, float y) {  // cv::norm(Vec2f)
    double s = 0.0;
    s += (double)x * (double)x;
    s += (double)y * (double)y;
    return sqrt(s);
}

struct KFilter {  // appends candidates through the backend's list taker (called by every lane)
    Ws w;
    const int* pre;
    static constexpr bool kBlockTake = true;
    template <class T>
    DOFS_HD void operator()(int f, int64_t i, bool valid, T& t) const {
        const Dims& d = w.d;
        bool c = false;
        // the size test first (a coalesced read): most merges are small, and only the others read
        // their replay record (a random 32-B gather by preorder position)
        if (valid && i < w.mreal && w.SZ[f * d.NL + d.N + i] >= w.min_size) {
            const NodeVal v = node_val(w, pre, f, d.N + i);
            const int y = v.root / d.W;
            c = root_ok(w, v.root) && v.size >= w.min_size && y >= d.H / 10 &&
                !(vec_norm(v.mx, v.my) < 3 * (y + 1) / (double)d.H);
        }
        const int k = t.take(w.C(f) + C_CAND, c);
        if (c) w.cand[f * d.M + k] = (int)i;
    }
};

DOFS_HD inline double event_score(const Ws& w, const NodeVal& v, int* cls, dofs_solution* best) {
    const int box[4] = {v.x0, v.y0, v.x1, v.y1};
    return score_event(mk(v.mx, v.my), box, w.L, cls, best);
}

struct KLift {
    Ws w;
    const int* pre;
    static constexpr bool kBlockTake = true;
    template <class T>
    DOFS_HD void operator()(int f, int64_t j, bool valid, T& t) const {
        const Dims& d = w.d;
        // no early return: every lane reaches the counters and the keyed max, which aggregates a
        // wave's lanes of one slot (a frame's largest cluster root takes most of its candidate events)
        bool scored = false, qual = false;
        int root = 0, merge = -1;
        double score = -1.0;
        if (valid && j < w.C(f)[C_CAND]) {
            const int i = w.cand[f * d.M + j];
            merge = i;
            const NodeVal v = node_val(w, pre, f, d.N + i);
            const double rect_area = (double)((v.x1 - v.x0 + 1) * (v.y1 - v.y0 + 1));
            const double convexity = v.size / rect_area;
            int cls;
            score = event_score(w, v, &cls, nullptr);
            root = v.root;
            scored = score != -1;
            if (!root_ok(w, root)) {  // (KFilter admitted it: a record rewritten since is refused, not used)
                root = 0;
                scored = false;
            }
            qual = scored && !(convexity < w.min_convexity[cls]) && score > w.score_threshold;
            w.cscore[f * d.M + j] = qual ? score : -1.0;
        }
        int unused[3];
        t.take3(w.C(f) + C_SCORED, scored, w.C(f) + C_QUAL, qual, nullptr, false, unused, unused + 1, unused + 2);
        dofs_agg_max_u64(w.sbest + f * d.N, root, dbits(score), qual);
        // segment_scores[root] = score for every scored candidate (graph.cpp:326): the latest merge wins
        dofs_agg_max(w.slast + f * d.N, root, merge, scored);
    }
};

struct KSlotInit {
    Ws w;
    DOFS_HD void operator()(int f, int64_t s) const {
        w.sbest[f * w.d.N + s] = 0ull;
        w.sevent[f * w.d.N + s] = kIntMax;
        w.slast[f * w.d.N + s] = -1;
    }
};

struct KSlotEvent {  // first event reaching the slot's maximum wins (strict '<' update, graph.cpp:352)
    Ws w;
    const int* pre;
    static constexpr bool kBlockTake = true;  // (takes nothing: the list launch's form, bounded by C_CAND)
    template <class T>
    DOFS_HD void operator()(int f, int64_t j, bool valid, T&) const {
        const Dims& d = w.d;
        if (!valid || j >= w.C(f)[C_CAND]) return;
        const double s = w.cscore[f * d.M + j];
        if (!(s > w.score_threshold)) return;
        const int i = w.cand[f * d.M + j];
        const int root = w.Rv[f * d.NL + pre[f * d.NL + d.N + i]].root;
        if (!root_ok(w, root)) return;
        if (dbits(s) == w.sbest[f * d.N + root]) dofs_amin(w.sevent + f * d.N + root, i);
    }
};

struct KSlotFlag {
    Ws w;
    DOFS_HD void operator()(int f, int64_t s) const {
        w.sflag[f * w.d.N + s] = w.sevent[f * w.d.N + s] != kIntMax ? 1 : 0;
    }
};

struct KSnapshot {
    Ws w;
    const int* pre;
    DOFS_HD void operator()(int f, int64_t s) const {
        const Dims& d = w.d;
        const int i = w.sevent[f * d.N + s];
        if (i == kIntMax) return;
        const int k = w.soff[f * d.N + s];
        if (k >= w.snap_cap) return;
        const NodeVal v = node_val(w, pre, f, d.N + i);
        dofs_snapshot sn;
        int cls;
        sn.score = event_score(w, v, &cls, &sn.sol);
        sn.slot = (int)s;
        sn.event = i;
        sn.size = v.size;
        sn.seg_begin = w.lscan[f * d.NL + pre[f * d.NL + d.N + i]];
        sn.bbox[0] = v.x0;
        sn.bbox[1] = v.y0;
        sn.bbox[2] = v.x1;
        sn.bbox[3] = v.y1;
        sn.move = vec_norm(v.mx, v.my);
        w.snaps[(int64_t)f * w.snap_cap + k] = sn;
        dofs_box_record rec;
        rec.frame = f;
        rec.slot = (int)s;
        rec.cls = sn.sol.cls;
        rec.size = v.size;
        rec.score = sn.score;
        rec.move = sn.move;
        for (int t = 0; t < 4; ++t) {
            rec.lower_face[t][0] = sn.sol.lower_face[t][0];
            rec.lower_face[t][1] = sn.sol.lower_face[t][1];
            rec.upper_face[t][0] = sn.sol.upper_face[t][0];
            rec.upper_face[t][1] = sn.sol.upper_face[t][1];
        }
        w.recs[(int64_t)f * w.snap_cap + k] = rec;
    }
};

// Forest::get_segment_best_score (graph.cpp:386-389) of every slot of frame f, on demand: the score of
// the slot's last scored candidate, recomputed from its merge's replay record by the scoring function
// KLift used (same operations, same result); 0.0, segment_scores' initial value (graph.cpp:139), where
// the slot never had one.
struct KSegScores {
    Ws w;
    const int* pre;
    int frame;
    double* out;
    DOFS_HD void operator()(int, int64_t s) const {
        const int i = w.slast[frame * w.d.N + s];
        double v = 0.0;
        if (i >= 0) {
            int cls;
            v = event_score(w, node_val(w, pre, frame, w.d.N + i), &cls, nullptr);
        }
        out[s] = v;
    }
};

// The final union-find roots of frame f's run and their boxes — Forest::get_bounding_box after the loop
// (graph.cpp:446-452): merge clears the non-root side's box (:208), so only the roots of the components
// left by the caller's merges keep one. Those components are the children of the completion merges
// mreal .. M-1 (dofs_pipeline run_a_edges: merge mreal + j joins the chain of components 0..j with
// component j + 1), written to out[5 * slot] = {root, xmin, ymin, xmax, ymax}: completion merge 0 fills
// slots 0 and 1, merge j >= 1 slot j + 1 (its other child is the chain). One thread per completion merge.
struct KFinalRoots {
    Ws w;
    const int* pre;
    int frame;
    int* out;
    DOFS_HD void operator()(int, int64_t j) const {
        const Dims& d = w.d;
        const int64_t k = w.mreal + j;
        const int c[2] = {w.lu[frame * d.M + k], w.lv[frame * d.M + k]};
        int slot = j == 0 ? 0 : (int)j + 1;
        for (int t = 0; t < 2; ++t) {
            if (c[t] >= d.N + w.mreal) continue;  // the chain of the earlier completion merges
            int* o = out + 5 * slot;
            if (c[t] < d.N) {  // a pixel no caller edge joined: its own box
                o[0] = c[t];
                o[1] = o[3] = c[t] % d.W;
                o[2] = o[4] = c[t] / d.W;
            } else {
                const RepVal r = w.Rv[frame * d.NL + pre[frame * d.NL + c[t]]];
                root_ok(w, r.root);  // (an output, not an index here: reported through the batch's error)
                o[0] = r.root;
                o[1] = r.bb.x0;
                o[2] = r.bb.y0;
                o[3] = r.bb.x1;
                o[4] = r.bb.y1;
            }
            ++slot;
        }
    }
};

struct KSnapCount {
    Ws w;
    DOFS_HD void operator()(int f, int64_t) const {
        const Dims& d = w.d;
        const int64_t last = f * d.N + d.N - 1;
        const int n = w.soff[last] + w.sflag[last];
        w.C(f)[C_SNAP] = n;
        if (n > w.snap_cap) {  // records beyond the capacity are not written: reported, never silent
            w.C(f)[C_OVF] = n;
            dofs_st(w.C(0) + C_OVF_ANY, 1);
        }
    }
};

struct KSingle {  // H*W == 1: one leaf, no merge (segment_graph performs no union)
    Ws w;
    DOFS_HD void operator()(int f, int64_t) const {
        w.leaf_order[f * w.d.N] = 0;
        w.labels[f * w.d.N] = -1;
        w.C(f)[C_SNAP] = 0;
        w.recs[(int64_t)f * w.snap_cap].slot = -1;
    }
};

struct KRecClear {
    Ws w;
    DOFS_HD void operator()(int f, int64_t k) const { w.recs[(int64_t)f * w.snap_cap + k].slot = -1; }
};

// ---------------------------------------------------------------------------------------------
// K7 — overlay labels (draw.cpp:118-147): max slot over painting snapshots containing the pixel,
// via a segment tree over leaf-order positions (snapshot = contiguous leaf range).
// ---------------------------------------------------------------------------------------------
struct KSegInit {
    Ws w;
    DOFS_HD void operator()(int f, int64_t t) const { w.seg[f * 2 * w.d.P2 + t] = -1; }
};

// One lane per history slot (not per compacted snapshot record), so the labels stay exact whatever
// the snapshot-record capacity: a slot with a winning event paints its member range if its score
// (the slot's arg-max score bits, KLift) exceeds the overlay threshold.
struct KPaint {
    Ws w;
    const int* pre;
    DOFS_HD void operator()(int f, int64_t s) const {
        const Dims& d = w.d;
        const int i = w.sevent[f * d.N + s];
        if (i == kIntMax) return;
        if (!(bitsd(w.sbest[f * d.N + s]) > w.overlay_min_score)) return;
        const int64_t x = d.N + i;
        const int begin = w.lscan[f * d.NL + pre[f * d.NL + x]];
        const int size = w.SZ[f * d.NL + x];
        int* seg = w.seg + f * 2 * d.P2;
        int64_t l = begin + d.P2, r = (int64_t)begin + size + d.P2;
        while (l < r) {
            if (l & 1) dofs_amax(seg + l++, (int)s);
            if (r & 1) dofs_amax(seg + --r, (int)s);
            l >>= 1;
            r >>= 1;
        }
    }
};

struct KLabel {
    Ws w;
    DOFS_HD void operator()(int f, int64_t q) const {
        const Dims& d = w.d;
        const int* seg = w.seg + f * 2 * d.P2;
        // the leaf-to-root walk's addresses are known up front: eight levels' loads per round are
        // issued together (levels above the root read the root again, which the walk visits anyway)
        int lab = -1;
        for (int64_t t = q + d.P2; t >= 1; t >>= 8) {
            int v[8];
            DOFS_UNROLL
            for (int k = 0; k < 8; ++k) v[k] = seg[(t >> k) >= 1 ? (t >> k) : 1];
            DOFS_UNROLL
            for (int k = 0; k < 8; ++k) lab = v[k] > lab ? v[k] : lab;
        }
        w.labels[f * d.N + w.leaf_order[f * d.N + q]] = lab;
    }
};

}  // namespace dofs
