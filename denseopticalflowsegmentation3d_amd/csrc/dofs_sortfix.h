// dofs_sortfix.h — the batch's MST edge sort on truncated keys, and the fix-up that makes it exact.
//
// Kruskal's order (segment.cpp:68 sorts the edges by weight, stably) is the order of the 64-bit key
// dbits(weight) with the emission value as tie-break. The batch sort (HipBackend::sort_mst) orders the
// pairs by key bits [cut, 63) only (cut = 24: 5 radix digits instead of 8; bit 63, the sign, is 0 for
// every weight — a set one raises the fallback below), stably, so the
// emission order already breaks ties among equal truncated keys. The result is exact except inside a
// "mixed group": a maximal run of equal truncated keys holding two different full keys (weights within
// 2^-28 relative of each other). Sorting every mixed group by (key, value) — all pairs are distinct:
// the value carries frame and emission index — gives the full-key stable order.
//
// Measured (tools/sortfix_stats.py, synthetic 1080p frames): 16 frames (33M MST edges): cut 24 → 343k
// mixed groups of at most 7 pairs, cut 32 → 3.4M of at most 47, cut 16 → 1.4k of 2; 112 frames (232M):
// cut 24 → 14.4M mixed groups (the batch's frames share weight values), cut 32 → groups beyond kFixScan.
//
// k_sortfix_local (no atomics but one per wave, no lists): a group inside a wave's 64 positions with at
// most kFixWin of them is ranked by (key, value) in registers and scattered; a longer or wave-crossing
// group is insertion-sorted in place by the lane at its first position (at most kFixScan positions).
// Only a group's sorter writes it, and the truncated keys every other lane reads never change under
// a permutation inside a group, so one pass suffices. A mixed group longer than kFixScan (never seen:
// long groups are exact ties, e.g. zero weights) or a negative key raises the fallback flag, and
// k_sortfix_merge — one launch that returns at once when the flag is clear — merge-sorts the whole
// batch by (key, value): slower, never wrong.
#pragma once
// (included inside namespace dofs by dofs_hip.hip)

constexpr int kSortCut = 24;   // low key bits the batch radix sort leaves to the fix-up
constexpr int kFixScan = 256;  // longest group the local pass sorts (longer mixed: the fallback)
constexpr int kFixBlock = 256;
constexpr int kFixWin = 16;    // longest group the wave ranks in registers (longer or wave-crossing: scalar)
inline int g_sort_cut = kSortCut;  // host: the cut of the next batch sorts (dofs_debug_sort_cut)
inline bool g_sort_fix = true;     // host: run the fix-up (off: the truncated order, for diagnosis only)
inline void* g_sort_dump[2] = {nullptr, nullptr};  // host: device buffers for the next batch's sorted pairs
inline int64_t g_sort_dump_cap = 0;

struct SortFix {
    unsigned long long* key;  // sorted keys (key_out), permuted in place
    unsigned* val;            // their values (the packed sort's middle buffer)
    unsigned long long* k2;   // free buffers of the same sizes (key_in / val_in): the fallback's
    unsigned* v2;
    int* ctr;  // frame 0's C_SORTFIX counters: [0] pairs the local pass moved, [1] fallback flag,
               // [2] the fallback's grid barrier
    int64_t n;
    int cut;
    unsigned vm;  // the frame and index bits of a value: below the singleton flags when Ws::single, else all
                  // 32 (a batch with vb + fb > 30 has frame bits in 30-31, and they keep the pairs distinct)
};

// values compare on their frame and emission index bits only (vm): with Ws::single the two top bits are the
// KRT sweep's singleton flags (dofs_kernels.h kValSingle*), not part of the pair's identity
__device__ inline bool fix_less(unsigned long long ka, unsigned va, unsigned long long kb, unsigned vb, unsigned vm) {
    return ka < kb || (ka == kb && (va & vm) < (vb & vm));
}

// the scalar path of one group [p, ...) from its first position: at most kFixScan positions, in place
__device__ inline int fix_group_scalar(const SortFix& s, int64_t p, unsigned long long b) {
    const unsigned long long T = b >> s.cut;
    int64_t e = p + 1;
    bool mixed = false;
    unsigned long long prev = b;
    while (e < s.n && e - p < kFixScan) {
        const unsigned long long k = s.key[e];
        if ((k >> s.cut) != T) break;
        mixed |= k != prev;
        prev = k;
        ++e;
    }
    if (!mixed) return 0;  // exact ties (or a long group's first kFixScan: its mixed pairs further on flag)
    if (e < s.n && (s.key[e] >> s.cut) == T) {  // longer than kFixScan and mixed: the fallback
        dofs_st(s.ctr + 1, 1);
        return 0;
    }
    int moved = 0;
    for (int64_t i = p + 1; i < e; ++i) {  // insertion sort by (key, value)
        const unsigned long long k = s.key[i];
        const unsigned v = s.val[i];
        int64_t j = i;
        while (j > p && fix_less(k, v, s.key[j - 1], s.val[j - 1], s.vm)) {
            s.key[j] = s.key[j - 1];
            s.val[j] = s.val[j - 1];
            --j;
        }
        if (j != i) {
            s.key[j] = k;
            s.val[j] = v;
            moved += (int)(i - j) + 1;
        }
    }
    return moved;
}

// One wave per 64 consecutive positions (grid-stride). A group that lies inside the wave with at most
// kFixWin positions is ranked in registers: rank = the group's pairs below this lane's (key, value),
// read by cross-lane shuffles, then one scatter store per moved pair (every lane read before any
// writes). A group that crosses the wave's ends or is longer takes the scalar path from its first
// position (the lane holding it, or the earlier wave's); its other lanes only check, at a mixed pair,
// that the group starts within kFixScan positions (else the fallback flag).
__global__ __launch_bounds__(kFixBlock) void k_sortfix_local(SortFix s) {
    const int lane = wave_lane();
    const int64_t nw = (int64_t)gridDim.x * (kFixBlock / 64);
    int moved = 0;
    for (int64_t wv = (int64_t)blockIdx.x * (kFixBlock / 64) + threadIdx.x / 64; wv * 64 < s.n; wv += nw) {
        const int64_t base = wv * 64, p = base + lane;
        const bool valid = p < s.n;
        const unsigned long long b = valid ? s.key[p] : 0ull;
        const unsigned long long T = b >> s.cut;
        if (valid && (b >> 63)) dofs_st(s.ctr + 1, 1);  // a negative weight (NaN flow): bits [cut, 63) sorted
        unsigned long long a = __shfl_up(b, 1, 64), c = __shfl_down(b, 1, 64);
        if (lane == 0 && valid && p >= 1) a = s.key[p - 1];
        if (lane == 63 && p + 1 < s.n) c = s.key[p + 1];
        const bool same_prev = valid && p >= 1 && (a >> s.cut) == T;
        const bool same_next = valid && p + 1 < s.n && (c >> s.cut) == T;
        const unsigned long long mix = __ballot(same_prev && a != b);  // mixed pairs (lane - 1, lane)
        const bool tail_open = __shfl(same_next ? 1 : 0, 63, 64) != 0;  // a group runs into the next wave
        if (!mix && !tail_open) continue;  // no mixed group here (one that began earlier: its first lane's)
        // this lane's group inside the wave: lanes [gs, ge); open at either end if it continues there
        const unsigned long long heads = __ballot(!same_prev);
        const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;
        const unsigned long long below = heads & upto, above = heads & ~upto;
        const bool left_open = below == 0;
        const int gs = left_open ? 0 : 63 - __clzll(below);
        const int ge = above ? __ffsll((long long)above) - 1 : 64;
        const bool right_open = above == 0 && tail_open;
        const int g = ge - gs;
        const unsigned long long gmask = (ge == 64 ? ~0ull : (1ull << ge) - 1ull) & ~((1ull << gs) - 1ull);
        const bool fast = valid && !left_open && !right_open && g >= 2 && g <= kFixWin && (mix & gmask);
        const unsigned v = fast ? s.val[p] : 0u;
        const int gmax = wave_reduce(fast ? g : 0, [](int x, int y) { return x > y ? x : y; });
        if (gmax) {
            int rank = 0;
            for (int d = 0; d < gmax; ++d) {
                const int j = (gs + d) & 63;
                const unsigned long long kj = __shfl(b, j, 64);
                const unsigned vj = __shfl(v, j, 64);
                rank += (fast && d < g && j != lane && fix_less(kj, vj, b, v, s.vm)) ? 1 : 0;
            }
            if (fast && gs + rank != lane) {
                s.key[base + gs + rank] = b;
                s.val[base + gs + rank] = v;
                ++moved;
            }
        }
        if (!valid || fast || (!left_open && !right_open && !(mix & gmask))) continue;  // done, or exact ties
        if (!same_prev) {
            moved += fix_group_scalar(s, p, b);  // the group's first position: the scalar path
        } else if (a != b) {
            // a mixed pair (p - 1, p) of a scalar-path group: its sorter covers [start, start + kFixScan),
            // so the pair is sorted only if p - start < kFixScan. Groups are contiguous runs, so
            // p - start >= kFixScan exactly when position p - kFixScan is still in the group: the fallback.
            if (p >= kFixScan && (s.key[p - kFixScan] >> s.cut) == T) dofs_st(s.ctr + 1, 1);
        }
    }
    const int tot = wave_reduce(moved, [](int x, int y) { return x + y; });
    if (tot && lane == 0) dofs_aadd(s.ctr, tot);
}

// fallback: merge passes lg = 0 .. lgs - 1 (runs of 2^lg pairs, ping-pong between (key, val) and (k2, v2);
// lgs even, so the result ends in (key, val)), one launch, a grid barrier between passes; returns at
// once when the flag is clear. A pair's destination = its offset in its run + the partner run's pairs
// below it (all pairs distinct). The barrier counts arrivals on ctr[2] (zero at the batch's start):
// every block's stores are complete at __syncthreads, lane 0 releases them with the agent fence,
// arrives, waits for the pass's full count, and acquires with the same fence.
__global__ __launch_bounds__(kFixBlock) void k_sortfix_merge(SortFix s, int lgs) {
    if (!dofs_ld(s.ctr + 1)) return;
    const int64_t step = (int64_t)gridDim.x * kFixBlock;
    for (int lg = 0; lg < lgs; ++lg) {
        const bool odd = lg & 1;
        const unsigned long long* ka = odd ? s.k2 : s.key;
        const unsigned* va = odd ? s.v2 : s.val;
        unsigned long long* kb = odd ? s.key : s.k2;
        unsigned* vb = odd ? s.val : s.v2;
        const int64_t W = (int64_t)1 << lg;
        for (int64_t p = (int64_t)blockIdx.x * kFixBlock + threadIdx.x; p < s.n; p += step) {
            const unsigned long long k = ka[p];
            const unsigned v = va[p];
            const int64_t a0 = p & ~(2 * W - 1), mid = a0 + W;
            int64_t lo, hi, off;
            if (p < mid) {  // left run: partner [mid, a0 + 2W)
                lo = mid < s.n ? mid : s.n;
                hi = a0 + 2 * W < s.n ? a0 + 2 * W : s.n;
                off = p - a0;
            } else {
                lo = a0;
                hi = mid;
                off = p - mid;
            }
            const int64_t l0 = lo;
            while (lo < hi) {  // partner pairs below (k, v)
                const int64_t m = lo + (hi - lo) / 2;
                if (fix_less(ka[m], va[m], k, v, s.vm))
                    lo = m + 1;
                else
                    hi = m;
            }
            const int64_t d = a0 + off + (lo - l0);
            kb[d] = k;
            vb[d] = v;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            dofs_aadd(s.ctr + 2, 1);
            while (dofs_ld(s.ctr + 2) < (lg + 1) * (int)gridDim.x) __builtin_amdgcn_s_sleep(4);
            __threadfence();
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// The default batch sort: 32-bit keys (key32_of, dofs_kernels.h) — a window of 2^(32 - m) binades below
// the frame's weight bound (from its largest blurred component, C_BMAX) with m = 27 mantissa bits, the
// precision of cut 24 in half the key bytes: four 8-bit digits of (u32 key, u32 value) pairs instead of
// five of (u64, u32). key32_of is monotone, so the stable pair sort is exact except inside mixed groups
// (equal 32-bit keys, different weights), which the fix-up below sorts by (full key, value) as above.
// The full keys are not stored: a pair's weight is recomputed from its value (frame, pixel p, edge slot
// k) and the blurred field, by the expression KMstEmit used (edge_weight), for the tied positions only.
// A group's 32-bit keys are equal, so only values move. Weights below the window (zero included) share
// key 0 and weights above it (none for finite flows) the largest key: a long mixed group there takes
// the fallback — slower, never wrong.
// host: mantissa bits of the 32-bit keys (0: the 64-bit keys and g_sort_cut); dofs_debug_sort_k32 sets it
// (tests/test_gpu_sortfix.py)
inline int g_sort_k32 = 27;
// host: exponent bits of the 32-bit keys (0: 32 - m, the full word). With m + e = 24 the pair sort takes
// three 8-bit digits instead of four; dofs_debug_sort_k32e sets it (measured slower: DESIGN.md §8)
inline int g_sort_k32e = 0;
inline int sort_k32_bits() { return g_sort_k32e && g_sort_k32 + g_sort_k32e < 32 ? g_sort_k32 + g_sort_k32e : 32; }

struct SortFix32 {
    const unsigned* key;      // sorted 32-bit keys (key_out's first half; never permuted)
    unsigned* val;            // their values (the packed sort's middle buffer), permuted in place
    unsigned long long* k64;  // the fallback's full keys (key_out's storage, 8 bytes per pair)
    unsigned long long* k2;   // scratch (key_in's storage): the scalar path's keys, the fallback's ping-pong
    unsigned* v2;
    const F2* blur;  // the batch's blurred fields (frame stride d.N)
    Dims d;
    int vb;       // value bits: the frame id above, the emission index 4 p + k below
    unsigned vm;  // the frame and index bits of a value (below the singleton flags when Ws::single)
    int* ctr;     // as SortFix::ctr
    int64_t n;
};

// A group is a run of equal 32-bit keys of one frame: the pair sort is stable and its input frame-major, so
// a run of equal keys holds each frame's pairs contiguously, and only the order within a frame matters
// (the frame pass that follows separates the frames stably). Most ties of a 112-frame batch are across
// frames (the frames share weight values) and need no full key.
__device__ inline unsigned fix_frame(const SortFix32& s, unsigned v) { return (v & s.vm) >> s.vb; }

// the full 64-bit key of a value (KMstEmit's weight of the MST edge (p, slot k) of its frame)
__device__ inline unsigned long long fix_full(const SortFix32& s, unsigned v) {
    v &= s.vm;
    const int64_t f = v >> s.vb;
    const unsigned idx = v & ((1u << s.vb) - 1u);
    const int64_t p = idx >> 2;
    return dbits(edge_weight(s.blur + f * s.d.N, p, edge_end(s.d, p, (int)(idx & 3))));
}

// the scalar path of one tied group [p, ...) whose first full key is b: its full keys go to k2 (the group's
// range only), then an insertion sort of (k2, val) — at most kFixScan positions, in place
__device__ inline int fix32_group_scalar(const SortFix32& s, int64_t p, unsigned T, unsigned F, unsigned long long b) {
    int64_t e = p + 1;
    bool mixed = false;
    s.k2[p] = b;
    while (e < s.n && e - p < kFixScan) {
        const unsigned ve = s.val[e];
        if (s.key[e] != T || fix_frame(s, ve) != F) break;
        const unsigned long long k = fix_full(s, ve);
        s.k2[e] = k;
        mixed |= k != b;
        ++e;
    }
    if (!mixed) return 0;  // exact ties (or a long group's first kFixScan: its mixed pairs further on flag)
    if (e < s.n && s.key[e] == T && fix_frame(s, s.val[e]) == F) {  // longer than kFixScan and mixed: the fallback
        dofs_st(s.ctr + 1, 1);
        return 0;
    }
    int moved = 0;
    for (int64_t i = p + 1; i < e; ++i) {
        const unsigned long long k = s.k2[i];
        const unsigned v = s.val[i];
        int64_t j = i;
        while (j > p && fix_less(k, v, s.k2[j - 1], s.val[j - 1], s.vm)) {
            s.k2[j] = s.k2[j - 1];
            s.val[j] = s.val[j - 1];
            --j;
        }
        if (j != i) {
            s.k2[j] = k;
            s.val[j] = v;
            moved += (int)(i - j) + 1;
        }
    }
    return moved;
}

// k_sortfix_local on 32-bit keys: groups are runs of equal 32-bit keys; a wave without a tie exits after
// one ballot, and only tied positions recompute their full keys
__global__ __launch_bounds__(kFixBlock) void k_sortfix32_local(SortFix32 s) {
    const int lane = wave_lane();
    const int64_t nw = (int64_t)gridDim.x * (kFixBlock / 64);
    int moved = 0;
    for (int64_t wv = (int64_t)blockIdx.x * (kFixBlock / 64) + threadIdx.x / 64; wv * 64 < s.n; wv += nw) {
        const int64_t base = wv * 64, p = base + lane;
        const bool valid = p < s.n;
        const unsigned T = valid ? s.key[p] : 0u;
        unsigned ta = __shfl_up(T, 1, 64), tc = __shfl_down(T, 1, 64);
        if (lane == 0 && valid && p >= 1) ta = s.key[p - 1];
        if (lane == 63 && p + 1 < s.n) tc = s.key[p + 1];
        if (!__ballot((valid && p >= 1 && ta == T) || (valid && p + 1 < s.n && tc == T))) continue;  // no tie
        // ties of the 32-bit key: a group also needs the same frame
        const unsigned v = valid ? s.val[p] : 0u;
        const unsigned F = fix_frame(s, v);
        unsigned fa = __shfl_up(F, 1, 64), fc = __shfl_down(F, 1, 64);
        if (lane == 0 && valid && p >= 1 && ta == T) fa = fix_frame(s, s.val[p - 1]);
        if (lane == 63 && p + 1 < s.n && tc == T) fc = fix_frame(s, s.val[p + 1]);
        const bool same_prev = valid && p >= 1 && ta == T && fa == F;
        const bool same_next = valid && p + 1 < s.n && tc == T && fc == F;
        if (!__ballot(same_prev || same_next)) continue;  // ties across frames only
        const bool tied = same_prev || same_next;
        const unsigned long long b = tied ? fix_full(s, v) : 0ull;
        unsigned long long a = __shfl_up(b, 1, 64);
        if (lane == 0 && same_prev) a = fix_full(s, s.val[p - 1]);
        const unsigned long long mix = __ballot(same_prev && a != b);  // mixed pairs (lane - 1, lane)
        const bool tail_open = __shfl(same_next ? 1 : 0, 63, 64) != 0;  // a group runs into the next wave
        if (!mix && !tail_open) continue;
        const unsigned long long heads = __ballot(!same_prev);
        const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;
        const unsigned long long below = heads & upto, above = heads & ~upto;
        const bool left_open = below == 0;
        const int gs = left_open ? 0 : 63 - __clzll(below);
        const int ge = above ? __ffsll((long long)above) - 1 : 64;
        const bool right_open = above == 0 && tail_open;
        const int g = ge - gs;
        const unsigned long long gmask = (ge == 64 ? ~0ull : (1ull << ge) - 1ull) & ~((1ull << gs) - 1ull);
        const bool fast = valid && !left_open && !right_open && g >= 2 && g <= kFixWin && (mix & gmask);
        const int gmax = wave_reduce(fast ? g : 0, [](int x, int y) { return x > y ? x : y; });
        if (gmax) {
            int rank = 0;
            for (int dd = 0; dd < gmax; ++dd) {
                const int j = (gs + dd) & 63;
                const unsigned long long kj = __shfl(b, j, 64);
                const unsigned vj = __shfl(v, j, 64);
                rank += (fast && dd < g && j != lane && fix_less(kj, vj, b, v, s.vm)) ? 1 : 0;
            }
            if (fast && gs + rank != lane) {  // the group's keys are equal: only the value moves
                s.val[base + gs + rank] = v;
                ++moved;
            }
        }
        if (!valid || fast || (!left_open && !right_open && !(mix & gmask))) continue;  // done, or exact ties
        if (!same_prev) {
            moved += fix32_group_scalar(s, p, T, F, b);
        } else if (a != b) {  // a mixed pair of a scalar-path group: inside its sorter's window?
            if (p >= kFixScan && s.key[p - kFixScan] == T && fix_frame(s, s.val[p - kFixScan]) == F)
                dofs_st(s.ctr + 1, 1);
        }
    }
    const int tot = wave_reduce(moved, [](int x, int y) { return x + y; });
    if (tot && lane == 0) dofs_aadd(s.ctr, tot);
}

// fallback only (returns at once when the flag is clear): every position's full key into k64, for
// k_sortfix_merge over (k64, val)
__global__ __launch_bounds__(kFixBlock) void k_sortfix32_keys(SortFix32 s) {
    if (!dofs_ld(s.ctr + 1)) return;
    const int64_t step = (int64_t)gridDim.x * kFixBlock;
    for (int64_t p = (int64_t)blockIdx.x * kFixBlock + threadIdx.x; p < s.n; p += step) s.k64[p] = fix_full(s, s.val[p]);
}
