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
// Measured (tools/sortfix_stats.py, 16 synthetic 1080p frames, 33M MST edges): cut 24 → 343k mixed
// groups of at most 7 pairs; cut 32 → 3.4M groups of at most 47; cut 16 → 1.4k groups of 2.
//
// k_sortfix_local, one lane per position p, no atomics, no lists:
//   - the lane at a group's first position owns the group: it scans forward (at most kFixScan
//     positions) and, if the group is short and mixed, insertion-sorts it in place by (key, value).
//     Only the owner writes a group, and the truncated keys every other lane reads never change
//     under a permutation inside the group, so the pass needs no second kernel;
//   - a lane at a mixed pair (p - 1, p) checks that its group starts within kFixScan positions. A
//     longer mixed group (never seen: long groups are exact ties, e.g. zero weights) raises the
//     fallback flag, and k_sortfix_merge — launched ceil_log2(n) times rounded up to an even count,
//     each launch returning at once when the flag is clear — merge-sorts the whole batch by (key,
//     value): slower, never wrong.
#pragma once
// (included inside namespace dofs by dofs_hip.hip)

constexpr int kSortCut = 24;   // low key bits the batch radix sort leaves to the fix-up
constexpr int kFixScan = 256;  // longest group the local pass sorts (longer mixed: the fallback)
constexpr int kFixBlock = 256;
inline int g_sort_cut = kSortCut;  // host: the cut of the next batch sorts (dofs_debug_sort_cut)
inline bool g_sort_fix = true;     // host: run the fix-up (off: the truncated order, for diagnosis only)
inline void* g_sort_dump[2] = {nullptr, nullptr};  // host: device buffers for the next batch's sorted pairs
inline int64_t g_sort_dump_cap = 0;

struct SortFix {
    unsigned long long* key;  // sorted keys (key_out), permuted in place
    unsigned* val;            // their values (the packed sort's middle buffer)
    unsigned long long* k2;   // free buffers of the same sizes (key_in / val_in): the fallback's
    unsigned* v2;
    int* ctr;  // frame 0's C_SORTFIX counters: [0] groups sorted by the local pass, [1] fallback flag
    int64_t n;
    int cut;
};

__device__ inline bool fix_less(unsigned long long ka, unsigned va, unsigned long long kb, unsigned vb) {
    return ka < kb || (ka == kb && va < vb);
}

__global__ __launch_bounds__(kFixBlock) void k_sortfix_local(SortFix s) {
    const int64_t step = (int64_t)gridDim.x * kFixBlock;
    int sorted = 0;
    for (int64_t p = (int64_t)blockIdx.x * kFixBlock + threadIdx.x; p < s.n; p += step) {
        const unsigned long long b = s.key[p];
        const unsigned long long T = b >> s.cut;
        if (b >> 63) dofs_st(s.ctr + 1, 1);  // a negative weight (NaN flow): the sort kept bits [cut, 63)
        bool head = true;
        if (p >= 1) {
            const unsigned long long a = s.key[p - 1];
            head = (a >> s.cut) != T;
            if (!head && a != b) {  // a mixed pair: its group must start within kFixScan positions
                int64_t q = p - 1;
                while (q >= 1 && p - q < kFixScan && (s.key[q - 1] >> s.cut) == T) --q;
                if (q >= 1 && (s.key[q - 1] >> s.cut) == T) dofs_st(s.ctr + 1, 1);
            }
        }
        if (!head) continue;
        int64_t e = p + 1;  // the group [p, e)
        bool mixed = false;
        unsigned long long prev = b;
        while (e < s.n && e - p < kFixScan) {
            const unsigned long long k = s.key[e];
            if ((k >> s.cut) != T) break;
            mixed |= k != prev;
            prev = k;
            ++e;
        }
        if (!mixed) continue;  // exact ties (or a long group's first kFixScan: its mixed pairs further on flag)
        if (e < s.n && (s.key[e] >> s.cut) == T) {  // longer than kFixScan and mixed: the fallback
            dofs_st(s.ctr + 1, 1);
            continue;
        }
        ++sorted;
        for (int64_t i = p + 1; i < e; ++i) {  // insertion sort by (key, value), in place
            const unsigned long long k = s.key[i];
            const unsigned v = s.val[i];
            int64_t j = i;
            while (j > p && fix_less(k, v, s.key[j - 1], s.val[j - 1])) {
                s.key[j] = s.key[j - 1];
                s.val[j] = s.val[j - 1];
                --j;
            }
            s.key[j] = k;
            s.val[j] = v;
        }
    }
    const int tot = wave_reduce(sorted, [](int x, int y) { return x + y; });
    if (tot && wave_lane() == 0) dofs_aadd(s.ctr, tot);
}

// fallback, pass `lg`: merges runs of 2^lg pairs from (ka, va) into (kb, vb); nothing when the flag
// is clear. Each pair's destination = its offset in its run + the partner run's pairs below it.
__global__ __launch_bounds__(kFixBlock) void k_sortfix_merge(SortFix s, int lg, int odd) {
    if (!dofs_ld(s.ctr + 1)) return;
    const unsigned long long* ka = odd ? s.k2 : s.key;
    const unsigned* va = odd ? s.v2 : s.val;
    unsigned long long* kb = odd ? s.key : s.k2;
    unsigned* vb = odd ? s.val : s.v2;
    const int64_t W = (int64_t)1 << lg;
    const int64_t step = (int64_t)gridDim.x * kFixBlock;
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
            if (fix_less(ka[m], va[m], k, v))
                lo = m + 1;
            else
                hi = m;
        }
        const int64_t d = a0 + off + (lo - l0);
        kb[d] = k;
        vb[d] = v;
    }
}
