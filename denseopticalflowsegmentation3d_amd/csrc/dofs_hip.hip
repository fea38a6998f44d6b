// dofs_hip.hip — HIP/CDNA4 (gfx950) backend of the dense-optical-flow clustering + 3D-lifting path
// and the exported C-ABI (include/dofs.h). Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off.
//
// Every per-element body in dofs_kernels.h runs here as a grid-stride kernel over a 2-D grid
// (x: elements, y: frames of the batch), 256-thread workgroups (4 wave64s). Atomics are agent-scope
// (coherent across the 8 XCDs); union-find loads inside a launch use relaxed agent-scope atomic loads
// so a stale L1/L2 line can never be re-read forever (MI355X_MICROARCH.md §inter-workgroup visibility).
#include <hip/hip_runtime.h>
#include <type_traits>
#include <utility>
#include <hipcub/hipcub.hpp>

#include <stdlib.h>

#include <algorithm>
#include <array>
#include <string>
#include <vector>

#define DOFS_HD __device__
#define DOFS_HDM __host__ __device__
#define DOFS_UNROLL _Pragma("unroll")

__device__ inline int dofs_ld(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline void dofs_st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline int dofs_cas(int* p, int expected, int v) {
    int old = expected;
    __hip_atomic_compare_exchange_strong(p, &old, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return old;
}
__device__ inline int dofs_exch(int* p, int v) { return atomicExch(p, v); }
__device__ inline unsigned long long dofs_cas64(unsigned long long* p, unsigned long long expected,
                                                unsigned long long v) {
    unsigned long long old = expected;
    __hip_atomic_compare_exchange_strong(p, &old, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return old;
}
__device__ inline unsigned long long dofs_ld64(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void dofs_st64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void dofs_amin_u64(unsigned long long* p, unsigned long long v) { atomicMin(p, v); }
__device__ inline void dofs_amax_u64(unsigned long long* p, unsigned long long v) { atomicMax(p, v); }
__device__ inline void dofs_amin_u32(unsigned* p, unsigned v) { atomicMin(p, v); }
__device__ inline void dofs_amin(int* p, int v) { atomicMin(p, v); }
__device__ inline void dofs_amax(int* p, int v) { atomicMax(p, v); }
__device__ inline int dofs_aadd(int* p, int v) { return atomicAdd(p, v); }
__device__ inline void dofs_aor(int* p, int v) { atomicOr(p, v); }

#include "dofs_common.h"
#include "dofs_knobs.h"

// Keyed atomic updates aggregated across the wave: when all 64 lanes are present, the lanes whose
// key equals the first active lane's key are reduced with cross-lane shuffles and updated by one
// atomic; the other active lanes update directly (min/max read first: monotone, often skipped).
// A big union-find component is the key of most lanes at the top divide-and-conquer levels, so
// this turns ~one atomic per lane on a single address into ~one per wave.
__device__ inline int wave_lane() { return __lane_id(); }
template <class T, class Op>
__device__ inline T wave_reduce(T v, Op op) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = op(v, __shfl_xor(v, m, 64));
    return v;
}
__device__ inline void dofs_amin(int* p, int v);
__device__ inline void dofs_amax(int* p, int v);
__device__ inline int dofs_aadd(int* p, int v);
__device__ inline void dofs_agg_add(int* base, int key, int val, bool act) {
    const unsigned long long present = __ballot(1);
    const unsigned long long on = __ballot(act);
    if (!on) return;
    bool done = false;
    if (present == ~0ull) {
        const int leader = __ffsll((long long)on) - 1;
        const int k0 = __shfl(key, leader, 64);
        const bool same = act && key == k0;
        const int sum = wave_reduce(same ? val : 0, [](int x, int y) { return x + y; });
        if (wave_lane() == leader) atomicAdd(base + k0, sum);
        done = same;
    }
    if (act && !done) atomicAdd(base + key, val);
}
template <bool kMax>
__device__ inline void agg_minmax(int* base, int key, int val, bool act) {
    const unsigned long long present = __ballot(1);
    const unsigned long long on = __ballot(act);
    if (!on) return;
    bool done = false;
    if (present == ~0ull) {
        const int leader = __ffsll((long long)on) - 1;
        const int k0 = __shfl(key, leader, 64);
        const bool same = act && key == k0;
        const int v = kMax ? wave_reduce(same ? val : (int)0x80000000, [](int a, int c) { return a > c ? a : c; })
                           : wave_reduce(same ? val : 0x7fffffff, [](int a, int c) { return a < c ? a : c; });
        if (wave_lane() == leader) {
            const int cur = __hip_atomic_load(base + k0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (kMax ? cur < v : cur > v) kMax ? atomicMax(base + k0, v) : atomicMin(base + k0, v);
        }
        done = same;
    }
    if (act && !done) {
        const int cur = __hip_atomic_load(base + key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (kMax ? cur < val : cur > val) kMax ? atomicMax(base + key, val) : atomicMin(base + key, val);
    }
}
__device__ inline void dofs_agg_max(int* base, int key, int val, bool act) { agg_minmax<true>(base, key, val, act); }
// Keyed u64 max / min where a few keys are very hot (the slot arg-max of KLift: one cluster root
// takes most candidate events of a frame). Up to four distinct keys of the wave are reduced in registers and written with
// one atomic each; an atomic is skipped when the stored value is already at least as good.
template <bool kMax>
__device__ inline void agg_u64(unsigned long long* base, int key, unsigned long long val, bool act) {
    auto better = [](unsigned long long a, unsigned long long c) { return kMax ? a > c : a < c; };
    const unsigned long long present = __ballot(1);
    if (present == ~0ull) {
        unsigned long long on = __ballot(act);
        for (int it = 0; it < 4 && on; ++it) {
            const int leader = __ffsll((long long)on) - 1;
            const int k0 = __shfl(key, leader, 64);
            const bool same = act && key == k0;
            const unsigned long long v = wave_reduce(same ? val : (kMax ? 0ull : ~0ull),
                                                     [&](unsigned long long a, unsigned long long c) {
                                                         return better(a, c) ? a : c;
                                                     });
            if (wave_lane() == leader) {
                const unsigned long long cur = __hip_atomic_load(base + k0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (better(v, cur)) kMax ? atomicMax(base + k0, v) : atomicMin(base + k0, v);
            }
            act = act && !same;
            on = __ballot(act);
        }
    }
    if (act) {
        const unsigned long long cur = __hip_atomic_load(base + key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (better(val, cur)) kMax ? atomicMax(base + key, val) : atomicMin(base + key, val);
    }
}
__device__ inline void dofs_agg_max_u64(unsigned long long* base, int key, unsigned long long val, bool act) {
    agg_u64<true>(base, key, val, act);
}

#include "dofs_kernels.h"

namespace dofs {

constexpr int kBlock = 256;

#ifdef DOFS_MEASURE
// measurement build: one wave that waits `us` microseconds (s_memrealtime: 100 MHz), holding nothing else
__global__ void k_delay(int us) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * (unsigned long long)us) __builtin_amdgcn_s_sleep(127);
}
#endif
template <class F>
__global__ __launch_bounds__(kBlock) void k_generic(F f, int64_t n) {
    const int fr = blockIdx.y;
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += step) f(fr, i);
}

// List appends through a per-frame counter (KPathInit, KFilter, KLift): one global atomic per
// block instead of one per wave — a frame's counter is a single address, and same-address atomics
// serialise at ~60 ns each (tools/counter_micro.hip: 2.0 ms vs 0.56 ms per 32 x 2M appends).
// take() is called by every thread of the block (the loop below is block-uniform).
struct BlockTaker {
    int* wsum;  // LDS: per-wave counts, then per-wave offsets (3 lists x kBlock / 64 words)
    int* base;  // LDS: the block's bases in the lists (3 words)
    // three appends at once (one set of barriers); a null counter is skipped
    __device__ void take3(int* c0, bool w0, int* c1, bool w1, int* c2, bool w2, int* r0, int* r1, int* r2) {
        constexpr int nw = kBlock / 64;
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const unsigned long long m0 = __ballot(w0), m1 = __ballot(w1), m2 = __ballot(w2);
        const unsigned long long below = (1ull << lane) - 1ull;
        if (lane == 0) {
            wsum[wid] = __popcll(m0);
            wsum[nw + wid] = __popcll(m1);
            wsum[2 * nw + wid] = __popcll(m2);
        }
        __syncthreads();
        if (threadIdx.x < 3) {
            int* ws = wsum + threadIdx.x * nw;
            int* c = threadIdx.x == 0 ? c0 : (threadIdx.x == 1 ? c1 : c2);
            int sum = 0;
            for (int k = 0; k < nw; ++k) {
                const int v = ws[k];
                ws[k] = sum;
                sum += v;
            }
            base[threadIdx.x] = (sum && c) ? atomicAdd(c, sum) : 0;
        }
        __syncthreads();
        *r0 = w0 ? base[0] + wsum[wid] + __popcll(m0 & below) : -1;
        *r1 = w1 ? base[1] + wsum[nw + wid] + __popcll(m1 & below) : -1;
        *r2 = w2 ? base[2] + wsum[2 * nw + wid] + __popcll(m2 & below) : -1;
        __syncthreads();
    }
    __device__ int take(int* ctr, bool want) {
        const unsigned long long m = __ballot(want);
        const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int below = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wid] = __popcll(m);
        __syncthreads();
        if (threadIdx.x == 0) {
            int s = 0;
            for (int k = 0; k < kBlock / 64; ++k) {
                const int c = wsum[k];
                wsum[k] = s;
                s += c;
            }
            *base = s ? atomicAdd(ctr, s) : 0;
        }
        __syncthreads();
        const int r = *base + wsum[wid] + below;
        __syncthreads();  // the LDS words are reused by the next take
        return want ? r : -1;
    }
};
template <class F>
__global__ __launch_bounds__(kBlock) void k_generic_take(F f, int64_t n) {
    __shared__ int wsum[3 * kBlock / 64];
    __shared__ int base[3];
    BlockTaker t{wsum, base};
    const int fr = blockIdx.y;
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t i0 = (int64_t)blockIdx.x * kBlock; i0 < n; i0 += step) {
        const int64_t i = i0 + threadIdx.x;
        f(fr, i, i < n, t);
    }
}
// list launch: elements [0, min(n, frame counter cidx)) — the bound is read on the device, so a
// shrinking list costs only the blocks it needs (the others exit at once)
// (at least three waves per SIMD: KLift's lifting needed 169 VGPRs, two waves per SIMD, beside the graph
// stage's sort passes)
#ifndef DOFS_COUNTED_WPE
#define DOFS_COUNTED_WPE 3
#endif
template <class F>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(DOFS_COUNTED_WPE))) void k_counted_take(F f, int64_t n, int cidx,
                                                                                                  int zidx) {
    __shared__ int wsum[3 * kBlock / 64];
    __shared__ int base[3];
    BlockTaker t{wsum, base};
    const int fr = blockIdx.y;
    if (zidx >= 0 && blockIdx.x == 0 && threadIdx.x == 0) f.w.C(fr)[zidx] = 0;  // a counter no block uses here
    const int64_t c = f.w.C(fr)[cidx];
    const int64_t m = c < n ? c : n;
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t i0 = (int64_t)blockIdx.x * kBlock; i0 < m; i0 += step) {
        const int64_t i = i0 + threadIdx.x;
        f(fr, i, i < m, t);
    }
}
template <class F, class = void>
struct takes : std::false_type {};
template <class F>
struct takes<F, std::void_t<decltype(F::kBlockTake)>> : std::true_type {};


// ---------------------------------------------------------------------------------------------
// K5 support: the replay's step records, staged in LDS by the long-path workers (dofs_dataflow.h).
// Rank and root of a running set travel as one key K = rank << 27 | root (H*W < 2^26, rank <= 26): the
// union-by-rank step (step_merge, graph.cpp:177-182, 210-213) becomes K' = max(K, LK) for unequal ranks
// and, for equal ranks, (B ? LK : K) + (1 << 27) — five VALU ops instead of eleven, which matters because
// one wave issues at most one instruction per four cycles and the chain loop is issue-bound.
// ---------------------------------------------------------------------------------------------
constexpr int kLongOk = 8;  // meta flag: the step's inputs are resolved
#ifndef DOFS_SPIN_SLEEP
#define DOFS_SPIN_SLEEP 8  // s_sleep units (64 cycles) between polls of a flag another workgroup sets
#endif

__device__ inline B4 bb_join(B4 a, B4 b) {
    B4 r;
    r.x0 = a.x0 < b.x0 ? a.x0 : b.x0;
    r.y0 = a.y0 < b.y0 ? a.y0 : b.y0;
    r.x1 = a.x1 > b.x1 ? a.x1 : b.x1;
    r.y1 = a.y1 > b.y1 ? a.y1 : b.y1;
    return r;
}
__device__ inline B4 bb_shfl_up(B4 b, int delta) {
    const int lo = __shfl_up((int)((unsigned short)b.x0 | ((unsigned)(unsigned short)b.y0 << 16)), delta, 64);
    const int hi = __shfl_up((int)((unsigned short)b.x1 | ((unsigned)(unsigned short)b.y1 << 16)), delta, 64);
    B4 r;
    r.x0 = (int16_t)(lo & 0xffff);
    r.y0 = (int16_t)(lo >> 16);
    r.x1 = (int16_t)(hi & 0xffff);
    r.y1 = (int16_t)(hi >> 16);
    return r;
}

constexpr int kRankShift = 27;
__device__ inline unsigned rk_pack(int rank, int root) { return ((unsigned)rank << kRankShift) | (unsigned)root; }
struct alignas(16) OneHalf {  // the part of a step record one chain reads: x (even lanes) or y (odd lanes)
    double r;
    float wb;  // wbx or wby
    float fs;
};
struct OneRec {  // step record (48 B): two reads per lane and step
    unsigned lk;   // light child's key (rank << 27 | root)
    unsigned bm;   // kStepB ? ~0 : 0
    unsigned lkp;  // lk + (1 << 27)
    unsigned pad;
    OneHalf h[2];
};
struct OneOut {  // per-step chain outputs, staged in LDS (one ds_write_b64 per lane per step)
    float v;     // mx (h = 0) or my (h = 1)
    unsigned k;  // key
};
}  // namespace dofs
#include "dofs_dataflow.h"
namespace dofs {


// ---------------------------------------------------------------------------------------------
// K3 deep levels: once the divide-and-conquer block size is kDeepS merges, every remaining level of
// a block only involves that block's merges and the labels they touch, so one workgroup runs all
// of them in LDS. The block's (at most 2*kDeepS) distinct labels get compact local ids — an LDS
// hash table of the global labels, then a workgroup scan over its occupied slots — and a component
// created at merge t of the block gets local id 2*kDeepS + t. The per-level union / compress /
// L-root / relabel / cleanup phases of dofs_kernels.h (KDnc*) run between workgroup barriers.
// Output: the final endpoint labels of the block's merges (their KRT children) and the sizes of
// its new components — identical to the global kernels (union-find shapes differ, results do not).
// ---------------------------------------------------------------------------------------------
#ifndef DOFS_DEEP_S
#define DOFS_DEEP_S 2048
#endif
// host: the depths below 32 merges of an LDS KRT block as one register window pass (1, the default: deep
// block 51.7 → 43.5 µs) or as union-find depths (0); dofs_debug_krt_deep_wave (tests/test_gpu_krt_dnc.py)
inline int g_deep_wave = 1;
constexpr int kDeepS = DOFS_DEEP_S;
constexpr int kDeepK = 2 * kDeepS;              // distinct labels of a block (two per merge)
constexpr int kDeepL = kDeepK + kDeepS;         // local label space
constexpr int kDeepHT = kDeepK + kDeepK / 2;    // hash slots (load factor <= 2/3)
constexpr int kDeepT = kDeepS >= 2048 ? 1024 : 512;  // threads per block
static_assert(kDeepL < 32768 && kDeepHT < 32768, "local ids are int16");

// LDS operations of one wave complete in order: waiting for them makes them visible to its other lanes
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// a workgroup barrier that orders LDS only: outstanding global loads and stores are not waited for
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ inline int lds_ld(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ inline void lds_st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ inline int lds_find(int* P, int x) {
    for (;;) {
        const int p = lds_ld(P + x);
        if (p == x) return x;
        const int gp = lds_ld(P + p);
        if (gp == p) return p;
        lds_st(P + x, gp);
        x = gp;
    }
}
__device__ inline int lds_union(int* P, const int* SZ, int a, int b) {
    for (;;) {
        a = lds_find(P, a);
        b = lds_find(P, b);
        if (a == b) return -1;
        const int sa = SZ[a], sb = SZ[b];
        if (!(sa != sb ? sa < sb : uf_above(a, b))) {  // dnc_above on the LDS arrays
            const int t = a;
            a = b;
            b = t;
        }
        int old = a;
        __hip_atomic_compare_exchange_strong(P + a, &old, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == a) return a;
    }
}

// Measurement build only (-DDOFS_KRT_TIMING): thread 0 of each KRT workgroup adds the wall-clock time
// (100 MHz counter) of each phase to g_kt[i] (read by dofs_debug_krt_timing; tools/krt_timing.py).
#ifdef DOFS_KRT_TIMING
__device__ unsigned long long g_kt[20];
#define KT_DECL unsigned long long kt_last = wall_clock64();
#define KT(i)                                                  \
    do {                                                       \
        if (threadIdx.x == 0) {                                \
            const unsigned long long kt_now = wall_clock64();  \
            atomicAdd(&g_kt[i], kt_now - kt_last);             \
            kt_last = kt_now;                                  \
        }                                                      \
    } while (0)
#else
#define KT_DECL
#define KT(i) \
    do {      \
    } while (0)
#endif

struct DeepShared {
    int hkey[kDeepHT];    // global label in the slot (-1 empty)
    short hval[kDeepHT];  // compact local id of the slot
    int P[kDeepL], SZ[kDeepL], CS[kDeepL], MX[kDeepL];
    short lu[kDeepS], lv[kDeepS], own[kDeepS], lrr[kDeepS];
    int wsum[kDeepT / 64];
};

// deep_block's 16-merge window pass: step J (merge J of the window) for every lane of each 16-lane row
struct WinLanes {
    int ca, cb, za, zb;  // the lane's endpoint labels and their component sizes
    int p, L0;           // the lane's position in its window, the window's first merge label
};
template <int J>
__device__ inline void win_step(WinLanes& v) {
    constexpr int pat = 0x10 | (J << 5);  // ds_swizzle bitmask mode: lane (lane & 0x10) | J of each 32-lane half
    const int sa = __builtin_amdgcn_ds_swizzle(v.ca, pat), sb = __builtin_amdgcn_ds_swizzle(v.cb, pat);
    const int nz = __builtin_amdgcn_ds_swizzle(v.za, pat) + __builtin_amdgcn_ds_swizzle(v.zb, pat);
    if (J < v.p) {
        if (v.ca == sa || v.ca == sb) {
            v.ca = v.L0 + J;
            v.za = nz;
        }
        if (v.cb == sa || v.cb == sb) {
            v.cb = v.L0 + J;
            v.zb = nz;
        }
    }
}
template <int... J>
__device__ inline void win_steps(WinLanes& v, std::integer_sequence<int, J...>) {
    (win_step<J>(v), ...);
}

// all depths of one block [s0, s0 + cnt) (cnt <= kDeepS) of frame f, in LDS
__device__ void deep_block(const Ws& w, DeepShared& sh, int f, int64_t s0, int cnt) {
    const Dims& d = w.d;
    const int64_t lb = f * d.NL, eb = f * d.M;
    const int tid = threadIdx.x;
    for (int x = tid; x < kDeepHT; x += kDeepT) sh.hkey[x] = -1;
    __syncthreads();
    constexpr int kPerT = kDeepS / kDeepT;  // merges per thread
    static_assert(kPerT * kDeepT == kDeepS, "deep block shape");
    int gl[2 * kPerT];  // the labels, all loaded before the first insert
#pragma unroll
    for (int u = 0; u < kPerT; ++u) {
        const int t = tid + u * kDeepT;
        gl[2 * u] = t < cnt ? w.lu[eb + s0 + t] : 0;
        gl[2 * u + 1] = t < cnt ? w.lv[eb + s0 + t] : 0;
    }
#pragma unroll
    for (int u = 0; u < kPerT; ++u) {  // hash the global labels
        const int t = tid + u * kDeepT;
        if (t >= cnt) continue;
        for (int side = 0; side < 2; ++side) {
            const int g = gl[2 * u + side];
            int h = (int)(uf_prio(g) % (unsigned)kDeepHT);
            for (;;) {
                int old = -1;
                __hip_atomic_compare_exchange_strong(sh.hkey + h, &old, g, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old == -1 || old == g) break;
                h = h + 1 == kDeepHT ? 0 : h + 1;
            }
            (side ? sh.lv : sh.lu)[t] = (short)h;
        }
    }
    __syncthreads();
    {  // compact ids: exclusive scan of slot occupancy (each thread a run of consecutive slots)
        constexpr int per = (kDeepHT + kDeepT - 1) / kDeepT;
        const int beg = tid * per, end = min(beg + per, kDeepHT);
        int c = 0;
        for (int x = beg; x < end; ++x) c += sh.hkey[x] != -1;
        int incl = c;  // wave inclusive scan
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (__lane_id() >= o) incl += v;
        }
        if (__lane_id() == 63) sh.wsum[tid >> 6] = incl;
        __syncthreads();
        int base = incl - c;
        for (int wv = 0; wv < (tid >> 6); ++wv) base += sh.wsum[wv];
        // the merge labels' sizes: every load issued before any is used (a pixel label is a leaf of
        // size 1 and an empty slot loads nothing useful: both read a valid dummy word)
        int gk[per], gz[per];
#pragma unroll
        for (int u = 0; u < per; ++u) {
            const int x = beg + u;
            gk[u] = x < end ? sh.hkey[x] : -1;
        }
        // agent-scope (L1-bypassing) loads: a label may be a merge of this block whose size this
        // workgroup stored moments ago (top_level, the first half's deep_block) into a line its L1
        // still holds from an earlier load — a plain load could return the line's old bytes
#pragma unroll
        for (int u = 0; u < per; ++u) gz[u] = dofs_ld(w.SZ + lb + (gk[u] >= d.N ? gk[u] : 0));
#pragma unroll
        for (int u = 0; u < per; ++u)
            if (gk[u] != -1) {
                sh.hval[beg + u] = (short)base;
                sh.SZ[base] = gk[u] < d.N ? 1 : gz[u];
                ++base;
            }
    }
    for (int x = tid; x < kDeepL; x += kDeepT) {
        sh.P[x] = x;
        sh.CS[x] = 0;
        sh.MX[x] = -1;
        if (x >= kDeepK) sh.SZ[x] = -1;  // the block's new nodes: written once, at the end
    }
    __syncthreads();
    for (int t = tid; t < cnt; t += kDeepT) {
        sh.lu[t] = sh.hval[sh.lu[t]];
        sh.lv[t] = sh.hval[sh.lv[t]];
    }
    __syncthreads();
    KT_DECL
    // a sub-block of S <= 64 merges lies in one wave (thread tid handles merges tid and tid + kDeepT,
    // 64 consecutive merges per wave) and its labels are no other sub-block's (a component current at
    // the sub-block's start was not merged by an earlier sub-block of the depth), so those depths
    // synchronise the wave only
    auto depth_sync = [&](int S) {
        if (S > 64)
            __syncthreads();
        else
            lds_wait();
    };
    const int s_last = w.deep_wave ? 32 : 2;  // the last depth of the LDS union-find form
    for (int S = kDeepS; S >= s_last; S >>= 1) {
        const int half = S >> 1;
        // union (L edges of sub-blocks whose R half exists)
        for (int t = tid; t < cnt; t += kDeepT) {
            const bool isL = (t & (S - 1)) < half && s0 + (t & ~(S - 1)) + half < d.M;
            if (isL) sh.own[t] = (short)lds_union(sh.P, sh.SZ, sh.lu[t], sh.lv[t]);
        }
        depth_sync(S);
        for (int t = tid; t < cnt; t += kDeepT) {  // compress + aggregate
            const bool isL = (t & (S - 1)) < half && s0 + (t & ~(S - 1)) + half < d.M;
            if (!isL) continue;
            const int h = sh.own[t];
            int r = h;
            for (int p = lds_ld(sh.P + r); p != r; p = lds_ld(sh.P + r)) r = p;
            for (int y = h; y != r;) {
                const int p = lds_ld(sh.P + y);
                if (p != r) lds_st(sh.P + y, r);
                y = p;
            }
            atomicAdd(sh.CS + r, sh.SZ[h]);
            atomicMax(sh.MX + r, t);
        }
        depth_sync(S);
        // L-roots: sizes of the new components; R edges: relabel (both only read P, MX, CS)
        for (int t = tid; t < cnt; t += kDeepT) {
            if ((t & (S - 1)) < half) {
                const bool isL = s0 + (t & ~(S - 1)) + half < d.M;
                if (!isL) continue;
                const int r = sh.P[sh.own[t]];
                if (sh.MX[r] != t) {
                    sh.lrr[t] = -1;
                    continue;
                }
                sh.lrr[t] = (short)r;
                sh.SZ[kDeepK + t] = sh.CS[r] + sh.SZ[r];  // to global at the end (no store drain per depth)
            } else {
                for (int side = 0; side < 2; ++side) {
                    short* lp = side ? sh.lv : sh.lu;
                    const int x = lp[t];
                    const int r = sh.P[x];
                    const int li = sh.MX[r];
                    if (r != x || li >= 0) lp[t] = (short)(kDeepK + li);
                }
            }
        }
        depth_sync(S);
        for (int t = tid; t < cnt; t += kDeepT) {  // cleanup
            const bool isL = (t & (S - 1)) < half && s0 + (t & ~(S - 1)) + half < d.M;
            if (!isL) continue;
            sh.P[sh.own[t]] = sh.own[t];
            const int r = sh.lrr[t];
            if (r >= 0) {
                sh.MX[r] = -1;
                sh.CS[r] = 0;
            }
        }
        depth_sync(S);
        KT(S >= 256 ? 9 : 10);  // the upper depths (S >= 256) and the lower ones
    }
    if (w.deep_wave) {
        // The depths S <= 16 as one pass over each 16-merge window (one row of 16 lanes; thread tid holds
        // merges tid and tid + kDeepT). After depth 32 a window's labels are the components' labels at
        // the window start and belong to no other window. In rank order j, merge j joins the components
        // whose labels its lane holds; every later lane of the window whose endpoint carries one of those
        // two labels takes merge j's label and the sum of the two sizes. A lane stops updating at its own
        // step, so after the pass it holds its merge's children (labels and sizes): the KRT children the
        // four depths compute, without their unions and barriers. Row broadcasts by ds_swizzle (the LDS
        // crossbar, no memory access): a wave-wide readlane loop over 64 lanes was VALU-bound (measured
        // slower than the depths it replaced).
        const int lane = tid & 63, p = lane & 15;
#pragma unroll
        for (int u = 0; u < kDeepS / kDeepT; ++u) {
            const int t = tid + u * kDeepT;
            const bool valid = t < cnt;
            int ca = valid ? sh.lu[t] : -1, cb = valid ? sh.lv[t] : -1;
            int za = valid ? sh.SZ[ca] : 0, zb = valid ? sh.SZ[cb] : 0;
            WinLanes v{ca, cb, za, zb, p, kDeepK + t - p};  // merge j of the window: label L0 + j
            win_steps(v, std::make_integer_sequence<int, 15>{});
            ca = v.ca, cb = v.cb, za = v.za, zb = v.zb;
            if (valid) {
                sh.lu[t] = (short)ca;
                sh.lv[t] = (short)cb;
                sh.SZ[kDeepK + t] = za + zb;
            }
        }
        lds_wait();  // a window's labels and sizes are read by its own wave only
        KT(10);
    }
    // final labels (the edge's KRT children) as global ids: a local id below kDeepK was never
    // relabeled, so it is still the edge's own input label
    for (int t = tid; t < cnt; t += kDeepT) {
        const int a = sh.lu[t], b = sh.lv[t];
        if (a >= kDeepK) w.lu[eb + s0 + t] = (int)(d.N + s0 + (a - kDeepK));
        if (b >= kDeepK) w.lv[eb + s0 + t] = (int)(d.N + s0 + (b - kDeepK));
        const int z = sh.SZ[kDeepK + t];
        if (z >= 0) w.SZ[lb + d.N + s0 + t] = z;
        w.hls[eb + s0 + t] = hl_pack(sh.SZ[a], sh.SZ[b]);  // the children's sizes, for the epilogue
    }
}

// The depth above the deep block size (block of kDeepTop = 2 kDeepS merges), in LDS too: only its
// L half's labels (<= kDeepK) enter the union-find; an R-half endpoint is relabelled if the LDS hash
// finds its label among them (a label touched by an L edge is in a component with an L edge).
constexpr int kDeepTop = 2 * kDeepS;
constexpr int kTopL = kDeepK + kDeepS;
struct TopShared {
    int hkey[kDeepHT];
    short hval[kDeepHT];
    int P[kTopL], SZ[kTopL], CS[kTopL], MX[kTopL];
    short lu[kDeepS], lv[kDeepS], own[kDeepS];
    int wsum[kDeepT / 64];
};
__device__ inline int top_lookup(const TopShared& sh, int g) {  // hash slot of label g, or -1
    int h = (int)(uf_prio(g) % (unsigned)kDeepHT);
    for (;;) {
        const int k = sh.hkey[h];
        if (k == g) return h;
        if (k == -1) return -1;
        h = h + 1 == kDeepHT ? 0 : h + 1;
    }
}
__device__ void top_level(const Ws& w, TopShared& sh, int f, int64_t s0, int cnt) {
    const Dims& d = w.d;
    const int64_t lb = f * d.NL, eb = f * d.M;
    const int tid = threadIdx.x;
    const int nl = kDeepS;  // L half (the R half [kDeepS, cnt) is non-empty)
    for (int x = tid; x < kDeepHT; x += kDeepT) sh.hkey[x] = -1;
    __syncthreads();
    for (int t = tid; t < nl; t += kDeepT) {
        for (int side = 0; side < 2; ++side) {
            const int g = side ? w.lv[eb + s0 + t] : w.lu[eb + s0 + t];
            int h = (int)(uf_prio(g) % (unsigned)kDeepHT);
            for (;;) {
                int old = -1;
                __hip_atomic_compare_exchange_strong(sh.hkey + h, &old, g, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old == -1 || old == g) break;
                h = h + 1 == kDeepHT ? 0 : h + 1;
            }
            (side ? sh.lv : sh.lu)[t] = (short)h;
        }
    }
    __syncthreads();
    {  // compact ids (as in deep_block)
        constexpr int per = (kDeepHT + kDeepT - 1) / kDeepT;
        const int beg = tid * per, end = min(beg + per, kDeepHT);
        int c = 0;
        for (int x = beg; x < end; ++x) c += sh.hkey[x] != -1;
        int incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (__lane_id() >= o) incl += v;
        }
        if (__lane_id() == 63) sh.wsum[tid >> 6] = incl;
        __syncthreads();
        int base = incl - c;
        for (int wv = 0; wv < (tid >> 6); ++wv) base += sh.wsum[wv];
        for (int x = beg; x < end; ++x)
            if (sh.hkey[x] != -1) {
                sh.hval[x] = (short)base;
                const int g = sh.hkey[x];
                sh.SZ[base] = g < d.N ? 1 : dofs_ld(w.SZ + lb + g);  // a pixel: a leaf of size 1 (no load)
                ++base;
            }
    }
    for (int x = tid; x < kTopL; x += kDeepT) {
        sh.P[x] = x;
        sh.CS[x] = 0;
        sh.MX[x] = -1;
    }
    __syncthreads();
    for (int t = tid; t < nl; t += kDeepT) {
        sh.lu[t] = sh.hval[sh.lu[t]];
        sh.lv[t] = sh.hval[sh.lv[t]];
    }
    __syncthreads();
    for (int t = tid; t < nl; t += kDeepT) sh.own[t] = (short)lds_union(sh.P, sh.SZ, sh.lu[t], sh.lv[t]);
    __syncthreads();
    for (int t = tid; t < nl; t += kDeepT) {  // compress + aggregate
        const int h = sh.own[t];
        int r = h;
        for (int p = lds_ld(sh.P + r); p != r; p = lds_ld(sh.P + r)) r = p;
        for (int y = h; y != r;) {
            const int p = lds_ld(sh.P + y);
            if (p != r) lds_st(sh.P + y, r);
            y = p;
        }
        atomicAdd(sh.CS + r, sh.SZ[h]);
        atomicMax(sh.MX + r, t);
    }
    __syncthreads();
    for (int t = tid; t < nl; t += kDeepT) {  // L-roots: sizes of the new components
        const int r = sh.P[sh.own[t]];
        if (sh.MX[r] == t) w.SZ[lb + d.N + s0 + t] = sh.CS[r] + sh.SZ[r];
    }
    for (int t = nl + tid; t < cnt; t += kDeepT) {  // relabel the R half in global memory
        for (int side = 0; side < 2; ++side) {
            int* gp = side ? (w.lv + eb + s0 + t) : (w.lu + eb + s0 + t);
            const int h = top_lookup(sh, *gp);
            if (h < 0) continue;
            const int x = sh.hval[h];
            const int r = sh.P[x];
            *gp = (int)(d.N + s0 + sh.MX[r]);
        }
    }
    __syncthreads();
}

// Epilogue of a block (KDncParent's work, plus block-local pointer jumping): the block's final labels
// are its merges' KRT children. Each merge splits them into heavy (larger subtree; ties -> A) and
// light, records the light side (hlB) and the path-top flags (lite), and seeds the heavy-first
// preorder's pointer-jumping words: a child's word = (parent, 1) if heavy, (parent, 2 size(heavy))
// if light. A child that is a merge of this block instead gets (the topmost ancestor inside the
// block, the sum of the offsets up to it), found by pointer jumping in LDS — so every global jump
// leaves a block, and the global pointer jumping needs ~log3(2 x blocks) launches, not log3(M).
struct ParentShared {
    // per block merge: (local parent index in the block, -1: parent outside) | offset sum << 32 —
    // one 64-bit word, so the jumping runs in place (every snapshot of an ancestor's word is valid)
    unsigned long long lw[kDeepTop];
    unsigned char lit[kDeepTop];  // path-top flag of a block merge whose parent is in the block
};
__device__ __forceinline__ unsigned long long lds_ld64(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ void deep_parent(const Ws& w, ParentShared& sh, int f, int64_t s0, int cnt) {
    const Dims& d = w.d;
    const int64_t lb = f * d.NL, eb = f * d.M;
    const int tid = threadIdx.x;
    const int64_t x0 = d.N + s0;  // node id of the block's first merge
    for (int t = tid; t < cnt; t += kDeepT) {
        sh.lw[t] = jump_pack(-1, 0);
        sh.lit[t] = 0xFF;
    }
    __syncthreads();
    for (int t = tid; t < cnt; t += kDeepT) {
        const int a = w.lu[eb + s0 + t], b = w.lv[eb + s0 + t];
        const unsigned long long zab = w.hls[eb + s0 + t];  // children's sizes (the deep blocks)
        const int sa = (int)(unsigned)(zab & 0xffffffffu), sb = (int)(unsigned)(zab >> 32);
        const bool lightB = sa >= sb;
        const int h = lightB ? a : b, l = lightB ? b : a;
        const int offl = 2 * (lightB ? sa : sb);
        w.hlB[eb + s0 + t] = lightB ? 1 : 0;
        w.hls[eb + s0 + t] = hl_pack(lightB ? sa : sb, lightB ? sb : sa);
        // path-top flags: read by KPathInit for merge nodes only (a leaf needs none); a child merge of
        // this block gets its flag in LDS (stored with the block's flags at the end, coalesced)
        if (h >= x0 && h < x0 + cnt) {
            sh.lw[h - x0] = jump_pack(t, 1);
            sh.lit[h - x0] = 0;
        } else if (w.jscatter && h >= d.N) {  // a merge child outside the block: its word and flag here
            w.J[lb + h] = jump_pack((int)(x0 + t), 1);
            w.lite[lb + h] = 0;
        }  // (else k_pre_sweep pushes its position and flag)
        if (l >= x0 && l < x0 + cnt) {
            sh.lw[l - x0] = jump_pack(t, offl);
            sh.lit[l - x0] = 1;
        } else if (w.jscatter && l >= d.N) {
            w.J[lb + l] = jump_pack((int)(x0 + t), offl);
            w.lite[lb + l] = 1;
        }
    }
    __syncthreads();
    // pointer jumping to the block-top ancestor (a node whose parent is outside the block keeps -1 and
    // its word is written by the block of its parent): in place, two hops per round on the freshest
    // words, one barrier per round, until a round in which no word advanced
    for (;;) {
        int moved = 0;
#pragma unroll
        for (int k = 0; k < kDeepTop / kDeepT; ++k) {
            const int t = tid + k * kDeepT;
            if (t >= cnt) continue;
            unsigned long long v = lds_ld64(sh.lw + t);
            bool mv = false;
#pragma unroll
            for (int hop = 0; hop < 2; ++hop) {
                const int p = jump_anc(v);
                if (p < 0) break;
                const unsigned long long u = lds_ld64(sh.lw + p);
                if (jump_anc(u) < 0) break;  // p is the block top
                v = jump_pack(jump_anc(u), jump_sum(v) + jump_sum(u));
                mv = true;
            }
            if (mv) {
                lds_st64(sh.lw + t, v);
                moved = 1;
            }
        }
        if (!__syncthreads_or(moved)) break;
    }
    const int64_t root = d.N + d.M - 1;
    for (int t = tid; t < cnt; t += kDeepT) {
        const unsigned long long v = sh.lw[t];
        const int p = jump_anc(v);
        const unsigned char c = sh.lit[t];
        if (c != 0xFF) w.lite[lb + x0 + t] = c;
        if (p >= 0) {
            w.J[lb + x0 + t] = jump_pack((int)(x0 + p), jump_sum(v));
        } else if (!w.jscatter) {  // a block top (parent outside the block) is marked -2: k_pre_sweep
            w.J[lb + x0 + t] = jump_pack(-2, 0);  // reads its pushed position
        } else if (x0 + t == root) {  // jumping: the root is converged at position 0 and a path top; the
            w.J[lb + x0 + t] = jump_pack(-1, 0);  // other tops' words come from their parents' blocks
            w.lite[lb + x0 + t] = 1;
        }
    }
}
static_assert(kDeepTop % kDeepT == 0, "parent epilogue shape");

constexpr size_t kDeepSmem0 = sizeof(DeepShared) > sizeof(TopShared) ? sizeof(DeepShared) : sizeof(TopShared);
constexpr size_t kDeepSmem = kDeepSmem0 > sizeof(ParentShared) ? kDeepSmem0 : sizeof(ParentShared);
// all depths of one kDeepTop-merge block of frame f in LDS, then its parents (block-uniform call);
// top: the block's first depth too (else the sweep did it: its labels are the two halves' starts)
__device__ void deep_item(const Ws& w, char* smem, int f, int64_t s0, bool top) {
    const Dims& d = w.d;
    const int cnt = (int)((d.M - s0) < kDeepTop ? (d.M - s0) : kDeepTop);
    KT_DECL
    if (top && cnt > kDeepS) top_level(w, *reinterpret_cast<TopShared*>(smem), f, s0, cnt);
    KT(5);
    deep_block(w, *reinterpret_cast<DeepShared*>(smem), f, s0, cnt < kDeepS ? cnt : kDeepS);
    __syncthreads();
    KT(6);
    if (cnt > kDeepS) deep_block(w, *reinterpret_cast<DeepShared*>(smem), f, s0 + kDeepS, cnt - kDeepS);
    __syncthreads();
    KT(7);
    deep_parent(w, *reinterpret_cast<ParentShared*>(smem), f, s0, cnt);
    __syncthreads();
    KT(8);
}
__global__ __launch_bounds__(kDeepT) void k_dnc_deep(Ws w, int top) {
    __shared__ __attribute__((aligned(16))) char smem[kDeepSmem];
    const int64_t s0 = (int64_t)blockIdx.x * kDeepTop;
    if (s0 >= w.d.M) return;
    deep_item(w, smem, blockIdx.y, s0, top != 0);
}

// ---------------------------------------------------------------------------------------------
// K2 Borůvka rounds >= 1, per-component minimum edge (KBoruvkaMinW / KBoruvkaMinI with workgroup
// pre-aggregation): one workgroup per 32x8 pixel tile, whose components are few (they are
// contiguous regions), combines its lanes' candidate edges per component in an LDS hash table and
// issues one global atomic per distinct component — instead of one per candidate edge endpoint.
// pass 0: minimum weight bits; pass 1: minimum emission index among the edges of that weight.
// ---------------------------------------------------------------------------------------------
constexpr int kTileX = 32, kTileY = 8, kMinHT = 512;  // 512 > 256 pixels + 82 halo keys per tile (no overflow)
// Tiles whose pixels have no cross-component edge left are done for good (components only merge):
// pass 0 marks them in `tdone` (per frame and tile) and later passes skip them.
// Pass 0: every pixel takes the lexicographic minimum (weight, index) over ALL its incident
// cross-component edges — the four it emits and the four its neighbours emit towards it — and
// keeps it (candw / candi); its component's minimum weight is the minimum over its pixels (an edge
// leaving the component has an end in it), reduced per wave and per tile before one global atomic.
// Pass 1 then only compares each pixel's kept weight with its component's minimum and reduces the
// kept indices of the equal ones — no weights recomputed, no neighbour reads.
__global__ __launch_bounds__(256) void k_boruvka_min(Ws w, int r, int pass, unsigned char* tdone,
                                                     unsigned long long* candw, unsigned* candi) {
    __shared__ int hk[kMinHT];
    __shared__ unsigned long long hv[kMinHT];
    __shared__ int any, tany;
    const Dims& d = w.d;
    const int f = blockIdx.y;
    if (pass == 0 ? (r > 0 && !w.C(f)[C_ACT + r - 1]) : !w.C(f)[C_ACT + r]) return;
    const int tiles_x = (d.W + kTileX - 1) / kTileX;
    const int tiles = tiles_x * ((d.H + kTileY - 1) / kTileY);
    const int* comp = w.comp + f * d.N;
    const F2* b = w.blur + f * d.N;
    unsigned long long* bw = w.bw + f * d.N;
    unsigned* bi = w.bi + f * d.N;
    unsigned long long* cw = candw + f * d.N;
    unsigned* ci = candi + f * d.N;
    const int tid = threadIdx.x;
    for (int x = tid; x < kMinHT; x += 256) {
        hk[x] = -1;
        hv[x] = ~0ull;
    }
    if (tid == 0) any = tany = 0;
    unsigned char* td = tdone + (int64_t)f * tiles;
    __syncthreads();
    auto put = [&](int key, unsigned long long v) {
        int slot = (int)(uf_prio(key) & (kMinHT - 1));
        for (;;) {
            int old = -1;
            __hip_atomic_compare_exchange_strong(hk + slot, &old, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == -1 || old == key) break;
            slot = (slot + 1) & (kMinHT - 1);
        }
        atomicMin(hv + slot, v);
    };
    for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
        if (td[t]) continue;  // block-uniform
        const int x = (t % tiles_x) * kTileX + (tid % kTileX), y = (t / tiles_x) * kTileY + tid / kTileX;
        int cp = -1;
        unsigned long long own = ~0ull;  // pass 0: the pixel's minimum weight; pass 1: its index
        if (x < d.W && y < d.H) {
            const int64_t p = (int64_t)y * d.W + x;
            if (pass == 0) {
                // all loads first, from in-frame addresses (an absent neighbour reads the pixel
                // itself and is masked below), so the wave waits on memory once per tile instead of
                // once per edge. Slots 0-3: the edges p emits (left, up, up-left, down-left); 4-7:
                // the edges its right, lower, lower-right and upper-right neighbours emit towards it.
                const int64_t W = d.W;
                const bool xl = x > 0, xr = x + 1 < d.W, yu = y > 0, yd = y + 1 < d.H;
                const bool ok[8] = {xl, yu, d.nbr8 && xl && yu, d.nbr8 && xl && yd,
                                    xr, yd, d.nbr8 && xr && yd, d.nbr8 && xr && yu};
                const int64_t nb[8] = {p - 1, p - W, p - W - 1, p + W - 1, p + 1, p + W, p + W + 1, p - W + 1};
                int64_t q[8];
                int cq[8];
                F2 bq[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) q[j] = ok[j] ? nb[j] : p;
                cp = comp[p];
                const F2 bp = b[p];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    cq[j] = comp[q[j]];
                    bq[j] = b[q[j]];
                }
                unsigned allow_bits = 0xff;  // bit j: slot j's edge may be in the MST
                if (w.allow) {               // launch-uniform
                    const unsigned char* al = w.allow + f * d.N;
                    const unsigned ap = al[p];
                    allow_bits = ap & 0xf;
#pragma unroll
                    for (int j = 4; j < 8; ++j) allow_bits |= ((al[q[j]] >> (j - 4)) & 1u) << j;
                }
                unsigned long long best = ~0ull;
                unsigned bidx = kNoEdge;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (!ok[j] || cq[j] == cp || !((allow_bits >> j) & 1)) continue;
                    // edge_weight(b, s, e) with s the emitting pixel: float differences, double squares
                    const F2 bs = j < 4 ? bp : bq[j], be = j < 4 ? bq[j] : bp;
                    const double dx = bs.x - be.x, dy = bs.y - be.y;
                    const unsigned long long wb = dbits(sqrt(sq_len(dx, dy)));
                    const unsigned idx = (unsigned)(4 * (j < 4 ? p : q[j]) + (j & 3));
                    if (wb < best || (wb == best && idx < bidx)) {
                        best = wb;
                        bidx = idx;
                    }
                }
                cw[p] = best;
                ci[p] = bidx;
                own = best;
                if (bidx != kNoEdge) any = tany = 1;
            } else {
                cp = comp[p];
                const unsigned long long wb = cw[p];
                const unsigned ix = ci[p];  // read beside the weight (one wait, then the minimum)
                if (wb != ~0ull && wb == bw[cp]) own = ix;
            }
        }
        {  // the lanes of a wave mostly share the component (a tile row of a contiguous region): one
           // put for the first such lane's component, reduced across the lanes that share it
            const bool has = own != ~0ull;
            const unsigned long long on = __ballot(has);
            if (on) {
                const int leader = __ffsll((long long)on) - 1;
                const int c0 = __shfl(cp, leader, 64);
                const bool same = has && cp == c0;
                unsigned long long m = same ? own : ~0ull;
                for (int o = 32; o >= 1; o >>= 1) {
                    const unsigned long long v = __shfl_xor(m, o, 64);
                    m = v < m ? v : m;
                }
                if (__lane_id() == leader) put(c0, m);
                if (has && !same) put(cp, own);
            }
        }
        __syncthreads();
        if (pass == 0 && tid == 0) {
            if (!tany) td[t] = (unsigned char)r;  // r >= 1: the last round that processed the tile
            tany = 0;
        }
        for (int x = tid; x < kMinHT; x += 256) {
            const int key = hk[x];
            if (key < 0) continue;
            const unsigned long long v = hv[x];
            if (pass == 0) {
                if (v < bw[key]) atomicMin(bw + key, v);
            } else {
                if ((unsigned)v < bi[key]) atomicMin(bi + key, (unsigned)v);
            }
            hk[x] = -1;
            hv[x] = ~0ull;
        }
        __syncthreads();
    }
    if (pass == 0 && tid == 0 && any) w.C(f)[C_ACT + r] = 1;
}

// Pixels of each frame's tiles by the round whose pass 0 found them done (0: never marked): tile t
// marked at round m was processed by pass 0 of rounds 1..m and pass 1 of rounds 1..m-1, so the host
// charges k_boruvka_min's bytes for exactly the pixels it touched (bench.py).
__global__ __launch_bounds__(256) void k_tile_hist(Ws w, const unsigned char* tdone) {
    __shared__ int bins[kRoundsMax];
    const Dims& d = w.d;
    const int f = blockIdx.y;
    const int tiles_x = (d.W + kTileX - 1) / kTileX;
    const int tiles = tiles_x * ((d.H + kTileY - 1) / kTileY);
    for (int k = threadIdx.x; k < kRoundsMax; k += blockDim.x) bins[k] = 0;
    __syncthreads();
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < tiles; t += gridDim.x * blockDim.x) {
        const int tx = t % tiles_x, ty = t / tiles_x;
        const int px = min(kTileX, d.W - tx * kTileX) * min(kTileY, d.H - ty * kTileY);
        const int m = tdone[(int64_t)f * tiles + t];
        atomicAdd(bins + (m < kRoundsMax ? m : 0), px);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kRoundsMax; k += blockDim.x)
        if (bins[k]) atomicAdd(w.tpx + (int64_t)f * kRoundsMax + k, bins[k]);
}

// ---------------------------------------------------------------------------------------------
// K2 Borůvka rounds >= 1 on frames of width % 4 == 0 without an edge mask (the hot path; other
// frames use k_boruvka_min): one wave per 32x8 tile, four pixels per lane (lane row = lane / 8,
// pixels 4 (lane % 8) .. + 3), no workgroup barrier.
//   k_boruvka_min4 (pass 0): each lane loads its three rows' labels as one 16-B load and flows as
//     two 16-B loads (+ the two halo columns), every pixel takes its lexicographic minimum over its
//     cross-component incident edges, and the wave reduces them per component in a wave-private
//     LDS hash to one (weight, index) record per (tile, component): the weight goes to the
//     component's global minimum, the record to the tile's k-th pixel slot of three pixel-strided
//     arrays. A tile with no record is done for good (as in k_boruvka_min).
//   k_boruvka_pick4 (pass 1): per record, the index goes to its component's minimum if its weight
//     is the component's minimum weight — records, not pixels.
//   k_boruvka_hookr: the record equal to its component's (weight, index) minimum hooks the component
//     along its edge and clears the minima (one winner per component: a cross edge has exactly one
//     end in it, so no two records of a component share an edge) — records, not a scan for roots.
// ---------------------------------------------------------------------------------------------
constexpr int kRecHT = 256;  // >= pixels of a tile, so the probing always finds a slot
struct RecHash {
    unsigned long long w[kRecHT];
    int k[kRecHT];
    unsigned i[kRecHT];
};
__device__ __forceinline__ int rec_slot(RecHash& h, int key) {
    int s = (int)(uf_prio(key) & (kRecHT - 1));
    for (;;) {
        int old = -1;
        __hip_atomic_compare_exchange_strong(h.k + s, &old, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == -1 || old == key) return s;
        s = (s + 1) & (kRecHT - 1);
    }
}
// pixel of tile t's record slot k (k < the tile's in-frame pixels, which bound its components)
__device__ __forceinline__ int64_t rec_px(const Dims& d, int tiles_x, int t, int k) {
    const int x0 = (t % tiles_x) * kTileX, y0 = (t / tiles_x) * kTileY;
    const int tw = min(kTileX, d.W - x0);
    return (int64_t)(y0 + k / tw) * d.W + x0 + k % tw;
}
struct RecBufs {  // the records: pixel-strided arrays free during the MST
    unsigned long long* rw;  // weight bits (the row-blur temporary)
    unsigned* ri;            // edge index (the MST count words)
    int* rk;                 // component (the MST emission offsets)
    unsigned char* td;       // per frame and tile: round that found it done (0: active)
    unsigned short* tc;      // per frame and tile: records of the last pass 0
};
__device__ __forceinline__ bool lexless(unsigned long long wa, unsigned ia, unsigned long long wb, unsigned ib) {
    return wa < wb || (wa == wb && ia < ib);
}
// The tiles a wave visits in a grid-stride loop (t = first + i * stride) that are still active: 64
// tiles' flags checked at once, one per lane (a done tile costs no dependent load of its own)
__device__ __forceinline__ unsigned long long active_tiles(const unsigned char* td, int t0, int stride, int tiles) {
    const int tl = t0 + __lane_id() * stride;
    return __ballot(tl < tiles && td[tl] == 0);
}
__global__ __launch_bounds__(256) void k_boruvka_min4(Ws w, int r, RecBufs rb) {
    __shared__ RecHash sh[4];
    const Dims& d = w.d;
    const int f = blockIdx.y;
    if (r > 0 && !w.C(f)[C_ACT + r - 1]) return;
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    RecHash& H = sh[wv];
    for (int k = lane; k < kRecHT; k += 64) {
        H.k[k] = -1;
        H.w[k] = ~0ull;
        H.i[k] = kNoEdge;
    }
    lds_wait();
    const int tiles_x = (d.W + kTileX - 1) / kTileX;
    const int tiles = tiles_x * ((d.H + kTileY - 1) / kTileY);
    const int* comp = w.comp + f * d.N;
    const F2* b = w.blur + f * d.N;
    unsigned long long* bw = w.bw + f * d.N;
    unsigned long long* rw = rb.rw + f * d.N;
    unsigned* ri = rb.ri + f * d.N;
    int* rk = rb.rk + f * d.N;
    unsigned char* td = rb.td + (int64_t)f * tiles;
    unsigned short* tc = rb.tc + (int64_t)f * tiles;
    const int W = d.W, Hh = d.H;
    int nrec = 0;
    for (int t0 = blockIdx.x * 4 + wv; t0 < tiles; t0 += 64 * gridDim.x * 4) {
        for (unsigned long long tm = active_tiles(td, t0, gridDim.x * 4, tiles); tm; tm &= tm - 1) {
            const int t = t0 + (__ffsll((long long)tm) - 1) * (gridDim.x * 4);
        const int x0 = (t % tiles_x) * kTileX + (lane & 7) * 4, y = (t / tiles_x) * kTileY + (lane >> 3);
        const bool valid = x0 < W && y < Hh;  // W % 4 == 0: the lane's four pixels are all in or all out
        const int yc = min(y, Hh - 1), xc = min(x0, W - 4);
        const int ry[3] = {max(yc - 1, 0), yc, min(yc + 1, Hh - 1)};
        const int xl = max(xc - 1, 0), xr = min(xc + 4, W - 1);
        // column j + 1 of the lane's row data holds pixel column xc + j (j = -1 .. 4)
        int C[3][6];
        F2 Fl[3][6];
#pragma unroll
        for (int R = 0; R < 3; ++R) {
            const int64_t o = (int64_t)ry[R] * W;
            const int4 c4 = *reinterpret_cast<const int4*>(comp + o + xc);
            const float4 fa = *reinterpret_cast<const float4*>(b + o + xc);
            const float4 fb = *reinterpret_cast<const float4*>(b + o + xc + 2);
            C[R][0] = comp[o + xl];
            C[R][1] = c4.x;
            C[R][2] = c4.y;
            C[R][3] = c4.z;
            C[R][4] = c4.w;
            C[R][5] = comp[o + xr];
            Fl[R][0] = b[o + xl];
            Fl[R][1] = F2{fa.x, fa.y};
            Fl[R][2] = F2{fa.z, fa.w};
            Fl[R][3] = F2{fb.x, fb.y};
            Fl[R][4] = F2{fb.z, fb.w};
            Fl[R][5] = b[o + xr];
        }
        // each pixel's lexicographic minimum (weight, index) over its cross-component incident edges
        bool has[4];
        int cp[4];
        unsigned long long mw[4];
        unsigned mi[4];
        const bool yu = y > 0, yd = y + 1 < Hh;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int x = xc + i;
            const int64_t p = (int64_t)y * W + x;
            const bool xlo = x > 0, xhi = x + 1 < W;
            const bool ok[8] = {xlo, yu, d.nbr8 && xlo && yu, d.nbr8 && xlo && yd,
                                xhi, yd, d.nbr8 && xhi && yd, d.nbr8 && xhi && yu};
            const int cq[8] = {C[1][i], C[0][i + 1], C[0][i], C[2][i], C[1][i + 2], C[2][i + 1], C[2][i + 2], C[0][i + 2]};
            const F2 fq[8] = {Fl[1][i], Fl[0][i + 1], Fl[0][i], Fl[2][i], Fl[1][i + 2], Fl[2][i + 1], Fl[2][i + 2], Fl[0][i + 2]};
            const int64_t nb[8] = {p - 1, p - W, p - W - 1, p + W - 1, p + 1, p + W, p + W + 1, p - W + 1};
            const int c0 = C[1][i + 1];
            const F2 f0 = Fl[1][i + 1];
            // edge_weight(b, s, e) = sqrt(sq) with s the emitting pixel (float differences, double
            // squares): sqrt is monotone and correctly rounded, so the minimum weight is sqrt of the
            // minimum sq, and an edge can tie with it only if its sq lies within 2^-48 (relative) of
            // the minimum — only those take a sqrt (the rounding interval of a weight is 2^-52 wide)
            // f32 prefilter: the squared lengths in f32 (relative error < 2^-22: the float differences are
            // the f64 path's own, then two multiplies and an add) pick the candidate edges; when one edge
            // alone lies within 2^-20 of the f32 minimum, no other edge can be within 2^-48 of it in f64
            // (the tie window below), so it is the minimum and takes the only f64 square and sqrt. Ties,
            // near-ties, NaN / infinite and tiny (< 2^-100: f32 underflow) minima take the f64 path over all
            // eight edges, as before — the result is the same bit for bit either way.
            float m32 = __builtin_huge_valf();
            float fxm = 0.f, fym = 0.f;
            unsigned im = kNoEdge;
            bool odd = false;
            float s32[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const F2 bs = j < 4 ? f0 : fq[j], be = j < 4 ? fq[j] : f0;
                const float fx = bs.x - be.x, fy = bs.y - be.y;
                const float q = fx * fx + fy * fy;
                const bool c = ok[j] && cq[j] != c0;
                s32[j] = c ? q : -1.0f;  // (-1: not a candidate)
                odd |= c && !(q < __builtin_huge_valf());
                if (c && q < m32) {
                    m32 = q;
                    fxm = fx;
                    fym = fy;
                    im = (unsigned)(4 * (j < 4 ? p : nb[j]) + (j & 3));
                }
            }
            const float thr32 = m32 * (1.0f + 0x1p-20f);
            int nsel = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) nsel += s32[j] >= 0.f && s32[j] <= thr32;
            unsigned long long best = ~0ull;
            unsigned bidx = kNoEdge;
            if (!odd && nsel == 1 && m32 >= 0x1p-100f) {
                best = dbits(sqrt(sq_len((double)fxm, (double)fym)));
                bidx = im;
            } else if (im != kNoEdge || odd) {
                unsigned long long sqb[8];
                unsigned long long msq = ~0ull;  // bits of non-negative doubles order like the values
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const F2 bs = j < 4 ? f0 : fq[j], be = j < 4 ? fq[j] : f0;
                    const double dx = bs.x - be.x, dy = bs.y - be.y;
                    sqb[j] = (ok[j] && cq[j] != c0) ? dbits(sq_len(dx, dy)) : ~0ull;
                    msq = sqb[j] < msq ? sqb[j] : msq;
                }
                if (msq != ~0ull) {
                    double mv;
                    memcpy(&mv, &msq, 8);
                    best = dbits(sqrt(mv));
                    const unsigned long long thr = dbits(mv * 1.0000000000000036);  // (1 + 2^-48) mv
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (sqb[j] > thr) continue;  // also the non-candidates (~0)
                        bool tie = sqb[j] == msq;
                        if (!tie) {
                            double v;
                            memcpy(&v, &sqb[j], 8);
                            tie = dbits(sqrt(v)) == best;
                        }
                        const unsigned idx = (unsigned)(4 * (j < 4 ? p : nb[j]) + (j & 3));
                        if (tie && idx < bidx) bidx = idx;
                    }
                }
            }
            has[i] = valid && bidx != kNoEdge;
            cp[i] = c0;
            mw[i] = best;
            mi[i] = bidx;
        }
        // a lane's pixels mostly share their component: fold equal ones into the first
#pragma unroll
        for (int i = 1; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < i; ++j)
                if (has[i] && has[j] && cp[i] == cp[j]) {
                    if (lexless(mw[i], mi[i], mw[j], mi[j])) {
                        mw[j] = mw[i];
                        mi[j] = mi[i];
                    }
                    has[i] = false;
                }
        const bool lany = has[0] || has[1] || has[2] || has[3];
        const unsigned long long on = __ballot(lany);
        if (on) {  // wave-uniform
            // the first such lane's first component, reduced across the wave by shuffles; the rest
            // through the wave's LDS hash (weight minimum, then the index among the equal weights)
            const int leader = __ffsll((long long)on) - 1;
            const int mycf = has[0] ? cp[0] : has[1] ? cp[1] : has[2] ? cp[2] : cp[3];
            const int cl = __shfl(mycf, leader, 64);
            unsigned long long lw = ~0ull;
            unsigned li = kNoEdge;
            int slot[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                slot[i] = -1;
                if (!has[i]) continue;
                if (cp[i] == cl) {
                    lw = mw[i];  // at most one pixel entry of the lane per component after the fold
                    li = mi[i];
                } else {
                    slot[i] = rec_slot(H, cp[i]);
                    atomicMin(H.w + slot[i], mw[i]);
                }
            }
            unsigned long long m = lw;
            for (int o = 32; o >= 1; o >>= 1) {
                const unsigned long long v = __shfl_xor(m, o, 64);
                m = v < m ? v : m;
            }
            unsigned mi2 = lw == m ? li : kNoEdge;
            for (int o = 32; o >= 1; o >>= 1) {
                const unsigned v = __shfl_xor(mi2, o, 64);
                mi2 = v < mi2 ? v : mi2;
            }
            int sl = -1;
            if (lane == leader) {
                sl = rec_slot(H, cl);
                atomicMin(H.w + sl, m);
            }
            lds_wait();
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (slot[i] >= 0 && H.w[slot[i]] == mw[i]) atomicMin(H.i + slot[i], mi[i]);
            if (sl >= 0 && H.w[sl] == m) atomicMin(H.i + sl, mi2);
            lds_wait();
        }
        // flush: per occupied slot the component's global minimum weight and the tile's record
        int cnt = 0;
#pragma unroll
        for (int s = 0; s < kRecHT / 64; ++s) {
            const int k = lane + 64 * s;
            const int key = H.k[k];
            const bool occ = key >= 0;
            const unsigned long long ob = __ballot(occ);
            if (occ) {
                const int pos = cnt + __popcll(ob & ((1ull << lane) - 1));
                const unsigned long long hw = H.w[k];
                const unsigned hi = H.i[k];
                atomicMin(bw + key, hw);  // no return value: no wait
                const int64_t px = rec_px(d, tiles_x, t, pos);
                rw[px] = hw;
                ri[px] = hi;
                rk[px] = key;
                H.k[k] = -1;
                H.w[k] = ~0ull;
                H.i[k] = kNoEdge;
            }
            cnt += __popcll(ob);
        }
        lds_wait();
        if (lane == 0) {
            tc[t] = (unsigned short)cnt;
            if (!cnt) td[t] = (unsigned char)r;  // r >= 1: the last round that processed the tile
        }
        nrec += cnt;
    }
    }
    if (lane == 0 && nrec) {
        w.C(f)[C_ACT + r] = 1;
        atomicAdd(w.trec + (int64_t)f * kRoundsMax + r, nrec);
    }
}
// pass 1 / hook over a frame's records (one wave per tile, lanes over its records)
template <bool kHook>
__global__ __launch_bounds__(256) void k_boruvka_recs(Ws w, int r, RecBufs rb) {
    const Dims& d = w.d;
    const int f = blockIdx.y;
    if (!w.C(f)[C_ACT + r]) return;
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    const int tiles_x = (d.W + kTileX - 1) / kTileX;
    const int tiles = tiles_x * ((d.H + kTileY - 1) / kTileY);
    unsigned long long* bw = w.bw + f * d.N;
    unsigned* bi = w.bi + f * d.N;
    const unsigned long long* rw = rb.rw + f * d.N;
    const unsigned* ri = rb.ri + f * d.N;
    const int* rk = rb.rk + f * d.N;
    const unsigned char* td = rb.td + (int64_t)f * tiles;
    const unsigned short* tc = rb.tc + (int64_t)f * tiles;
    __shared__ int pfx[4][65];  // per wave: record-count prefix over its 64 candidate tiles
    const int stride = gridDim.x * 4;
    for (int t0 = blockIdx.x * 4 + wv; t0 < tiles; t0 += 64 * stride) {
        // the records of 64 grid-stride tiles at once, flattened over the wave's lanes (later rounds
        // leave a tile few records: one tile per pass would leave most lanes idle behind a chain of
        // dependent loads); lane i reads tile i's flag and record count
        const int tl = t0 + lane * stride;
        const int c = (tl < tiles && td[tl] == 0) ? (int)tc[tl] : 0;
        int incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        const int total = __shfl(incl, 63, 64);
        if (!total) continue;  // wave-uniform
        pfx[wv][lane + 1] = incl;
        if (lane == 0) pfx[wv][0] = 0;
        lds_wait();
        for (int rr = lane; rr < total; rr += 64) {
            int lo = 0, hi = 64;  // pfx[lo] <= rr < pfx[hi]: the record's tile
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (pfx[wv][mid] <= rr) lo = mid; else hi = mid;
            }
            const int t = t0 + lo * stride, k = rr - pfx[wv][lo];
            const int64_t px = rec_px(d, tiles_x, t, k);
            const int key = rk[px];
            const unsigned long long wb = rw[px];
            const unsigned ix = ri[px];
            if (wb != bw[key]) continue;
            if (!kHook) {
                if (ix < bi[key]) atomicMin(bi + key, ix);
            } else if (ix == bi[key]) {  // the component's minimum edge: hook along it
                bw[key] = ~0ull;
                bi[key] = kNoEdge;
                const int64_t p = ix >> 2;
                const int e = ix & 3;
                const int64_t q = edge_end(d, p, e);
                const int* comp = w.comp + f * d.N;
                const int cp = comp[p], cq = comp[q];  // current roots: both ends lie in active tiles
                const int o = cp == key ? cq : cp;     // the component across the edge
                // Borůvka's hooking graph under a strict edge order is a forest plus one 2-cycle per tree
                // (two components whose minimum edge is the same edge), so the root points at the other
                // component directly — no finds, no CAS — and the edge's MST flag, set by an atomic OR, tells
                // the second of a mutual pair to root the pair at its smaller label (its partner's pointer
                // store was drained before the partner's OR). Round 6, same box: MST stage 29.4 → 27.5 ms,
                // 1,955 / 1,968 / 1,967 → 1,987 / 1,986 / 1,967 Mpix/s against the CAS union (uf_union)
                int* P = w.uf + f * d.N;
                dofs_st(P + key, o);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const unsigned bit = 1u << (8 * e);
                const unsigned old = __hip_atomic_fetch_or(reinterpret_cast<unsigned*>(w.mstbits + f * d.N + p), bit,
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old & bit) {
                    const int m = key < o ? key : o;
                    dofs_st(P + m, m);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K3 global depths, compress + aggregate (KDncCompress with workgroup pre-aggregation): agent-scope
// atomics execute at the memory side (MI355X_MICROARCH.md §Global float atomics; random 4-byte
// atomics measured at ~27 G/s by tools/atomic_micro.hip), so the 1024 lanes of a workgroup first
// combine their (component size, max L rank) contributions per root in an LDS hash table, and one
// lane per distinct root issues the two global atomics.
// ---------------------------------------------------------------------------------------------
constexpr int kAggT = 1024, kAggHT = 2048;
// test knob (dofs_debug_dnc_skew): the odd waves of every workgroup sleep about `skew` x 64 cycles before
// they read their slot's maximum, so the even waves reach the slot-table clear first — without the
// barrier between the read and the clear, that order loses L-roots in every iteration (the round-3 race)
__device__ int g_dnc_skew = 0;
__global__ __launch_bounds__(kAggT) void k_dnc_compress(Ws w, int64_t S, int ep) {
    __shared__ int hk[kAggHT], hcs[kAggHT], hmx[kAggHT];
    const int skew = g_dnc_skew;
    const Dims& d = w.d;
    const int f = blockIdx.y;
    const int64_t lb = f * d.NL;
    const unsigned tag = (unsigned)ep << kLabBits;
    const int mtag = ep << kRankBits;
    const int tid = threadIdx.x;
    for (int x = tid; x < kAggHT; x += kAggT) {
        hk[x] = -1;
        hcs[x] = 0;
        hmx[x] = 0;
    }
    __syncthreads();
    for (int64_t base = (int64_t)blockIdx.x * kAggT; base < d.M; base += (int64_t)gridDim.x * kAggT) {
        const int64_t i = base + tid;
        const bool act = i < d.M && dnc_is_L(d, i, S);
        int r = -1, slot = 0;
        if (act) {
            const int h = w.own[f * d.M + i];
            int szh;
            r = walk_compress(w.P + lb, h, tag, &szh);
            slot = (int)(uf_prio(r) & (kAggHT - 1));
            for (;;) {
                int old = -1;
                __hip_atomic_compare_exchange_strong(hk + slot, &old, r, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old == -1 || old == r) break;
                slot = (slot + 1) & (kAggHT - 1);
            }
            atomicAdd(hcs + slot, szh);
            atomicMax(hmx + slot, mtag | (int)i);
        }
        __syncthreads();
        if (skew && ((threadIdx.x >> 6) & 1))
            for (int z = 0; z < skew; ++z) __builtin_amdgcn_s_sleep(1);
        // only the workgroup's max rank of a component can be the component's max (its L-root):
        // own = the root for those candidates, -1 for the others (KDncLRootRelabel skips them)
        if (act) w.own[f * d.M + i] = hmx[slot] == (mtag | (int)i) ? r : -1;
        // every lane has read its slot's maximum before any slot is cleared below (without this
        // barrier a wave that is still on the line above can read a slot another wave has already
        // cleared: its L-root then never writes the component's size and CS[r] leaks into the next
        // depth — the DNC first-batch "size one too large" of round 3)
        __syncthreads();
        for (int x = tid; x < kAggHT; x += kAggT) {
            const int k = hk[x];
            if (k < 0) continue;
            atomicAdd(w.CS + lb + k, hcs[x]);
            const int m = hmx[x];
            if (__hip_atomic_load(w.MX + lb + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < m) atomicMax(w.MX + lb + k, m);
            hk[x] = -1;
            hcs[x] = 0;
            hmx[x] = 0;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// K3 block-start labels (KSeqInit, seq_*): one 1024-thread workgroup per frame sweeps the frame's
// rank blocks in order. Per block: (1) endpoint labels from the pixel union-find (roots kept in LDS),
// (2) the block's unions (lock-free; each hooked root recorded once), (3) per resulting root, in an
// LDS hash: the max rank in the block and the sizes of the roots hooked into it, then one write of
// its new label, size and the KRT node size. The frames' sweeps are latency-bound and use one CU
// each; the rest of the chip runs the other stream's replay stage meanwhile.
// ---------------------------------------------------------------------------------------------
constexpr int kSeqT = 1024, kSeqB = kDeepTop, kSeqK = kSeqB / kSeqT;
static_assert(kSeqK * kSeqT == kSeqB, "sweep shape");

// One workgroup owns a frame's union-find: workgroup-scope accesses (plain loads and stores that
// may stay in the CU's L1 / the XCD's L2; the kernel boundary publishes them to the next kernels)
__device__ __forceinline__ int wg_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void wg_st(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int wg_cas(int* p, int expect, int v) {
    __hip_atomic_compare_exchange_strong(p, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
    return expect;
}
// Union-find node of the sweep: parent, and at roots the component's max merge rank (-1: a single
// pixel) and size — one 16-byte record, so the find that reaches a root also reads its label and
// size (one memory request per hop). Kept in the StepIn region of the workspace, which KPathInit
// fills only after the KRT.
struct alignas(16) SeqRec {
    int par, pad, lab, sz;
};
static_assert(sizeof(SeqRec) == sizeof(StepIn), "the sweep's records live in the StepIn region, one per position");
struct KSeqInitRec {
    SeqRec* rec;
    int64_t NL2;  // records per frame stride (StepIn region: NL records of StepIn's size)
    DOFS_HD void operator()(int f, int64_t x) const {
        SeqRec r;
        r.par = (int)x;
        r.pad = 0;
        r.lab = -1;
        r.sz = 1;
        rec[f * NL2 + x] = r;
    }
};
// one 16-byte load (one request per hop: the finds are bounded by the CU's random-access rate); the
// empty asm keeps the unused pad word live, so the load is not narrowed into two requests
__device__ __forceinline__ SeqRec rec_ld(const SeqRec* p) {
    const int4 v = *reinterpret_cast<const int4*>(p);
    asm volatile("" ::"v"(v.y));
    SeqRec r;
    r.par = v.x;
    r.pad = v.y;
    r.lab = v.z;
    r.sz = v.w;
    return r;
}
__device__ __forceinline__ void rec_set_par(SeqRec* p, int v) { wg_st(&p->par, v); }

// finds of K chains at once, two hops per round (read-only: the sweep's phase D hooks every root one hop
// below its component's root, so paths stay short without compression, and the halving stores cost more
// than the hops they saved — round 5, same box: KRT −1 ms, +1.5 % end to end): each round issues every
// pending chain's load first; on return x[k] is the root and lab[k] / sz[k] its label and size (only the
// fields a caller needs stay live, to keep the sweep within 128 VGPRs)
template <int K>
__device__ __forceinline__ void rec_find(SeqRec* rec, int (&x)[K], bool (&pend)[K], int (&lab)[K], int (&sz)[K],
                                         int* rounds = nullptr) {
    for (;;) {
        if (rounds) ++*rounds;
        int pp[K], pl[K], ps[K];
        bool any = false;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (pend[k]) {
                const SeqRec r = rec_ld(rec + x[k]);
                pp[k] = r.par;
                pl[k] = r.lab;
                ps[k] = r.sz;
            }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (pend[k] && pp[k] == x[k]) {
                lab[k] = pl[k];
                sz[k] = ps[k];
                pend[k] = false;
            }
            any |= pend[k];
        }
        if (!any) return;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (pend[k]) {
                const SeqRec g = rec_ld(rec + pp[k]);
                if (g.par == pp[k]) {
                    x[k] = pp[k];
                    lab[k] = g.lab;
                    sz[k] = g.sz;
                    pend[k] = false;
                } else {
                    x[k] = g.par;
                }
            }
    }
}

// Per block of kSeqB merges:
//   A  endpoint roots at the block start -> labels (lu, lv): the only global finds of the block
//   B  the block-start roots into an LDS hash (the slot is the root's local id; the first inserter
//      keeps the root's block-start size)
//   C  the block's unions over slots, in LDS (lock-free, union by (block-start size, slot priority):
//      the key never changes during the block, so a component's LDS root is its largest root —
//      union by size keeps a frame's large components' roots stable, and the finds of later blocks
//      short); then per LDS root the max rank in the block (one LDS atomicMax per merge) and the
//      component's total size (every other slot adds its block-start size). The unions run in two
//      halves, which also does the LDS KRT's top level (the block's first depth): after the L half
//      (the first kDeepS merges) an R-half endpoint whose component holds an L merge is relabelled
//      to N + the component's max L rank, and the L-half component of the L half's last merge gets
//      its size (the only L-half node size the LDS blocks do not write themselves); the block's
//      labels are published after that, so each LDS-KRT block starts at its two halves' depths.
//   D  per slot, one global store: a hooked root's parent (directly its component's root), or at
//      the component's root its new label and size (8 bytes), plus the KRT node size SZ
// The global forest only gains the hooks of D, each root one hop below its component's root.
constexpr int kSeqHT = 12288;  // >= 2 kSeqB distinct roots at load <= 2/3
static_assert(kSeqHT >= 3 * kSeqB && kSeqHT < 65536 && kSeqB < 32767 && kSeqB == 2 * kDeepS, "sweep hash shape");
struct SweepShared {
    int key[kSeqHT];  // global root in the slot (-1 empty)
    int sz[kSeqHT];   // its size at the block start; at an LDS root after C, the component's total
    int pm[kSeqHT];   // LDS parent slot (low 16 bits); at an LDS root after C, (max rank + 1) << 16
    int rlast, zlast;  // the L half's last merge: its LDS root, its component's size
};
// finds in the slot forest (path halving; a non-root's high bits stay 0)
__device__ inline int swp_find(int* pm, int x) {
    for (;;) {
        const int p = lds_ld(pm + x) & 0xFFFF;
        if (p == x) return x;
        const int gp = lds_ld(pm + p) & 0xFFFF;
        if (gp == p) return p;
        lds_st(pm + x, gp);
        x = gp;
    }
}
__device__ inline void swp_union(int* pm, const int* sz, int a, int b) {
    for (;;) {
        a = swp_find(pm, a);
        b = swp_find(pm, b);
        if (a == b) return;
        const int sa = sz[a], sb = sz[b];
        if (!(sa != sb ? sa < sb : uf_above(a, b))) {
            const int t = a;
            a = b;
            b = t;
        }
        int old = lds_ld(pm + a);  // a root's word may carry its L-half max rank in the high bits
        if ((old & 0xFFFF) != a) continue;
        const int seen = old;
        __hip_atomic_compare_exchange_strong(pm + a, &old, b, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
        if (old == seen) return;
    }
}
// The sweep of frame f by one workgroup. progress (optional, stride kCounters per frame): after
// phase A of block b, the frame's word is set to b + 1 — the block's labels and every label size it refers to are then
// published (stored write-through, drained, one agent-scope flag store) for k_krt_fused's LDS-KRT
// workers.
__device__ void krt_sweep(const Ws& w, int f, SweepShared& sh, int* progress) {
    constexpr int K = kSeqK, K2 = 2 * kSeqK;
    int* key = sh.key;
    int* hsz = sh.sz;
    int* pm = sh.pm;
    const Dims& d = w.d;
    const int tid = threadIdx.x;
    SeqRec* rec = reinterpret_cast<SeqRec*>(w.In + f * d.NL);
    const int* EU = w.EU + f * d.M;
    const int* EV = w.EV + f * d.M;
    int* lu = w.lu + f * d.M;
    int* lv = w.lv + f * d.M;
    int* SZ = w.SZ + f * d.NL + d.N;
    for (int x = tid; x < kSeqHT; x += kSeqT) key[x] = -1;
    __syncthreads();
    KT_DECL
    for (int64_t s = 0; s < d.M; s += kSeqB) {
        const int cnt = (int)((d.M - s) < kSeqB ? (d.M - s) : kSeqB);
        // ---- A
        int e[K2], c[K2];
        bool act2[K2], pend[K2];
        int rtl[K2], rts[K2];  // roots' labels and sizes
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int t = tid + k * kSeqT;
            act2[2 * k] = act2[2 * k + 1] = t < cnt;
            e[2 * k] = t < cnt ? EU[s + t] : 0;
            e[2 * k + 1] = t < cnt ? EV[s + t] : 0;
        }
#pragma unroll
        for (int k = 0; k < K2; ++k) {  // a single pixel (its first merge, Ws::single) needs no find
            const bool one = (e[k] >> kSingleBit) & 1;
            e[k] &= kEndMask;
            c[k] = e[k];
            pend[k] = act2[k] && !one;
            rtl[k] = -1;
            rts[k] = 1;
        }
#ifdef DOFS_KRT_TIMING
        {  // the slowest thread's find rounds (two dependent loads each) in phase A
            int rounds = 0;
            rec_find<K2>(rec, c, pend, rtl, rts, &rounds);
            if (tid == 0) pm[0] = 0;
            __syncthreads();
            atomicMax(pm, rounds);
            __syncthreads();
            if (tid == 0) {
                atomicAdd(&g_kt[12], (unsigned long long)pm[0]);
                atomicAdd(&g_kt[13], 1ull);
            }
            __syncthreads();
        }
#else
        rec_find<K2>(rec, c, pend, rtl, rts);
#endif
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!act2[2 * k]) continue;
            const int t = tid + k * kSeqT;
            const int la = rtl[2 * k] < 0 ? e[2 * k] : (int)(d.N + rtl[2 * k]);
            const int lb = rtl[2 * k + 1] < 0 ? e[2 * k + 1] : (int)(d.N + rtl[2 * k + 1]);
            if (progress) {  // write-through (sc1): read by other workgroups after the flag
                __hip_atomic_store(lu + s + t, la, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(lv + s + t, lb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                lu[s + t] = la;
                lv[s + t] = lb;
            }
        }
        KT(0);
        // ---- B (after a barrier: the previous block's key clears precede the inserts; LDS only)
        lds_barrier();
        // A run of lanes holding the same root (consecutive merges of one component: late in a frame most
        // endpoints are the frame's largest component) inserts it once, by its first lane, and the others
        // find the slot with plain reads afterwards: CASes on one LDS word serialise, reads broadcast
        const int lane = __lane_id();
        int sl[K2];
        bool lead[K2];
#pragma unroll
        for (int k = 0; k < K2; ++k) {
            const int cp = __shfl_up(act2[k] ? c[k] : -1, 1, 64);
            lead[k] = act2[k] && !(lane > 0 && cp == c[k]);
            sl[k] = 0;
            if (!lead[k]) continue;
            int h = (int)(uf_prio(c[k]) % (unsigned)kSeqHT);
            for (;;) {
                int old = -1;
                __hip_atomic_compare_exchange_strong(key + h, &old, c[k], __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old == -1) {  // first inserter: the root's block-start size, a singleton slot
                    hsz[h] = rts[k];
                    pm[h] = h;
                    break;
                }
                if (old == c[k]) break;
                h = h + 1 == kSeqHT ? 0 : h + 1;
            }
            sl[k] = h;
        }
        // (the leaders' CASes have returned: their keys are in LDS, and a probe from the key's hash meets no
        // empty slot before it — keys are only set during this phase)
#pragma unroll
        for (int k = 0; k < K2; ++k) {
            if (!act2[k] || lead[k]) continue;
            int h = (int)(uf_prio(c[k]) % (unsigned)kSeqHT);
            while (lds_ld(key + h) != c[k]) h = h + 1 == kSeqHT ? 0 : h + 1;
            sl[k] = h;
        }
        __syncthreads();
        KT(1);
        // ---- C, L half (the merges t < kDeepS): unions, then per LDS root the max L rank
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (act2[2 * k] && tid + k * kSeqT < kDeepS) swp_union(pm, hsz, sl[2 * k], sl[2 * k + 1]);
        __syncthreads();
        // per LDS root the max rank: within a run of lanes of one root only the last (highest rank) lane's
        // atomic can raise it
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int t = tid + k * kSeqT;
            const bool a = act2[2 * k] && t < kDeepS;  // (t < kDeepS is uniform over a wave)
            const int r = a ? swp_find(pm, sl[2 * k]) : -1;
            const int rn = __shfl_down(r, 1, 64);
            if (a && !(lane < 63 && rn == r)) atomicMax(pm + r, r | ((t + 1) << 16));
            if (a && t == kDeepS - 1) sh.rlast = r;
        }
        if (tid == 0) sh.zlast = 0;
        __syncthreads();
        if (cnt > kDeepS) {  // the top level: R-half endpoints relabelled, the last L merge's size
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int t = tid + k * kSeqT;
                if (!act2[2 * k] || t < kDeepS) continue;
#pragma unroll
                for (int side = 0; side < 2; ++side) {
                    const int m = pm[swp_find(pm, sl[2 * k + side])] >> 16;  // (max L rank + 1), 0: none
                    if (!m) continue;
                    int* lp = side ? lv : lu;
                    const int lab = (int)(d.N + s + m - 1);
                    if (progress)
                        __hip_atomic_store(lp + s + t, lab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    else
                        lp[s + t] = lab;
                }
            }
            const int rl = sh.rlast;
            int z = 0;
            for (int x = tid; x < kSeqHT; x += kSeqT)
                if (key[x] >= 0 && swp_find(pm, x) == rl) z += hsz[x];
            if (z) atomicAdd(&sh.zlast, z);
            __syncthreads();
            if (tid == 0) {
                const int j = (int)(s + kDeepS - 1);
                if (progress)
                    __hip_atomic_store(SZ + j, sh.zlast, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else
                    SZ[j] = sh.zlast;
            }
        }
        if (progress) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        __syncthreads();
        if (progress && tid == 0)
            __hip_atomic_store(progress + (int64_t)f * kCounters, (int)(s / kSeqB) + 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        KT(4);
        // ---- C, R half: unions, max rank per LDS root (an L-only component keeps its L max), sizes
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (act2[2 * k] && tid + k * kSeqT >= kDeepS) swp_union(pm, hsz, sl[2 * k], sl[2 * k + 1]);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int t = tid + k * kSeqT;
            const bool a = act2[2 * k] && t >= kDeepS;
            const int r = a ? swp_find(pm, sl[2 * k]) : -1;
            const int rn = __shfl_down(r, 1, 64);
            if (a && !(lane < 63 && rn == r)) atomicMax(pm + r, r | ((t + 1) << 16));
        }
        for (int x = tid; x < kSeqHT; x += kSeqT) {
            if (key[x] < 0) continue;
            const int r = swp_find(pm, x);
            if (r != x) atomicAdd(hsz + r, hsz[x]);
        }
        __syncthreads();
        KT(2);
        // ---- D
        for (int x = tid; x < kSeqHT; x += kSeqT) {
            const int g = key[x];
            if (g < 0) continue;
            const int r = swp_find(pm, x);
            if (r != x) {
                rec_set_par(rec + g, key[r]);
                continue;
            }
            const int sz = hsz[x];
            const int j = (int)(s + (pm[x] >> 16) - 1);
            int2* lz = reinterpret_cast<int2*>(&rec[g].lab);
            *lz = make_int2(j, sz);
            if (progress)
                __hip_atomic_store(SZ + j, sz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                SZ[j] = sz;
        }
        __syncthreads();
        for (int x = tid; x < kSeqHT; x += kSeqT) key[x] = -1;  // next used after phase A's barrier
        KT(3);
    }
}

// ---------------------------------------------------------------------------------------------
// Borůvka per-pixel passes, four pixels per lane (one 16-byte label load): KBoruvkaHook and
// KBoruvkaRelabelFind of dofs_kernels.h. A frame's unaligned head and tail (H*W % 4 != 0) run
// one pixel per lane.
// ---------------------------------------------------------------------------------------------
struct Span4 {  // [0, head) scalar, [head, head + 4 n4) as int4, [tail, N) scalar
    int64_t head, n4, tail;
};
__device__ __forceinline__ Span4 span4(const int* frame, int64_t N) {
    Span4 sp;
    const int64_t mis = (int64_t)(((uintptr_t)frame >> 2) & 3);
    sp.head = mis ? 4 - mis : 0;
    if (sp.head > N) sp.head = N;
    sp.n4 = (N - sp.head) / 4;
    sp.tail = sp.head + 4 * sp.n4;
    return sp;
}
__global__ __launch_bounds__(256) void k_boruvka_hook4(Ws w, int r) {
    const int f = blockIdx.y;
    if (!w.C(f)[C_ACT + r]) return;
    const int64_t N = w.d.N;
    const int* comp = w.comp + f * N;
    const Span4 sp = span4(comp, N);
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < sp.n4; i += step) {
        const int64_t c = sp.head + 4 * i;
        const int4 v = *reinterpret_cast<const int4*>(comp + c);
        if (v.x == (int)c) boruvka_hook_root(w, f, c);
        if (v.y == (int)(c + 1)) boruvka_hook_root(w, f, c + 1);
        if (v.z == (int)(c + 2)) boruvka_hook_root(w, f, c + 2);
        if (v.w == (int)(c + 3)) boruvka_hook_root(w, f, c + 3);
    }
    if (i0 < sp.head + (N - sp.tail)) {
        const int64_t c = i0 < sp.head ? i0 : sp.tail + (i0 - sp.head);
        if (comp[c] == (int)c) boruvka_hook_root(w, f, c);
    }
}
// uf_find with plain (L1-cacheable) loads: no union runs during a relabel, so a root's word is final
// and any word read — stale or not — points to an ancestor; path halving stores stay as they are
__device__ __forceinline__ int uf_find_ro_halve(int* P, int x) {
    for (;;) {
        const int p = P[x];
        if (p == x) return x;
        const int gp = P[p];
        if (gp == p) return p;
        P[x] = gp;
        x = gp;
    }
}
// self: the chains run in comp itself (after k_boruvka_tile0: a pixel's root or a tile exit, an ancestor)
template <bool kSelf = false>
__global__ __launch_bounds__(256) void k_boruvka_relabel4(Ws w, int r) {
    const int f = blockIdx.y;
    if (!w.C(f)[C_ACT + r]) return;
    const int64_t N = w.d.N;
    int* comp = w.comp + f * N;
    int* uf = kSelf ? comp : w.uf + f * N;
    const Span4 sp = span4(comp, N);
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int64_t i = i0; i < sp.n4; i += step) {
        int4* p4 = reinterpret_cast<int4*>(comp + sp.head + 4 * i);
        const int4 v = *p4;
        int4 o;
        o.x = uf_find_ro_halve(uf, v.x);
        o.y = v.y == v.x ? o.x : uf_find_ro_halve(uf, v.y);
        o.z = v.z == v.y ? o.y : uf_find_ro_halve(uf, v.z);
        o.w = v.w == v.z ? o.z : uf_find_ro_halve(uf, v.w);
        if (o.x != v.x || o.y != v.y || o.z != v.z || o.w != v.w) *p4 = o;
    }
    if (i0 < sp.head + (N - sp.tail)) {
        const int64_t p = i0 < sp.head ? i0 : sp.tail + (i0 - sp.head);
        const int c = comp[p];
        const int root = uf_find_ro_halve(uf, c);
        if (root != c) comp[p] = root;
    }
}

// Round 0's KBoruvkaPairs and the first half of its relabel, per 64 x 32 tile (k_boruvka_relabel4 over
// comp finishes). KBoruvkaFirst left each pixel's pointer along its minimum edge
// in uf: a forest whose only cycles are the mutual pairs, each rooted at its smaller pixel. The tile and a
// 4-pixel halo are staged in LDS as cell pointers (a pointer goes to one of the eight neighbours, so only
// a halo cell can point out of the region: then the cell keeps the target pixel, encoded negative). The
// pairs are rooted (a pair leaving the region is checked in uf), then every cell finds its root or exit in
// LDS with path halving — the min-edge chains are long, and a walk without compression costs the square
// of a chain's length. A tile pixel's comp becomes its root, or the pixel its chain leaves the region by
// (an ancestor): k_boruvka_relabel4 on comp then follows those tile hops to the roots. The pair's smaller
// pixel roots itself in uf (the later rounds start their finds from the roots).
constexpr int kT0X = 64, kT0Y = 32, kT0H = 4, kT0RX = kT0X + 2 * kT0H, kT0RY = kT0Y + 2 * kT0H;
constexpr int kT0C = kT0RX * kT0RY, kT0T = 256, kT0K = (kT0C + kT0T - 1) / kT0T;  // cells per thread
__global__ __launch_bounds__(kT0T) void k_boruvka_tile0(Ws w) {
    __shared__ int U[kT0C];
    const Dims& d = w.d;
    const int f = blockIdx.y;
    if (!w.C(f)[C_ACT + 0]) return;
    const int W = d.W, H = d.H;
    int* uf = w.uf + f * d.N;
    int* comp = w.comp + f * d.N;
    const int tx = (W + kT0X - 1) / kT0X, ty = (H + kT0Y - 1) / kT0Y;
    const int tid = threadIdx.x;
    for (int64_t bi = blockIdx.x; bi < (int64_t)tx * ty; bi += gridDim.x) {
        const int bx = (int)(bi % tx) * kT0X - kT0H, by = (int)(bi / tx) * kT0Y - kT0H;  // region origin
        // cell pointers: the target cell, the cell itself (no edge), -1 (outside the frame), or -(2 + target
        // pixel) when the target lies outside the region
#pragma unroll
        for (int k = 0; k < kT0K; ++k) {
            const int e = tid + k * kT0T;
            if (e >= kT0C) break;
            const int cx = e % kT0RX, cy = e / kT0RX, gx = bx + cx, gy = by + cy;
            int v = -1;
            if (gx >= 0 && gx < W && gy >= 0 && gy < H) {
                const int g = gy * W + gx, t = uf[g];
                const int dl = t - g, dy = dl > 1 ? 1 : (dl < -1 ? -1 : 0), dx = dl - dy * W;
                const int nx = cx + dx, ny = cy + dy;
                v = (nx >= 0 && nx < kT0RX && ny >= 0 && ny < kT0RY) ? ny * kT0RX + nx : -(2 + t);
            }
            U[e] = v;
        }
        __syncthreads();
        // the pairs: the smaller pixel of a mutual pair becomes a root (decided on the staged pointers)
        bool root[kT0K];
#pragma unroll
        for (int k = 0; k < kT0K; ++k) {
            const int e = tid + k * kT0T;
            root[k] = false;
            if (e >= kT0C) continue;
            const int v = U[e];
            const int g = (by + e / kT0RX) * W + bx + e % kT0RX;
            if (v >= 0 && v != e) {
                const int t = (by + v / kT0RX) * W + bx + v % kT0RX;
                root[k] = U[v] == e && g < t;
            } else if (v <= -2) {
                const int t = -(v + 2);
                root[k] = g < t && uf[t] == g;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kT0K; ++k) {
            const int e = tid + k * kT0T;
            if (!root[k]) continue;
            U[e] = e;
            const int cx = e % kT0RX, cy = e / kT0RX;
            if (cx >= kT0H && cx < kT0H + kT0X && cy >= kT0H && cy < kT0H + kT0Y)  // the tile's own pixel
                uf[(by + cy) * W + bx + cx] = (by + cy) * W + bx + cx;
        }
        __syncthreads();
        // finds in LDS with path halving (concurrent halving stores only ever point to an ancestor)
        for (int e = tid; e < kT0C; e += kT0T) {
            int x = e;
            for (;;) {
                const int y = U[x];
                if (y < 0 || y == x) break;
                const int z = U[y];
                if (z < 0 || z == y) {
                    x = y;
                    break;
                }
                U[x] = z;
                x = z;
            }
            const int cx = e % kT0RX, cy = e / kT0RX;
            if (cx < kT0H || cx >= kT0H + kT0X || cy < kT0H || cy >= kT0H + kT0Y) continue;  // halo
            const int gx = bx + cx, gy = by + cy;
            if (gx >= W || gy >= H) continue;
            const int y = U[x];  // x: the root cell, or the cell whose pointer leaves the region
            comp[gy * W + gx] = y == x ? (by + x / kT0RX) * W + bx + x % kT0RX : -(y + 2);
        }
        __syncthreads();
    }
}

// Round 0's KBoruvkaInit + KBoruvkaFirst per 64 x 16 tile, for frames of width % 4 == 0 (at least 4) without
// an edge mask: the tile's blurred flows and a 2-pixel halo are staged in LDS once (one coalesced load per
// pixel instead of nine), every pixel of the tile and of its 1-pixel ring takes its minimum-edge slot
// (first_min_slot, as KBoruvkaFirst), and each tile pixel writes its whole MST-flag word — byte k set when
// its edge k is its own minimum (slot k) or the minimum of the neighbour that edge leads to (slot 4 + k
// there) — so no pass clears the words first; pointer, minima words and flags as 16-byte stores of four
// pixels per lane. Labels need no initialisation: k_boruvka_tile0 writes every pixel's.
constexpr int kF1X = 64, kF1Y = 16, kF1T = 256;
constexpr int kF1BX = kF1X + 4, kF1BY = kF1Y + 4;  // staged flows: a 2-pixel halo
constexpr int kF1SX = kF1X + 2, kF1SY = kF1Y + 2;  // slots: the tile and a 1-pixel ring
static_assert(kF1T == kF1Y * (kF1X / 4), "one lane per four pixels of the tile");
__global__ __launch_bounds__(kF1T) void k_boruvka_first_t(Ws w) {
    __shared__ F2 fb[kF1BY * kF1BX];
    __shared__ unsigned char sj[kF1SY * kF1SX];
    const Dims& d = w.d;
    const int f = blockIdx.y;
    const int W = d.W, H = d.H;
    const int64_t W64 = W;
    const F2* b = w.blur + f * d.N;
    const int tx = (W + kF1X - 1) / kF1X, ty = (H + kF1Y - 1) / kF1Y;
    const int tid = threadIdx.x;
    for (int64_t t = blockIdx.x; t < (int64_t)tx * ty; t += gridDim.x) {
        const int x0 = (int)(t % tx) * kF1X, y0 = (int)(t / tx) * kF1Y;
        // flows of [x0 - 2, x0 + 66) x [y0 - 2, y0 + 18), addresses clamped into the frame (a clamped cell
        // stands for no pixel: the slots' ok[] never reads it)
        for (int e = tid; e < kF1BY * kF1BX; e += kF1T) {
            int gx = x0 - 2 + e % kF1BX, gy = y0 - 2 + e / kF1BX;
            gx = gx < 0 ? 0 : (gx >= W ? W - 1 : gx);
            gy = gy < 0 ? 0 : (gy >= H ? H - 1 : gy);
            fb[e] = b[(int64_t)gy * W64 + gx];
        }
        __syncthreads();
        for (int e = tid; e < kF1SY * kF1SX; e += kF1T) {
            const int cx = e % kF1SX, cy = e / kF1SX;  // pixel (x0 - 1 + cx, y0 - 1 + cy)
            const int x = x0 - 1 + cx, y = y0 - 1 + cy;
            int jb = 0xFF;
            if (x >= 0 && x < W && y >= 0 && y < H) {
                const int64_t p = (int64_t)y * W64 + x;
                const bool xl = x > 0, xr = x + 1 < W, yu = y > 0, yd = y + 1 < H;
                const bool ok[8] = {xl, yu, d.nbr8 && xl && yu, d.nbr8 && xl && yd,
                                    xr, yd, d.nbr8 && xr && yd, d.nbr8 && xr && yu};
                const int64_t nb[8] = {p - 1, p - W64, p - W64 - 1, p + W64 - 1, p + 1, p + W64, p + W64 + 1, p - W64 + 1};
                const int c = (cy + 1) * kF1BX + cx + 1;
                const int nc[8] = {c - 1, c - kF1BX, c - kF1BX - 1, c + kF1BX - 1, c + 1, c + kF1BX, c + kF1BX + 1, c - kF1BX + 1};
                int64_t q[8];
                F2 bq[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    q[j] = ok[j] ? nb[j] : p;
                    bq[j] = fb[ok[j] ? nc[j] : c];
                }
                unsigned bidx;
                jb = first_min_slot(fb[c], bq, ok, 0xffu, p, q, &bidx);
            }
            sj[e] = (unsigned char)jb;
        }
        __syncthreads();
        const int ly = tid >> 4, lx = (tid & 15) * 4;
        const int x = x0 + lx, y = y0 + ly;
        if (x < W && y < H) {  // W % 4 == 0: the lane's four pixels are all in the frame
            const int64_t p = (int64_t)y * W64 + x;
            int far[4], jbs[4];
            unsigned mb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int cx = lx + i + 1, cy = ly + 1;
                const int jb = sj[cy * kF1SX + cx];
                const int64_t pi = p + i;
                const int64_t nb[8] = {pi - 1, pi - W64, pi - W64 - 1, pi + W64 - 1, pi + 1, pi + W64, pi + W64 + 1, pi - W64 + 1};
                int64_t fa = pi;
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (jb == j) fa = nb[j];
                far[i] = (int)fa;
                jbs[i] = jb;
                // edge k leads to the neighbour left, up, up-left, down-left, where it is slot 4 + k
                const int n0 = sj[cy * kF1SX + cx - 1], n1 = sj[(cy - 1) * kF1SX + cx];
                const int n2 = sj[(cy - 1) * kF1SX + cx - 1], n3 = sj[(cy + 1) * kF1SX + cx - 1];
                mb[i] = ((jb == 0 || n0 == 4) ? 1u : 0u) | ((jb == 1 || n1 == 5) ? 1u << 8 : 0u) |
                        ((jb == 2 || n2 == 6) ? 1u << 16 : 0u) | ((jb == 3 || n3 == 7) ? 1u << 24 : 0u);
            }
            const int64_t o = f * d.N + p;  // 16-byte aligned: N and p are multiples of 4
            *reinterpret_cast<int4*>(w.uf + o) = make_int4(far[0], far[1], far[2], far[3]);
            *reinterpret_cast<int4*>(w.mstbits + o) = make_int4((int)mb[0], (int)mb[1], (int)mb[2], (int)mb[3]);
            const unsigned long long none = ~0ull;
            reinterpret_cast<ulonglong2*>(w.bw + o)[0] = make_ulonglong2(none, none);
            reinterpret_cast<ulonglong2*>(w.bw + o)[1] = make_ulonglong2(none, none);
            *reinterpret_cast<uint4*>(w.bi + o) = make_uint4(kNoEdge, kNoEdge, kNoEdge, kNoEdge);
            if (w.single) {
                unsigned char* lt = w.lite + f * d.NL + p;
#pragma unroll
                for (int i = 0; i < 4; ++i) lt[i] = (unsigned char)jbs[i];
            }
            if (p == 0 && jbs[0] != 0xFF) w.C(f)[C_ACT + 0] = 1;
        }
        __syncthreads();  // the next tile's staging reuses fb and sj
    }
}

// KBoruvkaRelabelFind of rounds >= 1 on the record path, one wave per 32x8 tile (four pixels per lane):
// a tile is relabelled only while it or one of its eight neighbours is active. Pass 0 reads a tile's
// labels only for the tile itself or as the halo of a neighbour, the hook reads the labels of its
// edge's two ends (both ends have a cross-component edge, so both tiles were active in the last round
// too and were relabelled at its end), and nothing reads them after the MST — so a done tile among
// done tiles keeps its stale labels (tile flags: the round that found the tile done, written by this
// round's pass 0).
__global__ __launch_bounds__(256) void k_boruvka_relabel_t(Ws w, int r, RecBufs rb) {
    const Dims& d = w.d;
    const int f = blockIdx.y;
    if (!w.C(f)[C_ACT + r]) return;
    const int lane = __lane_id(), wv = threadIdx.x >> 6;
    const int tiles_x = (d.W + kTileX - 1) / kTileX, tiles_y = (d.H + kTileY - 1) / kTileY;
    const int tiles = tiles_x * tiles_y;
    const unsigned char* td = rb.td + (int64_t)f * tiles;
    int* comp = w.comp + f * d.N;
    int* uf = w.uf + f * d.N;
    const int stride = gridDim.x * 4;
    for (int t0 = blockIdx.x * 4 + wv; t0 < tiles; t0 += 64 * stride) {
        // lane i decides for tile t0 + i * stride: it or one of its neighbours still active (the
        // nine flags of 64 tiles loaded at once)
        bool act = false;
        {
            const int tl = t0 + lane * stride;
            if (tl < tiles) {
                const int tx = tl % tiles_x, ty = tl / tiles_x;
                unsigned char fl[9];
#pragma unroll
                for (int n = 0; n < 9; ++n) {
                    const int nx = tx + n % 3 - 1, ny = ty + n / 3 - 1;
                    const bool in = nx >= 0 && nx < tiles_x && ny >= 0 && ny < tiles_y;
                    fl[n] = td[in ? ny * tiles_x + nx : tl];
                }
#pragma unroll
                for (int n = 0; n < 9; ++n) act |= fl[n] == 0;
            }
        }
        for (unsigned long long tm = __ballot(act); tm; tm &= tm - 1) {
            const int t = t0 + (__ffsll((long long)tm) - 1) * stride;
            const int tx = t % tiles_x, ty = t / tiles_x;
            const int x0 = tx * kTileX + (lane & 7) * 4, y = ty * kTileY + (lane >> 3);
            if (x0 >= d.W || y >= d.H) continue;  // W % 4 == 0: a lane's four pixels are all in or all out
            int4* p4 = reinterpret_cast<int4*>(comp + (int64_t)y * d.W + x0);
            const int4 v = *p4;
            int4 o;
            o.x = uf_find_ro_halve(uf, v.x);
            o.y = v.y == v.x ? o.x : uf_find_ro_halve(uf, v.y);
            o.z = v.z == v.y ? o.y : uf_find_ro_halve(uf, v.z);
            o.w = v.w == v.z ? o.z : uf_find_ro_halve(uf, v.w);
            if (o.x != v.x || o.y != v.y || o.z != v.z || o.w != v.w) *p4 = o;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K1 blur, LDS-tiled (KBlurRow / KBlurCol of dofs_kernels.h, same float operations in the same
// order): a row segment of 256 outputs (+ reflect-101 halo) or a 64 x 64 column tile (+ halo rows)
// is staged once in LDS with coalesced loads, then every output reads its taps from LDS.
// ---------------------------------------------------------------------------------------------
constexpr int kBlurSeg = 256, kBlurR = kMaxTaps / 2;  // radius <= 31 (bn <= 63)
__global__ __launch_bounds__(kBlurSeg) void k_blur_row(Ws w) {
    __shared__ F2 buf[kBlurSeg + 2 * kBlurR];
    const int W = w.d.W, H = w.d.H;
    const int segs = (W + kBlurSeg - 1) / kBlurSeg;
    const int f = blockIdx.y;
    const int r = w.bn / 2;
    for (int64_t bi = blockIdx.x; bi < (int64_t)segs * H; bi += gridDim.x) {
        const int y = (int)(bi / segs), x0 = (int)(bi % segs) * kBlurSeg;
        const F2* row = w.flow + f * w.flow_fstride + (int64_t)y * W;
        for (int k = threadIdx.x; k < kBlurSeg + 2 * r; k += kBlurSeg) buf[k] = row[reflect101(x0 - r + k, W)];
        __syncthreads();
        const int x = x0 + threadIdx.x;
        if (x < W) {
            const F2* b = buf + threadIdx.x;
            float sx = w.bk[0] * b[0].x, sy = w.bk[0] * b[0].y;
            for (int t = 1; t < w.bn; ++t) {
                sx += w.bk[t] * b[t].x;
                sy += w.bk[t] * b[t].y;
            }
            F2 o;
            o.x = sx;
            o.y = sy;
            w.tmp[f * w.d.N + (int64_t)y * W + x] = o;
        }
        __syncthreads();
    }
}
constexpr int kColW = 64, kColH = 64, kColT = 256;
// one atomic per wave: the frame's largest |blurred component| (nonnegative float bits order as ints)
__device__ inline void blur_max_out(const Ws& w, int f, int mb) {
    mb = wave_reduce(mb, [](int x, int y) { return x > y ? x : y; });
    if (wave_lane() == 0 && mb > 0) atomicMax(w.C(f) + C_BMAX, mb);
}
__global__ __launch_bounds__(kColT) void k_blur_col(Ws w) {
    __shared__ F2 buf[(kColH + 2 * kBlurR) * kColW];
    const int W = w.d.W, H = w.d.H;
    const int tx = (W + kColW - 1) / kColW, ty = (H + kColH - 1) / kColH;
    const int f = blockIdx.y;
    const int r = w.bn / 2;
    const F2* src = w.tmp + f * w.d.N;
    const int cx = threadIdx.x % kColW, cg = threadIdx.x / kColW;  // column, row group
    int mb = 0;  // the largest |component| written (float bits): the frame's C_BMAX (key32_etop)
    for (int64_t bi = blockIdx.x; bi < (int64_t)tx * ty; bi += gridDim.x) {
        const int x0 = (int)(bi % tx) * kColW, y0 = (int)(bi / tx) * kColH;
        const int x = x0 + cx;
        const int rows = kColH + 2 * r;
        if (x < W)
            for (int k = cg; k < rows; k += kColT / kColW)
                buf[k * kColW + cx] = src[(int64_t)reflect101(y0 - r + k, H) * W + x];
        __syncthreads();
        if (x < W) {
            for (int yy = cg; yy < kColH; yy += kColT / kColW) {
                const int y = y0 + yy;
                if (y >= H) break;
                const F2* c = buf + (yy + r) * kColW + cx;
                float sx = w.bk[r] * c[0].x + 0.0f, sy = w.bk[r] * c[0].y + 0.0f;
                for (int j = 1; j <= r; ++j) {
                    const F2 a = c[j * kColW], b = c[-j * kColW];
                    sx += w.bk[r + j] * (a.x + b.x);
                    sy += w.bk[r + j] * (a.y + b.y);
                }
                F2 o;
                o.x = sx;
                o.y = sy;
                w.blur[f * w.d.N + (int64_t)y * W + x] = o;
                mb = max(mb, max(__float_as_int(fabsf(sx)), __float_as_int(fabsf(sy))));
            }
        }
        __syncthreads();
    }
    blur_max_out(w, f, mb);
}

// K1 in one pass (the blur radius of the reference's sigma = 3: 25 taps): per 64 x 32 output tile the
// input rows and columns it needs, (32 + 2r) x (64 + 2r) with reflect-101 in both directions, are
// staged in LDS once; the row filter writes (32 + 2r) x 64 row outputs to LDS (KBlurRow's operations
// and order), the column filter the tile (KBlurCol's). A lane computes 8 consecutive outputs from a
// 32-element window. No row-filtered field in HBM: 8 B in (plus halo) and 8 B out per pixel.
constexpr int kFbW = 64, kFbH = 32, kFbR = 12, kFbT = 256;
constexpr int kFbIW = kFbW + 2 * kFbR, kFbRH = kFbH + 2 * kFbR, kFbWin = 8 + 2 * kFbR;
static_assert(kFbW == 64 && kFbH % 8 == 0 && (kFbW / 64) * (kFbH / 8) * 64 == kFbT, "fused blur shape");
__global__ __launch_bounds__(kFbT) void k_blur_fused(Ws w) {
    __shared__ F2 in[kFbRH * kFbIW];
    __shared__ F2 ro[kFbRH * kFbW];
    const int W = w.d.W, H = w.d.H;
    const int tx = (W + kFbW - 1) / kFbW, ty = (H + kFbH - 1) / kFbH;
    const int f = blockIdx.y;
    const int tid = threadIdx.x;
    const F2* src = w.flow + f * w.flow_fstride;
    F2* dst = w.blur + f * w.d.N;
    float k[2 * kFbR + 1];
#pragma unroll
    for (int t = 0; t <= 2 * kFbR; ++t) k[t] = w.bk[t];
    constexpr int kLd = (kFbRH * kFbIW + kFbT - 1) / kFbT;  // staged elements per lane
    int mb = 0;  // the largest |component| written (float bits): the frame's C_BMAX (key32_etop)
    for (int64_t bi = blockIdx.x; bi < (int64_t)tx * ty; bi += gridDim.x) {
        const int x0 = (int)(bi % tx) * kFbW, y0 = (int)(bi / tx) * kFbH;
        // every lane's loads issued before any is stored (one memory wait per tile); reflect-101 by
        // one reflection, branch-free (the launcher keeps frames of W >= 128, H >= 64 here, so no
        // coordinate of a tile and its halo reflects twice)
        F2 st[kLd];
#pragma unroll
        for (int u = 0; u < kLd; ++u) {
            const int e = tid + u * kFbT;
            const int i = e / kFbIW, c = e % kFbIW;
            int yy = y0 - kFbR + i, xx = x0 - kFbR + c;
            yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);
            xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
            if (e < kFbRH * kFbIW) st[u] = src[(int64_t)yy * W + xx];
        }
#pragma unroll
        for (int u = 0; u < kLd; ++u) {
            const int e = tid + u * kFbT;
            if (e < kFbRH * kFbIW) in[e] = st[u];
        }
        __syncthreads();
        for (int it = tid; it < kFbRH * (kFbW / 8); it += kFbT) {  // row filter, 8 outputs per item
            const int i = it / (kFbW / 8), j = it % (kFbW / 8);
            if (x0 + 8 * j >= W) continue;  // columns beyond the frame feed no output
            const F2* r = in + i * kFbIW + 8 * j;
            F2 v[kFbWin];
#pragma unroll
            for (int q = 0; q < kFbWin; ++q) v[q] = r[q];
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                float sx = k[0] * v[o].x, sy = k[0] * v[o].y;
#pragma unroll
                for (int t = 1; t <= 2 * kFbR; ++t) {
                    sx += k[t] * v[o + t].x;
                    sy += k[t] * v[o + t].y;
                }
                F2 out;
                out.x = sx;
                out.y = sy;
                ro[i * kFbW + 8 * j + o] = out;
            }
        }
        __syncthreads();
        {  // column filter: lane = column, 8 rows per lane
            const int c = tid % kFbW, j = tid / kFbW;
            const int x = x0 + c;
            if (x < W) {
                F2 v[kFbWin];
#pragma unroll
                for (int q = 0; q < kFbWin; ++q) v[q] = ro[(8 * j + q) * kFbW + c];
#pragma unroll
                for (int o = 0; o < 8; ++o) {
                    const int y = y0 + 8 * j + o;
                    const F2 cc = v[o + kFbR];
                    float sx = k[kFbR] * cc.x + 0.0f, sy = k[kFbR] * cc.y + 0.0f;
#pragma unroll
                    for (int jj = 1; jj <= kFbR; ++jj) {
                        const F2 a = v[o + kFbR + jj], b = v[o + kFbR - jj];
                        sx += k[kFbR + jj] * (a.x + b.x);
                        sy += k[kFbR + jj] * (a.y + b.y);
                    }
                    F2 out;
                    out.x = sx;
                    out.y = sy;
                    if (y < H) {
                        dst[(int64_t)y * W + x] = out;
                        mb = max(mb, max(__float_as_int(fabsf(sx)), __float_as_int(fabsf(sy))));
                    }
                }
            }
        }
        __syncthreads();
    }
    blur_max_out(w, f, mb);
}

// ---------------------------------------------------------------------------------------------
// K3 fused: one persistent launch in which the
// latency-bound sweeps and the LDS KRT blocks share the chip. Every workgroup first claims a frame's
// sweep while any is unclaimed (a claimed sweep runs to its end without waiting on anything), then
// takes LDS-KRT blocks in block-major order; a block waits (agent-scope poll of its frame's
// progress word, then one acquire) until the sweep has published the block's labels. No workgroup
// ever waits on a workgroup that is not running, whatever the dispatch order.
//   ctl = C(0) words: [C_FUSE] sweep claims, [C_FUSE + 1] block claims; progress = C(f)[C_PROG]
// ---------------------------------------------------------------------------------------------
static_assert(kSeqT == kDeepT, "one workgroup shape for both roles");
constexpr size_t kFusedSmem = sizeof(SweepShared) > kDeepSmem ? sizeof(SweepShared) : kDeepSmem;
__global__ __launch_bounds__(kDeepT) void k_krt_fused(Ws w, int* progress) {
    __shared__ __attribute__((aligned(16))) char smem[kFusedSmem];
    __shared__ int item;
    const Dims& d = w.d;
    const int B = d.B;
    int* ctl = w.ctr + C_FUSE;
    const int tid = threadIdx.x;
    for (;;) {  // sweeps
        if (tid == 0) item = atomicAdd(ctl, 1);
        __syncthreads();
        const int f = item;
        __syncthreads();
        if (f >= B) break;
        krt_sweep(w, f, *reinterpret_cast<SweepShared*>(smem), progress);
        __syncthreads();
    }
    const int64_t nblk = (d.M + kDeepTop - 1) / kDeepTop;
    for (;;) {  // LDS KRT blocks, block-major over the frames
        if (tid == 0) item = atomicAdd(ctl + 1, 1);
        __syncthreads();
        const int it = item;
        __syncthreads();
        if (it >= nblk * B) break;
        const int f = it % B;
        const int64_t k = it / B;
        KT_DECL
        if (tid == 0) {
            while (__hip_atomic_load(progress + f * kCounters, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k + 1)
                __builtin_amdgcn_s_sleep(DOFS_SPIN_SLEEP);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        KT(11);
        deep_item(w, smem, f, k * kDeepTop, false);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// K4 preorder positions by one top-down sweep per frame over the KRT blocks (in place of the global
// pointer jumping, KJump, which the emulator keeps). A merge's parent has a higher rank; after the
// LDS KRT's epilogue a merge's word is (its block-top ancestor, offset sum) or, at a block top, the
// mark -2. The frame's blocks are taken last to first: a block top's position was pushed into pre[]
// by its parent's block (bit 31: it is a light child, a path top), the other merges add their offset
// sum to their top's position (LDS), and every merge then pushes its merge children outside the
// block (tops of earlier blocks) their positions (heavy: +1, light: +2 size(heavy)). Per block one
// coalesced read of pushed positions, no gathers; the merges' pre / ord entries, converged words and
// the tops' path-top flags come out of this pass, the leaves' from KLeafPos (parallel) after it.
// One workgroup per frame: latency-bound, it leaves the other CUs to the replay stage.
// ---------------------------------------------------------------------------------------------
constexpr int kPreT = 1024, kPreK = kDeepTop / kPreT;
static_assert(kPreK * kPreT == kDeepTop, "preorder sweep shape");
constexpr int kPushLight = (int)0x80000000u;
// The merges' ord[] entries and StepIn records are not written here (KLeafPos and KPathInit write them,
// chip-wide after the sweep): random stores from the one CU of a frame's sweep are bound by its waves'
// outstanding-store slots and sit inside its latency chain (round 4: −1.5 % and −0.3 % end to end).
__global__ __launch_bounds__(kPreT) void k_pre_sweep(Ws w) {
    __shared__ int lpos[kDeepTop];
    const Dims& d = w.d;
    const int f = blockIdx.x;
    const int64_t lb = f * d.NL, eb = f * d.M;
    unsigned long long* J = w.J + lb;
    int* pre = w.pre + lb;
    const int tid = threadIdx.x;
    const int64_t nblk = (d.M + kDeepTop - 1) / kDeepTop;
    const int64_t root = d.N + d.M - 1;
    struct Node {  // a merge's static inputs (final until swept)
        unsigned long long v, hl;
        int a, b;
        unsigned char lB;  // light side
    };
    Node nd[kPreK];
    auto load = [&](int64_t blk, Node (&o)[kPreK]) {
        const int64_t s0 = blk * kDeepTop;
        const int cnt = (int)((d.M - s0) < kDeepTop ? (d.M - s0) : kDeepTop);
#pragma unroll
        for (int k = 0; k < kPreK; ++k) {
            const int t = tid + k * kPreT;
            if (t < cnt) {
                o[k].v = J[d.N + s0 + t];
                o[k].hl = w.hls[eb + s0 + t];
                o[k].a = w.lu[eb + s0 + t];
                o[k].b = w.lv[eb + s0 + t];
                o[k].lB = w.hlB[eb + s0 + t];
            }
        }
    };
    if (nblk > 0) load(nblk - 1, nd);
    KT_DECL
    for (int64_t blk = nblk - 1; blk >= 0; --blk) {
        const int64_t s0 = blk * kDeepTop, x0 = d.N + s0;
        const int cnt = (int)((d.M - s0) < kDeepTop ? (d.M - s0) : kDeepTop);
        int pos[kPreK];
        bool top[kPreK];
        int pushed[kPreK];
#pragma unroll
        for (int k = 0; k < kPreK; ++k) {  // the tops' pushed positions (complete: the last barrier)
            const int t = tid + k * kPreT;
            top[k] = t < cnt && jump_anc(nd[k].v) == -2;
            pushed[k] = top[k] && x0 + t != root ? pre[x0 + t] : 0;
        }
        Node nx[kPreK];
        if (blk > 0) load(blk - 1, nx);  // prefetch the next block's inputs
#pragma unroll
        for (int k = 0; k < kPreK; ++k) {
            const int t = tid + k * kPreT;
            if (!top[k]) continue;
            pos[k] = pushed[k] & 0x7FFFFFFF;
            lpos[t] = pos[k];
            // path-top flag of a top: bit 31 of its push (the root: a path top)
            w.lite[lb + x0 + t] = x0 + t == root || (pushed[k] & kPushLight) ? 1 : 0;
        }
        lds_barrier();
        KT(14);
#pragma unroll
        for (int k = 0; k < kPreK; ++k) {
            const int t = tid + k * kPreT;
            if (t >= cnt) continue;
            const int64_t x = x0 + t;
            if (!top[k]) pos[k] = jump_sum(nd[k].v) + lpos[jump_anc(nd[k].v) - x0];
            pre[x] = pos[k];  // (the converged word is not needed: nothing reads J after this pass)
            // push the merge children outside the block (tops of earlier blocks) their positions;
            // the leaves get theirs from KLeafPos, in parallel after the sweep
            const int sh = (int)(unsigned)(nd[k].hl & 0xffffffffu);
            const int h = nd[k].lB ? nd[k].a : nd[k].b, l = nd[k].lB ? nd[k].b : nd[k].a;
            if (h < x0 && h >= d.N) pre[h] = pos[k] + 1;
            if (l < x0 && l >= d.N) pre[l] = (pos[k] + 2 * sh) | kPushLight;
        }
        KT(15);
        __syncthreads();  // the pushes are read by the blocks below
        if (blk > 0) {
#pragma unroll
            for (int k = 0; k < kPreK; ++k) nd[k] = nx[k];
        }
        KT(16);
    }
}

// K4 for small batches (Ws::jscatter): chip-wide pointer jumping instead of the per-frame sweep. After the
// LDS KRT's epilogue a merge's word points to its block-top ancestor inside the block (offset sum), and a
// block top's word to its parent outside the block (heavy +1, light +2 size(heavy)); the root's is (-1, 0).
// Only the tops jump: the in-block words are final (top, sum) snapshots, so a hop over a non-top lands on
// its block's top and costs nothing in the tree of tops, while a hop over a top follows that top's current
// word. Two hops over tops per launch, on the freshest words, at least triple every distance in the tree
// of tops (KJump's invariant, dofs_kernels.h), whose depth is at most the number of blocks.
DOFS_HD inline bool jump_in_block(const Dims& d, int a, int64_t x) {  // a (a merge node) in x's KRT block
    return (a - d.N) / kDeepTop == (x - d.N) / kDeepTop;
}
struct KJumpTop {
    Ws w;
    DOFS_HD void operator()(int f, int64_t k) const {
        const Dims& d = w.d;
        const int64_t lb = f * d.NL, x = d.N + k;
        unsigned long long v = dofs_ld64(w.J + lb + x);
        int a = jump_anc(v);
        if (a < 0 || jump_in_block(d, a, x)) return;  // converged, or not a block top
        for (int h = 0; h < 2 && a >= 0;) {
            const unsigned long long u = dofs_ld64(w.J + lb + a);
            const int na = jump_anc(u);
            if (na < 0 || !jump_in_block(d, na, a)) ++h;  // a is a top (a non-top points into its block)
            v = jump_pack(na, jump_sum(v) + jump_sum(u));
            a = na;
        }
        dofs_st64(w.J + lb + x, v);
    }
};
// then every merge's position: the sum of the offsets up to the root — a top's converged word, or an
// in-block word plus its top's. Every word is a valid (ancestor, sum) snapshot, so a word that is not
// converged is walked to the root here (never after enough KJumpTop launches: a guard, not a path).
struct KOrdMerge {
    Ws w;
    DOFS_HD void operator()(int f, int64_t k) const {
        const Dims& d = w.d;
        const int64_t lb = f * d.NL, x = d.N + k;
        const unsigned long long v = w.J[lb + x];
        int a = jump_anc(v);
        int q = jump_sum(v);
        while (a >= 0) {
            const unsigned long long u = w.J[lb + a];
            q += jump_sum(u);
            a = jump_anc(u);
        }
        w.pre[lb + x] = q;
        w.ord[lb + q] = (int)x;
    }
};

// the leaves' ord[] entries from their parents' positions (after k_pre_sweep): one lane per merge
// (a merge's own ord[] entry only has to say "a merge": ord is read for leaf pixels and tested >= N —
// KLeafOrder, the leaf scan, the replay's path starts — so the merges' positions get one coalesced fill,
// kOrdMerge, instead of a random store each)
constexpr int kOrdMerge = 0x7FFFFFFF;
struct KLeafPos {
    Ws w;
    DOFS_HD void operator()(int f, int64_t k) const {
        const Dims& d = w.d;
        const int64_t lb = f * d.NL, e = f * d.M + k;
        const int a = w.lu[e], b = w.lv[e];
        if (a >= d.N && b >= d.N) return;
        const int q = w.pre[lb + d.N + k];
        const int sh = (int)(unsigned)(w.hls[e] & 0xffffffffu);
        const bool lB = w.hlB[e] != 0;
        const int h = lB ? a : b, l = lB ? b : a;
        if (h < d.N) w.ord[lb + q + 1] = h;  // (a leaf's pre[] is not read: KPathInit uses lposr)
        if (l < d.N) w.ord[lb + q + 2 * sh] = l;
    }
};

#include "dofs_sortfix.h"

// The batch sort's onesweep shape: 512-thread sort blocks of 12 items per thread instead of rocPRIM's gfx950
// default (1024 x 16). The sort runs beside stage B of the previous batch (the replay's persistent workers, the
// scoring); a 1,024-thread block needs a quarter of a CU's wave slots free at once, and one pass's decoupled
// look-back chain waited behind such blocks (one pass 1.5 ms alone, 14.4 ms beside KLift / KLabel in the
// round-5 pipelined trace). Same box, B = 112, two runs each (round 6): default 1,874 / 1,902 Mpix/s, 512 x 12
// 1,928 / 1,945, with the default 1024 x 16 histogram blocks 1,943 / 1,945; 256 x 12 1,889 / 1,888, 512 x 16
// 1,895 / 1,904, 512 x 8 1,917 / 1,926. Build-time knobs for that A/B: DOFS_SORT_BS x DOFS_SORT_IPT per sort
// block, DOFS_SORT_HBS x DOFS_SORT_HIPT per histogram block.
#ifndef DOFS_SORT_BS
#define DOFS_SORT_BS 512
#define DOFS_SORT_IPT 12
#define DOFS_SORT_HBS 1024
#define DOFS_SORT_HIPT 16
#endif
using SortCfg = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<DOFS_SORT_HBS, DOFS_SORT_HIPT>,
                                        rocprim::kernel_config<DOFS_SORT_BS, DOFS_SORT_IPT>, 8,
                                        rocprim::block_radix_rank_algorithm::match>>;

struct HipBackend {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    hipError_t last = hipSuccess;
    std::string msg;
    struct Temp {
        hipStream_t s;
        void* p;
        size_t n;
    };
    std::vector<Temp> tmps;  // hipcub scratch, one per stream (the pipeline's phases run concurrently)
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> events;

    static bool device_ok(int dev) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n) return false;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
        return std::string(prop.gcnArchName).rfind("gfx950", 0) == 0;
    }

    Knobs kn;  // the context's runtime knobs (dofs_knobs.h), read when it was created
    HipBackend(int dev, const Knobs& k) : device(dev), kn(k) {
        note(hipSetDevice(dev), "hipSetDevice");
        note(hipStreamCreateWithFlags(&own, hipStreamNonBlocking), "hipStreamCreate");
        stream = own;
    }
    ~HipBackend() {
        for (auto e : pool) (void)hipEventDestroy(e);
        for (auto e : events) (void)hipEventDestroy(e);
        for (auto& t : tmps)
            if (t.p) (void)hipFree(t.p);
        if (flow_ctl) (void)hipFree(flow_ctl);
        if (flow_stream) (void)hipStreamDestroy(flow_stream);
        for (auto e : flow_ev)
            if (e) (void)hipEventDestroy(e);
        for (auto st : streams) (void)hipStreamDestroy(st);
        if (own) (void)hipStreamDestroy(own);
    }
    void note(hipError_t e, const char* what) {
        if (e != hipSuccess && last == hipSuccess) {
            last = e;
            msg = std::string(what) + ": " + hipGetErrorString(e);
        }
    }
    bool ok() const { return last == hipSuccess; }
    std::string error() const { return msg; }
    // caller stream of the device-resident API: NULL is the default (null) stream, as in HIP
    void set_stream(void* s) {
        (void)hipSetDevice(device);
        stream = (hipStream_t)s;
    }
    void use_own() {  // host-buffer API: the context's private stream
        (void)hipSetDevice(device);
        stream = own;
    }

    void* cur_stream() const { return stream; }
    void use(void* s) { stream = (hipStream_t)s; }
    // prio: 0 = default, > 0 = the device's greatest (most urgent) priority, < 0 = its least
    void* new_stream(int prio = 0) {
        hipStream_t st = nullptr;
        int least = 0, greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
        const int p = prio > 0 ? greatest : (prio < 0 ? least : 0);
        note(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, p), "hipStreamCreate");
        if (st) streams.push_back(st);
        return st;
    }
    void* new_event() {
        hipEvent_t e = nullptr;
        note(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        if (e) events.push_back(e);
        return e;
    }
    void record(void* ev, void* s) { note(hipEventRecord((hipEvent_t)ev, (hipStream_t)s), "hipEventRecord"); }
    void wait(void* s, void* ev) { note(hipStreamWaitEvent((hipStream_t)s, (hipEvent_t)ev, 0), "hipStreamWaitEvent"); }
    void event_sync(void* ev) { note(hipEventSynchronize((hipEvent_t)ev), "hipEventSynchronize"); }
    bool profiling() const { return prof; }

    void* alloc(size_t bytes) {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            note(e, "hipMalloc");
            return nullptr;
        }
        return p;
    }
    void free(void* p) {
        if (p) note(hipFree(p), "hipFree");
    }
    void memset(void* p, int v, size_t bytes) { note(hipMemsetAsync(p, v, bytes, stream), "hipMemsetAsync"); }
#ifdef DOFS_MEASURE
    void delay_us(int us) { hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, stream, us); }
#endif
    void h2d(void* d, const void* h, size_t bytes) {
        note(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync H2D");
        sync();
    }
    void d2h(void* h, const void* d, size_t bytes) {
        note(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync D2H");
    }
    void sync() { note(hipStreamSynchronize(stream), "hipStreamSynchronize"); }
    // one device int, read synchronously (the caller has waited for the work that wrote it)
    int read_int(const int* d) {
        int v = 0;
        note(hipMemcpy(&v, d, sizeof(int), hipMemcpyDeviceToHost), "hipMemcpy D2H");
        return v;
    }
    void copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height) {
        note(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, stream),
             "hipMemcpy2DAsync");
    }

    // ---- stage timing: events at stage boundaries, resolved lazily (no sync in the hot path) ----
    static constexpr int kStages = 8;
    bool prof = false;
    std::vector<std::array<hipEvent_t, kStages + 1>> pending;
    std::array<hipEvent_t, kStages + 1> cur{};
    double acc[kStages] = {0};
    int batches = 0;
    std::vector<hipEvent_t> pool;
    hipEvent_t ev_get() {
        hipEvent_t e;
        if (!pool.empty()) {
            e = pool.back();
            pool.pop_back();
        } else {
            note(hipEventCreate(&e), "hipEventCreate");
        }
        return e;
    }
    void profile(bool on) { prof = on; }
    void mark(int id) {
        if (!prof) return;
        if (id == 0) cur.fill(nullptr);
        cur[id] = ev_get();
        note(hipEventRecord(cur[id], stream), "hipEventRecord");
        if (id == kStages) pending.push_back(cur);
    }
    int profile_read(double* ms) {
        sync();
        for (auto& ev : pending) {
            int prev = -1;
            for (int s = 0; s <= kStages; ++s) {
                if (!ev[s]) continue;
                if (prev >= 0) {
                    float t = 0.f;
                    note(hipEventElapsedTime(&t, ev[prev], ev[s]), "hipEventElapsedTime");
                    acc[prev] += t;
                }
                prev = s;
            }
            for (auto e : ev)
                if (e) pool.push_back(e);
            ++batches;
        }
        pending.clear();
        for (int s = 0; s < kStages; ++s) {
            ms[s] = acc[s];
            acc[s] = 0;
        }
        int n = batches;
        batches = 0;
        return n;
    }

    // total workgroups of one grid-stride launch (all frames): enough to fill 256 CUs several
    // times over, few enough that near-empty passes (converged rounds) cost little to dispatch
    // (round 4, same box: a cap of 32,768 1,752-1,759 Mpix/s, 8,192 1,719-1,725, uncapped 1,622-1,628 against
    // 1,781-1,785 at 16,384 — converged Borůvka rounds pay for their grids)
    static constexpr int64_t grid_cap() { return 16384; }
    // The preorder-position scatters (KLeafPos, KLeafOrder, KPathInit) read and write one frame's
    // position-indexed arrays at random. Launched uncapped, one lane per merge, the dispatcher hands out
    // workgroups frame by frame (blockIdx.x fastest), and short workgroups hand their CU slots back within
    // microseconds to the graph stage's urgent kernels (round 4, same box: 1,749-1,751 → 1,778-1,779
    // Mpix/s; the scoring gathers launched the same way were 0.3 % slower)
    template <class F>
    static constexpr bool frame_major() {
        return std::is_same_v<F, KPathInit> || std::is_same_v<F, KLeafOrder> || std::is_same_v<F, KLeafPos>;
    }
    template <class F>
    static int launch_on(hipStream_t s, int nf, int64_t n, const F& f) {
        if (n <= 0 || nf <= 0) return DOFS_OK;
        int64_t gx = (n + kBlock - 1) / kBlock;
        const int64_t cap = std::max<int64_t>(1, grid_cap() / nf);
        if (gx > cap && !(frame_major<F>() && gx <= (int64_t)1 << 30)) gx = cap;
        if constexpr (takes<F>::value)
            hipLaunchKernelGGL(k_generic_take<F>, dim3((unsigned)gx, (unsigned)nf), dim3(kBlock), 0, s, f, n);
        else
            hipLaunchKernelGGL(k_generic<F>, dim3((unsigned)gx, (unsigned)nf), dim3(kBlock), 0, s, f, n);
        return hipGetLastError() == hipSuccess ? DOFS_OK : DOFS_ERR_DEVICE;
    }
    template <class F>
    static int launch_static(void* s, int nf, int64_t n, const F& f) {
        return launch_on((hipStream_t)s, nf, n, f);
    }
    // ---- kernel probe: device events around every launch of the named kernels ----------------
    // names: comma-separated kernel names (functor names of dofs_kernels.h or the HIP kernels'
    // names passed to timed()); per name, the accumulated event time and launch count
    std::vector<std::string> probe_names;
    std::vector<std::pair<int, std::array<hipEvent_t, 2>>> probe_ev;
    std::vector<double> probe_ms_acc;
    std::vector<int64_t> probe_launches;
    template <class F>
    static const char* type_name() {
        return __PRETTY_FUNCTION__;  // "... [F = dofs::KDncCompress]"
    }
    void probe(const char* names) {
        probe_names.clear();
        std::string s = names ? names : "";
        size_t a = 0;
        while (a < s.size()) {
            size_t b = s.find(',', a);
            if (b == std::string::npos) b = s.size();
            if (b > a) probe_names.push_back(s.substr(a, b - a));
            a = b + 1;
        }
        probe_ms_acc.assign(probe_names.size(), 0.0);
        probe_launches.assign(probe_names.size(), 0);
    }
    // per probed name: ms[i], launches[i] (n entries at most); returns the number of names
    int probe_read_n(int n, double* ms, int64_t* launches) {
        for (auto& pe : probe_ev) {
            auto& e = pe.second;
            note(hipEventSynchronize(e[1]), "hipEventSynchronize");
            float t = 0.f;
            note(hipEventElapsedTime(&t, e[0], e[1]), "hipEventElapsedTime");
            probe_ms_acc[pe.first] += t;
            ++probe_launches[pe.first];
            pool.push_back(e[0]);
            pool.push_back(e[1]);
        }
        probe_ev.clear();
        const int k = (int)probe_names.size();
        for (int i = 0; i < k && i < n; ++i) {
            ms[i] = probe_ms_acc[i];
            if (launches) launches[i] = probe_launches[i];
            probe_ms_acc[i] = 0;
            probe_launches[i] = 0;
        }
        return k;
    }
    int64_t probe_read(double* ms) {  // the first probed name
        int64_t n = 0;
        *ms = 0;
        std::vector<double> m(probe_names.size() + 1);
        std::vector<int64_t> l(probe_names.size() + 1);
        if (probe_read_n((int)probe_names.size(), m.data(), l.data()) > 0) {
            *ms = m[0];
            n = l[0];
        }
        return n;
    }
    // run `fn` (which enqueues one kernel on `stream`) between probe events if `name` is probed
    template <class Fn>
    void timed(const std::string& name, Fn&& fn) {
        int idx = -1;
        for (size_t i = 0; i < probe_names.size(); ++i)
            if (probe_names[i] == name) idx = (int)i;
        std::array<hipEvent_t, 2> ev{};
        if (idx >= 0) {
            ev = {ev_get(), ev_get()};
            note(hipEventRecord(ev[0], stream), "hipEventRecord");
        }
        fn();
        if (idx >= 0) {
            note(hipEventRecord(ev[1], stream), "hipEventRecord");
            probe_ev.push_back({idx, ev});
        }
    }
    template <class F>
    static std::string functor_name() {  // "KDncUnion" from "... [F = dofs::KDncUnion]"
        const std::string tn = type_name<F>();
        const size_t at = tn.find("F = dofs::");
        if (at == std::string::npos) return tn;
        const size_t end = tn.find_first_of("];", at);
        return tn.substr(at + 10, end == std::string::npos ? std::string::npos : end - at - 10);
    }
    template <class F>
    void launch(int nf, int64_t n, const F& f) {
        if (n <= 0 || nf <= 0) return;
        auto fn = [&] {
            if (launch_on(stream, nf, n, f) != DOFS_OK) note(hipErrorLaunchFailure, "kernel launch");
        };
        if (probe_names.empty())
            fn();
        else
            timed(functor_name<F>(), fn);
    }

    template <class F>
    void launch_counted(int nf, int64_t n, const F& f, int cidx, int zidx = -1) {
        if (n <= 0 || nf <= 0) return;
        int64_t gx = (n + kBlock - 1) / kBlock;
        const int64_t cap = std::max<int64_t>(1, grid_cap() / nf);
        if (gx > cap) gx = cap;
        timed(functor_name<F>(), [&] {
            hipLaunchKernelGGL(k_counted_take<F>, dim3((unsigned)gx, (unsigned)nf), dim3(kBlock), 0, stream, f, n, cidx,
                               zidx);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_counted_take launch");
    }
    static constexpr int64_t deep_block() { return kDeepTop; }
    void dnc_parent(const Ws&) {}  // done by k_dnc_deep's epilogue
    // the merges' ord entries for stage B's preorder (k_pre_sweep): the merge mark, one fill (KLeafPos places the
    // leaves). Issued in stage A after the blur — ord is no stage-A array — off stage B's chain of one sweep
    // per frame then KLeafPos (the jumping form, Ws::jscatter, writes the merges' entries itself)
    void ord_mark(const Ws& w) {
        if (pre_jump(w.d)) return;
        note(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(w.ord), kOrdMerge, (size_t)w.d.B * w.d.NL, stream),
             "hipMemsetD32Async");
    }
    void blur(const Ws& w) {  // KBlurRow + KBlurCol, LDS-tiled
        const int64_t cap = std::max<int64_t>(1, grid_cap() / w.d.B);
        if (w.bn == 2 * kFbR + 1 && w.d.W >= 128 && w.d.H >= 64) {  // sigma = 3: one pass
            const int64_t ft = (int64_t)((w.d.W + kFbW - 1) / kFbW) * ((w.d.H + kFbH - 1) / kFbH);
            timed("k_blur_fused", [&] {
                hipLaunchKernelGGL(k_blur_fused, dim3((unsigned)std::min(ft, cap), (unsigned)w.d.B), dim3(kFbT), 0,
                                   stream, w);
            });
            if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "blur launch");
            return;
        }
        const int64_t segs = (int64_t)((w.d.W + kBlurSeg - 1) / kBlurSeg) * w.d.H;
        const int64_t tiles = (int64_t)((w.d.W + kColW - 1) / kColW) * ((w.d.H + kColH - 1) / kColH);
        timed("k_blur_row", [&] {
            hipLaunchKernelGGL(k_blur_row, dim3((unsigned)std::min(segs, cap), (unsigned)w.d.B), dim3(kBlurSeg), 0,
                               stream, w);
        });
        timed("k_blur_col", [&] {
            hipLaunchKernelGGL(k_blur_col, dim3((unsigned)std::min(tiles, cap), (unsigned)w.d.B), dim3(kColT), 0,
                               stream, w);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "blur launch");
    }
    static constexpr bool kKrtLabelWords = false;  // the LDS KRT and the sweep keep their own words
    // small batches take the top-down global depths (4K, one frame: KRT 111 → 12 ms; 1080p, 8 frames:
    // 386 vs 312 Mpix/s). Round 3's first-batch size error of this path (1 in 6 fresh contexts) was the
    // slot-table race in k_dnc_compress, fixed there; tests/test_gpu_krt_dnc.py holds the two modes equal.
    static constexpr bool kDncAuto = true;
    static constexpr bool kSingleFlags = true;  // KMstEmit / KEdgeInit mark single-pixel endpoints (Ws::single)
    // Ws::rv_lean is honoured (the dataflow replay; the emulator's rounds store every record, but a lean
    // batch refuses dofs_events either way)
    static constexpr bool kLeanReplay = true;
    // longest pointer chain the preorder's global jumping starts from: every word leaves its block
    // or goes to the block's top, so at most two words per block on any path
    static int64_t jump_chain_bound(int64_t M) { return 2 * ((M + kDeepTop - 1) / kDeepTop) + 1; }
    // the frames' sweeps + the LDS KRT in one persistent launch (k_krt_fused), one 1,024-thread workgroup per
    // CU: a workgroup holds a whole CU (151 KB of LDS, all VGPRs). With the graph stage urgent and the
    // constant-key replay (round 3, B = 112, same box) every CU: 256 workgroups 1,593 / 1,586 / 1,584 / 1,587
    // Mpix/s against 240 (1/16 of the CUs left to the replay) 1,551 / 1,543 / 1,549 / 1,544
    void krt_seq(const Ws& w) {
        launch(w.d.B, w.d.N, KSeqInitRec{reinterpret_cast<SeqRec*>(w.In), w.d.NL});
        int nwg = 256;
        (void)hipDeviceGetAttribute(&nwg, hipDeviceAttributeMultiprocessorCount, device);
        Ws wk = w;
        wk.deep_wave = g_deep_wave;
        timed("k_krt_fused", [&] {
            hipLaunchKernelGGL(k_krt_fused, dim3((unsigned)std::max(1, nwg)), dim3(kDeepT), 0, stream, wk, w.ctr + C_PROG);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_krt_fused launch");
        fused_done = true;
    }
    bool fused_done = false;  // the last krt_seq already ran the LDS KRT (k_krt_fused)
    void dnc_deep(const Ws& w) {
        if (fused_done) {
            fused_done = false;
            return;
        }
        const unsigned nb = (unsigned)((w.d.M + kDeepTop - 1) / kDeepTop);
        Ws wk = w;
        wk.deep_wave = g_deep_wave;
        timed("k_dnc_deep", [&] {  // after the top-down global depths (DNC KRT): the block's top level too
            hipLaunchKernelGGL(k_dnc_deep, dim3(nb, (unsigned)w.d.B), dim3(kDeepT), 0, stream, wk, 1);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_dnc_deep launch");
    }
    void boruvka_hook(const Ws& w, int r) {
        if (rec_path(w)) {
            rec_launch(w, r, k_boruvka_recs<true>, "k_boruvka_hookr");
            return;
        }
        pixel4(w, r, k_boruvka_hook4, "KBoruvkaHook");
    }
    // K4 merge positions by the top-down sweep (k_pre_sweep) instead of KJump (which the emulator
    // keeps): it also writes the block tops' path-top flags, which the LDS KRT's epilogue leaves out
    bool pre_sweep(const Ws& w) {
        if (w.jscatter) {  // small batches: chip-wide jumping over the block tops (KJumpTop, KOrdMerge)
            int launches = 0;  // the tree of tops is at most one top per block deep
            const int64_t depth = (w.d.M + kDeepTop - 1) / kDeepTop + 1;
            for (int64_t span = 1; span < depth; span *= 3) ++launches;
            for (int t = 0; t < launches; ++t) launch(w.d.B, w.d.M, KJumpTop{w});
            launch(w.d.B, w.d.M, KOrdMerge{w});
        } else {
            timed("k_pre_sweep", [&] {
                hipLaunchKernelGGL(k_pre_sweep, dim3((unsigned)w.d.B), dim3(kPreT), 0, stream, w);
            });
            if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_pre_sweep launch");
        }
        launch(w.d.B, w.d.M, KLeafPos{w});
        return true;
    }
    // K4 by jumping (Ws::jscatter) for batches of at most DOFS_PRE_JUMP frames (default 8; 0 = always the
    // sweep): the sweep is one workgroup per frame, so a lone 4K frame walks its ~2,000 KRT blocks on one CU
    // while the rest of the chip idles
    bool pre_jump(const Dims& d) const { return d.B <= kn.pre_jump; }
    void boruvka_relabel(const Ws& w, int r) {
        if (r >= 1 && rec_path(w)) {  // round 0 runs before the tile flags exist
            rec_launch(w, r, k_boruvka_relabel_t, "k_boruvka_relabelt");
            return;
        }
        if (r == 0 && w.d.W >= 3) {  // KBoruvkaPairs + the relabel's in-tile part, then tile hops
            const int64_t tiles = (int64_t)((w.d.W + kT0X - 1) / kT0X) * ((w.d.H + kT0Y - 1) / kT0Y);
            const int64_t cap = std::max<int64_t>(1, grid_cap() / w.d.B);
            timed("k_boruvka_tile0", [&] {
                hipLaunchKernelGGL(k_boruvka_tile0, dim3((unsigned)std::min(tiles, cap), (unsigned)w.d.B), dim3(kT0T), 0,
                                   stream, w);
            });
            if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_boruvka_tile0 launch");
            pixel4(w, r, k_boruvka_relabel4<true>, "KBoruvkaRelabelFind");
            return;
        }
        pixel4(w, r, k_boruvka_relabel4<false>, "KBoruvkaRelabelFind");
    }
    // round 0's init + minimum edges per LDS tile (k_boruvka_first_t) on the record path's frames, whose
    // round 0 relabels by k_boruvka_tile0 (it writes every pixel's label); false: KBoruvkaInit + KBoruvkaFirst
    bool boruvka_first(const Ws& w) {
        if (!rec_path(w) || w.d.W < 4 || !pairs_in_relabel(w)) return false;
        const int64_t tiles = (int64_t)((w.d.W + kF1X - 1) / kF1X) * ((w.d.H + kF1Y - 1) / kF1Y);
        const int64_t cap = std::max<int64_t>(1, grid_cap() / w.d.B);
        timed("k_boruvka_first_t", [&] {
            hipLaunchKernelGGL(k_boruvka_first_t, dim3((unsigned)std::min(tiles, cap), (unsigned)w.d.B), dim3(kF1T), 0,
                               stream, w);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_boruvka_first_t launch");
        return true;
    }
    // round 0's pairs and relabel per LDS tile (k_boruvka_tile0) on frames at least 3 wide; narrower ones
    // take KBoruvkaPairs + k_boruvka_relabel4 over uf
    static bool pairs_in_relabel(const Ws& w) { return w.d.W >= 3; }
    void pixel4(const Ws& w, int r, void (*k)(Ws, int), const char* name) {
        const int64_t n4 = (w.d.N + 3) / 4;
        int64_t gx = (n4 + 255) / 256;
        const int64_t cap = std::max<int64_t>(1, grid_cap() / w.d.B);
        if (gx > cap) gx = cap;
        if (gx < 1) gx = 1;
        timed(name, [&] { hipLaunchKernelGGL(k, dim3((unsigned)gx, (unsigned)w.d.B), dim3(256), 0, stream, w, r); });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, name);
    }
    static int64_t tile_count(const Dims& d) {
        return (int64_t)((d.W + kTileX - 1) / kTileX) * ((d.H + kTileY - 1) / kTileY);
    }
    // the record-based rounds (k_boruvka_min4, ...): 16-byte label loads need W % 4 == 0; the tile
    // counts (u16) sit after the tile flags in the heavy/light bytes, which hold 3 bytes per tile
    static bool rec_path(const Ws& w) {
        return !w.allow && w.d.W % 4 == 0 && w.d.N >= 1024 && 3 * tile_count(w.d) + 2 <= w.d.M;
    }
    RecBufs rec_bufs(const Ws& w) {
        const int64_t tiles = tile_count(w.d);
        RecBufs rb;
        rb.rw = reinterpret_cast<unsigned long long*>(w.tmp);  // dead after the blur
        rb.ri = reinterpret_cast<unsigned*>(w.cnt);            // written only after the MST
        rb.rk = w.off;                                         // written only after the MST
        rb.td = w.hlB;                                         // filled by KDncParent after the KRT
        rb.tc = reinterpret_cast<unsigned short*>(w.hlB + ((tiles * w.d.B + 1) & ~(int64_t)1));
        return rb;
    }
    // the late rounds' grids shrink from round 11: by then few tiles of a 1080p batch are active, and a full
    // grid of early-exiting workgroups per kernel cost ~40 µs, 4 kernels a round for the ~12 rounds until
    // ceil(log2 N) + 2 (the tile loops are grid-stride, so any grid covers every tile)
    static constexpr int boruvka_shrink() { return 11; }
    void rec_launch(const Ws& w, int r, void (*k)(Ws, int, RecBufs), const char* name) {
        int64_t gx = std::min<int64_t>((tile_count(w.d) + 3) / 4, std::max<int64_t>(1, grid_cap() / w.d.B));
        const int sr = boruvka_shrink();
        if (sr > 0 && r >= sr) gx = std::max<int64_t>(std::min<int64_t>(gx, 8), gx >> std::min(r - sr + 1, 20));
        const RecBufs rb = rec_bufs(w);
        timed(name, [&] { hipLaunchKernelGGL(k, dim3((unsigned)gx, (unsigned)w.d.B), dim3(256), 0, stream, w, r, rb); });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, name);
    }
    void boruvka_min(const Ws& w, int r, int pass) {
        const int64_t tiles = tile_count(w.d);
        const int64_t gx = std::min<int64_t>(tiles, std::max<int64_t>(1, grid_cap() / w.d.B));
        unsigned char* tdone = w.hlB;  // free during the MST (KDncParent fills it after the KRT)
        static_assert(sizeof(*w.hlB) == 1, "tile flags are bytes");
        if (r == 1 && pass == 0) {
            memset(tdone, 0, (size_t)tiles * w.d.B);  // tiles <= M per frame
            memset(w.trec, 0, sizeof(int) * kRoundsMax * (size_t)w.d.B);
        }
        if (rec_path(w)) {
            rec_launch(w, r, pass == 0 ? k_boruvka_min4 : k_boruvka_recs<false>,
                       pass == 0 ? "k_boruvka_min4" : "k_boruvka_pick4");
            return;
        }
        timed("k_boruvka_min", [&] {
            // kept candidates: the row-blur temporary (8 B per pixel, dead after the blur) and the
            // MST-count words (written only after the MST)
            hipLaunchKernelGGL(k_boruvka_min, dim3((unsigned)gx, (unsigned)w.d.B), dim3(256), 0, stream, w, r, pass,
                               tdone, reinterpret_cast<unsigned long long*>(w.tmp), reinterpret_cast<unsigned*>(w.cnt));
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_boruvka_min launch");
    }
    void boruvka_tiles(const Ws& w) {
        const int64_t tiles = (int64_t)((w.d.W + kTileX - 1) / kTileX) * ((w.d.H + kTileY - 1) / kTileY);
        memset(w.tpx, 0, sizeof(int) * kRoundsMax * (size_t)w.d.B);
        if (w.d.N <= 1) return;  // no Borůvka round ran (the tile flags were never cleared)
        const unsigned gx = (unsigned)std::min<int64_t>((tiles + 255) / 256, 64);
        hipLaunchKernelGGL(k_tile_hist, dim3(gx, (unsigned)w.d.B), dim3(256), 0, stream, w, (const unsigned char*)w.hlB);
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_tile_hist launch");
    }
    void dnc_compress(const Ws& w, int64_t S, int ep) {
        int64_t gx = (w.d.M + kAggT - 1) / kAggT;
        const int64_t cap = std::max<int64_t>(1, 4096 / w.d.B);
        if (gx > cap) gx = cap;
        timed("k_dnc_compress", [&] {
            hipLaunchKernelGGL(k_dnc_compress, dim3((unsigned)gx, (unsigned)w.d.B), dim3(kAggT), 0, stream, w, S, ep);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_dnc_compress launch");
    }
    // K5 as one dataflow launch (dofs_dataflow.h): the round launches the emulator runs are not built here
    static constexpr bool kReplayFlow = true;
    int* flow_ctl = nullptr;
    size_t flow_ctl_n = 0;
    hipStream_t flow_stream = nullptr;
    hipEvent_t flow_ev[2] = {nullptr, nullptr};
    unsigned flow_epoch = 0;
    // short-path workers (waves). Round 5, B = 112, same box, two runs each: 512 → 1,749 / 1,750 Mpix/s (replay
    // 42 ms), 1,024 → 1,822 / 1,819 (29 ms), 2,048 → 1,889 / 1,896 (21 ms), 3,072 → 1,876 / 1,877, 4,096 → 1,876 /
    // 1,868: the short paths' lanes are the replay's parallelism until about 2,048 waves
    static constexpr int flow_grid() { return 2048; }
    // long-path workers (waves): DOFS_FLOW_LONG, default 256 (round 5, B = 112, same box, two runs each:
    // 128 → 1,816 / 1,823 Mpix/s, replay stage 36.7 ms; 256 → 1,869 / 1,869, 22.4 ms; 512 → 1,830 / 1,828)
    int flow_long_workers() const { return kn.flow_long > 0 ? kn.flow_long : 256; }
    bool replay_flow(const Ws& w) {
        if ((int64_t)w.d.B * w.d.N > kMaxBatchPixels) {  // (api_run refuses such batches)
            note(hipErrorInvalidValue, "batch too large for the replay's task words");
            return false;
        }
        const size_t n = FC_HDR + 3 * (size_t)(w.d.B + 1);
        if (n > flow_ctl_n) {
            if (flow_ctl) {
                note(hipDeviceSynchronize(), "hipDeviceSynchronize");  // a launch in flight may still use it
                free(flow_ctl);
            }
            flow_ctl = (int*)alloc(sizeof(int) * n);
            flow_ctl_n = flow_ctl ? n : 0;
            if (!flow_ctl) return false;
        }
        flow_epoch = flow_epoch % kFlowEpochs + 1;  // queue-slot tag of this launch (never 0)
        hipLaunchKernelGGL(k_flow_prep, dim3(1), dim3(64), 0, stream, w, flow_ctl);
        if (!flow_stream) {  // the long workers' launch runs beside the short workers' (no dependency)
            int least = 0, greatest = 0;
            (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
            note(hipStreamCreateWithPriority(&flow_stream, hipStreamNonBlocking, greatest), "hipStreamCreate");
            note(hipEventCreateWithFlags(&flow_ev[0], hipEventDisableTiming), "hipEventCreate");
            note(hipEventCreateWithFlags(&flow_ev[1], hipEventDisableTiming), "hipEventCreate");
        }
        timed("k_replay_flow", [&] {
            const int gs = (flow_grid() + kFlowShortW - 1) / kFlowShortW;
            const int gl = (flow_long_workers() + kFlowLongW - 1) / kFlowLongW;
            note(hipEventRecord(flow_ev[0], stream), "hipEventRecord");
            note(hipStreamWaitEvent(flow_stream, flow_ev[0], 0), "hipStreamWaitEvent");
            const int kf = g_keyfast;
            // g_flow_order (test entry dofs_debug_flow_order): 1 / 2 run the two launches one after the other on
            // one stream (long workers first / short workers first) — the replay must complete either way
            const int order = g_flow_order;
            hipStream_t ls = order ? stream : flow_stream;
            // wave pairs (chain and tail on two waves, flow_pair) for batches of at most kPairFrames frames, where
            // a frame's longest chain bounds the replay (one 4K frame: replay 59.2 → 43.8 ms); one wave per long
            // path for larger batches, where the long paths' throughput does and the pairs' extra waves slow the
            // graph stage beside them (B = 112, same box: 1,860 / 1,861 Mpix/s single waves, 1,826 / 1,825 with
            // 128 pairs, 1,826 / 1,824 with 256)
            auto long_launch = [&] {
                if (w.d.B <= kPairFrames)
                    hipLaunchKernelGGL(k_replay_flow_pair, dim3((unsigned)std::max(1, flow_long_workers() / 2)),
                                       dim3(128), 0, ls, w, flow_ctl, flow_epoch, kf);
                else
                    hipLaunchKernelGGL((k_replay_flow<true, kFlowLongW>), dim3((unsigned)gl), dim3(64 * kFlowLongW), 0, ls,
                                       w, flow_ctl, flow_epoch, kf);
            };
            if (order != 2) long_launch();
            hipLaunchKernelGGL((k_replay_flow<false, kFlowShortW>), dim3((unsigned)gs), dim3(64 * kFlowShortW), 0, stream,
                               w, flow_ctl, flow_epoch, kf);
            if (order == 2) long_launch();
            note(hipEventRecord(flow_ev[1], flow_stream), "hipEventRecord");
            note(hipStreamWaitEvent(stream, flow_ev[1], 0), "hipStreamWaitEvent");
        });
        hipLaunchKernelGGL(k_flow_report, dim3(1), dim3(64), 0, stream, w, flow_ctl, g_flow_giveup);
        if (g_bad_root) hipLaunchKernelGGL(k_bad_root, dim3(1), dim3(64), 0, stream, w);
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_replay_flow launch");
        return true;
    }

    void* temp(size_t bytes) {
        Temp* t = nullptr;
        for (auto& x : tmps)
            if (x.s == stream) t = &x;
        if (!t) {
            tmps.push_back(Temp{stream, nullptr, 0});
            t = &tmps.back();
        }
        if (bytes > t->n) {
            sync();
            if (t->p) (void)hipFree(t->p);
            t->p = alloc(bytes);
            t->n = t->p ? bytes : 0;
        }
        return t->p;
    }
    // exclusive prefix sum of each frame's segment [f*n, (f+1)*n): one scan over all frames, then
    // each frame's running total at its start is subtracted (one launch sequence, not one per frame)
    struct KFrameStart {
        const int* out;
        int* start;
        int64_t n;
        __device__ void operator()(int f, int64_t) const { start[f] = out[f * n]; }
    };
    struct KFrameRebase {
        int* out;
        const int* start;
        int64_t n;
        __device__ void operator()(int f, int64_t i) const { out[f * n + i] -= start[f]; }
    };
    void scan_excl(const int* in, int* out, int64_t n, int nf) { scan_excl_it(in, out, n, nf); }
    // as scan_excl, for segments whose sums are all `total` (a frame's MST edge counts: N - 1 for a connected
    // grid): subtracting it at every segment's last element makes the batch-wide sum segment-local, as the leaf
    // scan below does — no rebase pass. total < 0: unknown (scan_excl)
    struct FixedSum {
        const int* in;
        int64_t n;
        int total;
        __host__ __device__ int operator()(int64_t i) const { return in[i] - ((i + 1) % n == 0 ? total : 0); }
    };
    void scan_excl_total(const int* in, int* out, int64_t n, int nf, int total) {
        if (total < 0 || nf <= 1 || (int64_t)n * nf >= (int64_t)0x7FFFFFFF) {
            scan_excl_it(in, out, n, nf);
            return;
        }
        hipcub::CountingInputIterator<int64_t> ci(0);
        hipcub::TransformInputIterator<int, FixedSum, hipcub::CountingInputIterator<int64_t>> it(ci, FixedSum{in, n, total});
        scan_excl_it(it, out, n * nf, 1);
    }
    // leaf ranks in preorder: exclusive scan of (ord[q] < N) read through a transform iterator
    // (no flag array written by KOrd)
    struct IsLeaf {
        int N;
        __host__ __device__ int operator()(int x) const { return x < N ? 1 : 0; }
    };
    // a frame holds exactly N leaves, so subtracting N at every frame's last position makes the
    // batch-wide exclusive sum frame-local (it is 0 at each frame's first): no per-frame rebase pass
    struct LeafFlag {
        const int* ord;
        int64_t n;
        int N;
        __host__ __device__ int operator()(int64_t i) const {
            return (ord[i] < N ? 1 : 0) - ((i + 1) % n == 0 ? N : 0);  // -N at each frame's last
        }
    };
    void scan_excl_leaf(const int* ord, int* out, int64_t n, int nf, int64_t N) {
        if ((int64_t)n * nf < (int64_t)0x7FFFFFFF) {
            hipcub::CountingInputIterator<int64_t> ci(0);
            hipcub::TransformInputIterator<int, LeafFlag, hipcub::CountingInputIterator<int64_t>> it(
                ci, LeafFlag{ord, n, (int)N});
            scan_excl_it(it, out, n * nf, 1);  // the whole batch, already frame-local
            return;
        }
        hipcub::TransformInputIterator<int, IsLeaf, const int*> it(ord, IsLeaf{(int)N});
        scan_excl_it(it, out, n, nf);
    }
    template <class It>
    void scan_excl_it(It in, int* out, int64_t n, int nf) {
        const int64_t tot = n * nf;
        size_t bytes = 0;
        note(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, (int)tot, stream), "scan size");
        const size_t sb = (bytes + 255) & ~(size_t)255;
        char* t = (char*)temp(sb + sizeof(int) * (size_t)nf);
        note(hipcub::DeviceScan::ExclusiveSum(t, bytes, in, out, (int)tot, stream), "scan");
        if (nf > 1) {
            int* start = (int*)(t + sb);
            launch_on(stream, nf, 1, KFrameStart{out, start, n});
            launch_on(stream, nf, n, KFrameRebase{out, start, n});
        }
    }
    // stable LSD radix sort of (key, value) pairs by the 64-bit key, per frame (build_graph's edge list)
    void sort_pairs(unsigned long long* kin, unsigned long long* kout, unsigned* vin, unsigned* vout, int64_t n,
                    int nf, int) {
        for (int f = 0; f < nf; ++f) {
            size_t bytes = 0;
            note(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, kin + f * n, kout + f * n, vin + f * n, vout + f * n,
                                                    (int)n, 0, 64, stream),
                 "sort size");
            void* t = temp(bytes);
            note(hipcub::DeviceRadixSort::SortPairs(t, bytes, kin + f * n, kout + f * n, vin + f * n, vout + f * n,
                                                    (int)n, 0, 64, stream),
                 "sort");
        }
    }
    static int frame_bits(int nf) {
        int fb = 0;
        while ((1 << fb) < nf) ++fb;
        return fb;
    }
    // The whole batch's MST edges in one sort when the frame id fits above the value_bits index bits
    // (KMstEmit then writes it there): pairs by the 64-bit weight key, then the values alone, stably,
    // by the frame bits — a 4-byte keys-only pass; the weights stay in global key order.
    static bool mst_packed(int64_t n, int nf, int value_bits) {
        return nf > 1 && value_bits + frame_bits(nf) <= 32 && n * nf < ((int64_t)1 << 31);
    }
    // Kruskal order of each frame's MST edges into w.val_out (values of frame f at [f n, (f + 1) n)).
    // Packed: w.EU (written later by KEdgeInit) is the scratch between the two passes.
    static int sort_k32() { return g_sort_k32; }  // KMstEmit's 32-bit keys for the packed sort (0: 64-bit)
    static int sort_k32_bits() { return dofs::sort_k32_bits(); }
    // the batch sort's (u32 key, u32 value) pair passes and the frame pass, through rocPRIM's onesweep with
    // SortCfg's block shape
    hipError_t sort_pairs32(void* t, size_t& b, const unsigned* kin, unsigned* kout, const unsigned* vin, unsigned* vout,
                            int n, int bit0, int bit1) {
        return rocprim::radix_sort_pairs<SortCfg>(t, b, kin, kout, vin, vout, (size_t)n, (unsigned)bit0, (unsigned)bit1,
                                                  stream);
    }
    hipError_t sort_keys32(void* t, size_t& b, const unsigned* kin, unsigned* kout, int n, int bit0, int bit1) {
        return rocprim::radix_sort_keys<SortCfg>(t, b, kin, kout, (size_t)n, (unsigned)bit0, (unsigned)bit1, stream);
    }
    void sort_mst(Ws& w, int64_t n, int nf, int value_bits, bool packed) {
        if (!packed) {
            sort_pairs(w.key_in, w.key_out, w.val_in, w.val_out, n, nf, value_bits);
            return;
        }
        const int fb = frame_bits(nf);
        const int tot = (int)(n * nf);
        if (g_sort_k32 > 0) {  // 32-bit keys (dofs_sortfix.h): four digits of (u32, u32) pairs, then the fix-up
            const unsigned* k32_in = reinterpret_cast<const unsigned*>(w.key_in);
            unsigned* k32_out = reinterpret_cast<unsigned*>(w.key_out);
            unsigned* vmid = reinterpret_cast<unsigned*>(w.EU);
            size_t b1 = 0, b2 = 0;
            const int kb = sort_k32_bits();
            note(sort_pairs32(nullptr, b1, k32_in, k32_out, w.val_in, vmid, tot, 0, kb), "sort size");
            note(sort_keys32(nullptr, b2, vmid, w.val_out, tot, value_bits, value_bits + fb), "sort size");
            void* t = temp(std::max(b1, b2));
            note(sort_pairs32(t, b1, k32_in, k32_out, w.val_in, vmid, tot, 0, kb), "sort");
            if (g_sort_fix) sort_fixup32(w, vmid, tot, value_bits);
            if (g_sort_dump[0]) {  // diagnosis: 32-bit keys (4 bytes each) and values after the fix-up
                const size_t m = (size_t)std::min<int64_t>(tot, g_sort_dump_cap);
                note(hipMemcpyAsync(g_sort_dump[0], k32_out, 4 * m, hipMemcpyDeviceToDevice, stream), "dump");
                note(hipMemcpyAsync(g_sort_dump[1], vmid, 4 * m, hipMemcpyDeviceToDevice, stream), "dump");
                g_sort_dump[0] = g_sort_dump[1] = nullptr;
            }
            note(sort_keys32(t, b2, vmid, w.val_out, tot, value_bits, value_bits + fb), "sort frames");
            return;
        }
        const int cut = g_sort_cut;
        unsigned* vmid = reinterpret_cast<unsigned*>(w.EU);
        size_t b1 = 0, b2 = 0;
        // bits [cut, 63) when truncated: the weights are >= 0 (a sign bit raises the fix-up's fallback), and
        // this image's rocPRIM sorts [cut > 0, 64) of u64 keys wrongly on its merge-sort path (2k .. 1M
        // pairs; tools/sort_check.hip) while [cut, 63) is right at every size
        const int endb = cut > 0 ? 63 : 64;
        note(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, w.key_in, w.key_out, w.val_in, vmid, tot, cut, endb, stream),
             "sort size");
        note(hipcub::DeviceRadixSort::SortKeys(nullptr, b2, vmid, w.val_out, tot, value_bits, value_bits + fb, stream),
             "sort size");
        void* t = temp(std::max(b1, b2));
        note(hipcub::DeviceRadixSort::SortPairs(t, b1, w.key_in, w.key_out, w.val_in, vmid, tot, cut, endb, stream),
             "sort");
        if (cut > 0 && g_sort_fix) sort_fixup(w, vmid, tot, cut);
        if (g_sort_dump[0]) {  // diagnosis: the batch order after the fix-up (dofs_debug_sort_dump)
            const size_t m = (size_t)std::min<int64_t>(tot, g_sort_dump_cap);
            note(hipMemcpyAsync(g_sort_dump[0], w.key_out, 8 * m, hipMemcpyDeviceToDevice, stream), "dump");
            note(hipMemcpyAsync(g_sort_dump[1], vmid, 4 * m, hipMemcpyDeviceToDevice, stream), "dump");
            g_sort_dump[0] = g_sort_dump[1] = nullptr;
        }
        note(hipcub::DeviceRadixSort::SortKeys(t, b2, vmid, w.val_out, tot, value_bits, value_bits + fb, stream),
             "sort frames");
    }
    // dofs_sortfix.h, 32-bit keys: the mixed groups sorted by (recomputed full key, value); key_in / val_in
    // (dead after the pair sort) the scratch, key_out's storage the fallback's full keys
    void sort_fixup32(Ws& w, unsigned* vmid, int64_t tot, int vb) {
        SortFix32 s{reinterpret_cast<const unsigned*>(w.key_out), vmid, w.key_out, w.key_in, w.val_in, w.blur, w.d,
                    vb, w.single ? 0x3FFFFFFFu : ~0u, w.ctr + C_SORTFIX, tot};
        const int64_t cap = grid_cap() > 0 ? grid_cap() : 8192;
        const unsigned gx = (unsigned)std::min<int64_t>((tot + kFixBlock - 1) / kFixBlock, cap);
        int lgs = 0;
        while (((int64_t)1 << lgs) < tot) ++lgs;
        lgs += lgs & 1;  // an even number of merge passes ends in (k64, vmid)
        timed("k_sortfix", [&] {
            hipLaunchKernelGGL(k_sortfix32_local, dim3(gx), dim3(kFixBlock), 0, stream, s);
            int cus = 256;
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
            // the fallback (both return at once unless the flag is up): full keys, then the merge sort
            hipLaunchKernelGGL(k_sortfix32_keys, dim3(2 * cus), dim3(kFixBlock), 0, stream, s);
            hipLaunchKernelGGL(k_sortfix_merge, dim3(2 * cus), dim3(kFixBlock), 0, stream,
                               SortFix{w.key_out, vmid, w.key_in, w.val_in, w.ctr + C_SORTFIX, tot, 1, s.vm}, lgs);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "sort fix-up launch");
    }
    // dofs_sortfix.h: the groups of equal truncated keys sorted by the full key (val_out, written by the
    // frame pass next, holds the lists; key_in / val_in, dead after the pair sort, the scratch)
    void sort_fixup(Ws& w, unsigned* vmid, int64_t tot, int cut) {
        SortFix s{w.key_out, vmid, w.key_in, w.val_in, w.ctr + C_SORTFIX, tot, cut, w.single ? 0x3FFFFFFFu : ~0u};
        const int64_t cap = grid_cap() > 0 ? grid_cap() : 8192;
        const unsigned gx = (unsigned)std::min<int64_t>((tot + kFixBlock - 1) / kFixBlock, cap);
        int lgs = 0;
        while (((int64_t)1 << lgs) < tot) ++lgs;
        lgs += lgs & 1;  // an even number of merge passes ends in (key_out, vmid)
        timed("k_sortfix", [&] {
            hipLaunchKernelGGL(k_sortfix_local, dim3(gx), dim3(kFixBlock), 0, stream, s);
            // (returns at once unless the flag is up; two blocks per CU, all resident for its barrier)
            int cus = 256;
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
            hipLaunchKernelGGL(k_sortfix_merge, dim3(2 * cus), dim3(kFixBlock), 0, stream, s, lgs);
        });
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "sort fix-up launch");
    }
};

}  // namespace dofs

#ifdef DOFS_KRT_TIMING
// Measurement build only: the KRT phase times accumulated since the last call (microseconds), then reset.
extern "C" int dofs_debug_krt_timing(double* out_us, int n) {
    unsigned long long v[20] = {0};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(dofs::g_kt), sizeof(v)) != hipSuccess) return -1;
    const unsigned long long z[20] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(dofs::g_kt), z, sizeof(z));
    for (int i = 0; i < n && i < 20; ++i) out_us[i] = (double)v[i] / 100.0;  // 100 MHz wall clock
    return 20;
}
#endif


// Test knob: the low key bits the batch MST sort leaves to the fix-up (dofs_sortfix.h), 0 .. 48
// (0: the full 64-bit sort; 48: 16-bit keys, every weight class a mixed group: the fallback's test).
// cut < 0 only reads it. Returns the previous value. The fix-up's counters: frame 0's C_SORTFIX .. + 2.
extern "C" int dofs_debug_sort_cut(int cut) {
    const int old = dofs::g_sort_cut;
    if (cut >= 0 && cut <= 48) dofs::g_sort_cut = cut;
    return old;
}
// Test knob: the mantissa bits of the packed sort's 32-bit keys (dofs_sortfix.h), 4 .. 30, or 0 for the
// 64-bit keys (then dofs_debug_sort_cut applies); m < 0 only reads it. Returns the previous value.
// Few bits make long mixed groups: the fallback's test.
extern "C" int dofs_debug_sort_k32(int m) {
    const int old = dofs::g_sort_k32;
    if (m == 0 || (m >= 4 && m <= 30)) dofs::g_sort_k32 = m;
    return old;
}
// Test knob: the exponent bits of those keys, 1 .. 8 (m + e < 32: a key of m + e bits, fewer sort digits),
// or 0 for 32 - m; e < 0 only reads it. Returns the previous value.
extern "C" int dofs_debug_sort_k32e(int e) {
    const int old = dofs::g_sort_k32e;
    if (e >= 0 && e <= 8) dofs::g_sort_k32e = e;
    return old;
}
// Diagnosis only: fix-up on / off (the truncated order is not Kruskal's: results differ), and a copy of
// the next packed batch's sorted (key, value) pairs — at most cap — into device buffers.
extern "C" void dofs_debug_sort_fix(int on) { dofs::g_sort_fix = on != 0; }
// Test knob: the batches issued while on = 1 report a replay give-up (C_FLOWERR) although their replay
// completed — the error path through the accessors (records copy, fetch, gather). Returns the previous value.
extern "C" int dofs_debug_flow_giveup(int on) {
    const int old = dofs::g_flow_giveup;
    if (on >= 0) dofs::g_flow_giveup = on ? 1 : 0;
    return old;
}
// Test knob: the batches issued while on = 1 have an out-of-range union-find root written into every frame's
// last merge record after the replay (k_bad_root) — the scoring's guards must refuse it (DOFS_ERR_INVALID_RESULT
// from every accessor) instead of using it as an index. Returns the previous value.
extern "C" int dofs_debug_bad_root(int on) {
    const int old = dofs::g_bad_root;
    if (on >= 0) dofs::g_bad_root = on ? 1 : 0;
    return old;
}
// Test knob: constant-key chunks of the long-path replay (dofs_dataflow.h g_keyfast; 1 = on, the default).
// Returns the previous value; on < 0 only reads it.
extern "C" int dofs_debug_replay_keyfast(int on) {
    const int old = dofs::g_keyfast;
    if (on >= 0) dofs::g_keyfast = on ? 1 : 0;
    return old;
}
// Test knob: the LDS KRT's depths below 32 merges as one register window pass (1, the default) or as
// union-find depths (0), g_deep_wave. Returns the previous value; on < 0 only reads it.
extern "C" int dofs_debug_krt_deep_wave(int on) {
    const int old = dofs::g_deep_wave;
    if (on >= 0) dofs::g_deep_wave = on ? 1 : 0;
    return old;
}
// Test knob: k_dnc_compress's wave skew (0 = off), see g_dnc_skew. Returns 0 or a HIP error code.
extern "C" int dofs_debug_dnc_skew(int skew) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(dofs::g_dnc_skew), &skew, sizeof(int));
}
// Test entry: the fix-up (k_sortfix_local, then k_sortfix_merge when its flag is up) over a caller's n
// device pairs already sorted stably by key bits [cut, 64) — keys u64, values u32 (distinct) — in place,
// with d_k2 / d_v2 (n each) as the fallback's scratch and d_ctr (3 zeroed int32) receiving the counters
// (moved pairs, fallback flag, barrier). Synchronous on the null stream; returns 0 or a HIP error code.
extern "C" int dofs_debug_sortfix_run(void* d_keys, void* d_vals, void* d_k2, void* d_v2, int64_t n, int cut,
                                      int* d_ctr) {
    using namespace dofs;
    if (n <= 0 || cut < 1 || cut > 48 || !d_keys || !d_vals || !d_k2 || !d_v2 || !d_ctr) return (int)hipErrorInvalidValue;
    SortFix s{(unsigned long long*)d_keys, (unsigned*)d_vals, (unsigned long long*)d_k2, (unsigned*)d_v2, d_ctr, n, cut, ~0u};
    int lgs = 0;
    while (((int64_t)1 << lgs) < n) ++lgs;
    lgs += lgs & 1;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned gx = (unsigned)std::min<int64_t>((n + kFixBlock - 1) / kFixBlock, 8192);
    hipLaunchKernelGGL(k_sortfix_local, dim3(gx), dim3(kFixBlock), 0, nullptr, s);
    hipLaunchKernelGGL(k_sortfix_merge, dim3(2 * cus), dim3(kFixBlock), 0, nullptr, s, lgs);
    const hipError_t e = hipDeviceSynchronize();
    return e == hipSuccess ? (int)hipGetLastError() : (int)e;
}
// Test-only: the 32-bit keys' fix-up (k_sortfix32_local, then the fallback's full keys and merge sort) over
// n (32-bit key, value) pairs in truncated-key stable order. d_keys: 8 n bytes, the 32-bit keys in its
// first 4 n (the fallback overwrites it with full keys); values 4 p + k of the frames' edges, frame above
// bit vb; d_blur: B frames of H x W blurred flow (float2), the weights' source. d_ctr: 3 ints (moved,
// fallback flag, -).
extern "C" int dofs_debug_sortfix32_run(void* d_keys, void* d_vals, void* d_k2, void* d_v2, int64_t n, const void* d_blur,
                                        int B, int H, int W, int vb, int* d_ctr) {
    using namespace dofs;
    if (n <= 0 || B < 1 || H < 1 || W < 1 || vb < 3 || vb > 31 || !d_keys || !d_vals || !d_k2 || !d_v2 || !d_blur ||
        !d_ctr)
        return (int)hipErrorInvalidValue;
    Dims d{};
    d.H = H;
    d.W = W;
    d.N = (int64_t)H * W;
    d.M = d.N - 1;
    d.NL = d.N + d.M;
    d.B = B;
    d.nbr8 = 0;
    if (4 * d.N > ((int64_t)1 << vb)) return (int)hipErrorInvalidValue;
    SortFix32 s{(const unsigned*)d_keys, (unsigned*)d_vals, (unsigned long long*)d_keys, (unsigned long long*)d_k2,
                (unsigned*)d_v2, (const F2*)d_blur, d, vb, ~0u, d_ctr, n};
    int lgs = 0;
    while (((int64_t)1 << lgs) < n) ++lgs;
    lgs += lgs & 1;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned gx = (unsigned)std::min<int64_t>((n + kFixBlock - 1) / kFixBlock, 8192);
    hipLaunchKernelGGL(k_sortfix32_local, dim3(gx), dim3(kFixBlock), 0, nullptr, s);
    hipLaunchKernelGGL(k_sortfix32_keys, dim3(2 * cus), dim3(kFixBlock), 0, nullptr, s);
    hipLaunchKernelGGL(k_sortfix_merge, dim3(2 * cus), dim3(kFixBlock), 0, nullptr,
                       SortFix{(unsigned long long*)d_keys, (unsigned*)d_vals, (unsigned long long*)d_k2, (unsigned*)d_v2,
                               d_ctr, n, 1, s.vm},
                       lgs);
    const hipError_t e = hipDeviceSynchronize();
    return e == hipSuccess ? (int)hipGetLastError() : (int)e;
}
// Test knob: the dataflow replay's two worker launches (dofs_dataflow.h) side by side on two streams (0, the
// default), or one after the other on the stage's stream: 1 = long workers first, 2 = short workers first.
// Neither role waits for work the other launch has yet to produce, so every order completes. Returns the
// previous value; order < 0 only reads it.
extern "C" int dofs_debug_flow_order(int order) {
    const int old = dofs::g_flow_order;
    if (order >= 0 && order <= 2) dofs::g_flow_order = order;
    return old;
}
extern "C" void dofs_debug_sort_dump(void* d_keys, void* d_vals, int64_t cap) {
    dofs::g_sort_dump[0] = d_keys;
    dofs::g_sort_dump[1] = d_vals;
    dofs::g_sort_dump_cap = cap;
}

using DofsBackend = dofs::HipBackend;
#include "dofs_cabi.inc.h"

// Inspection: the dataflow replay's worker counts (waves) — long-path workers (DOFS_FLOW_LONG) and short ones.
extern "C" int dofs_flow_workers(dofs_ctx* ctx, int* long_waves, int* short_waves) {
    if (!ctx) return DOFS_ERR_INVALID_ARG;
    if (long_waves) *long_waves = ctx->be.flow_long_workers();
    if (short_waves) *short_waves = dofs::HipBackend::flow_grid();
    return 0;
}

// Diagnosis only (tools/flow_dump.py): device pointers of the last batch's workspace arrays, after a sync:
// out = {cur, ptop, list_long, In, the path-top state words (Rv + 24 bytes: stride 32), ord, lite, ctr, Rv, pre,
// flow control block, bw, lu, lv, SZ, hls, hlB, lscan}, and the batch's B, N, NL in dims.
extern "C" int dofs_debug_ws_ptrs(dofs_ctx* ctx, unsigned long long* out, long long* dims) {
    if (!ctx || !out || !dims || !ctx->have_batch()) return DOFS_ERR_INVALID_ARG;
    const int slot = ctx->last_slot();
    ctx->drain();
    const dofs::Ws& w = ctx->pipe(slot).w;
    const void* p[18] = {w.cur, w.ptop, w.list_long, w.In, reinterpret_cast<const char*>(w.Rv) + offsetof(dofs::RepVal, pad0), w.ord, w.lite, w.ctr, w.Rv,
                         w.pre, ctx->be.flow_ctl, w.bw, w.lu, w.lv, w.SZ, w.hls, w.hlB, w.lscan};
    for (int i = 0; i < 18; ++i) out[i] = (unsigned long long)(uintptr_t)p[i];
    dims[0] = w.d.B;
    dims[1] = w.d.N;
    dims[2] = w.d.NL;
    return DOFS_OK;
}

// Measurement: the context's last dataflow replay launch's anatomy (dofs_dataflow.h FlowStat, kept in the
// context's control block), after draining the context. Returns FS_N or a negative error.
extern "C" int dofs_debug_flow_stats(dofs_ctx* ctx, unsigned long long* out, int n) {
    if (!ctx || !out || !ctx->be.flow_ctl) return -1;
    ctx->drain();
    unsigned long long v[dofs::FS_N * dofs::kFsStride] = {0};
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpy(v, ctx->be.flow_ctl + dofs::FC_FS, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (int i = 0; i < n && i < dofs::FS_N; ++i) out[i] = v[i * dofs::kFsStride];
    return dofs::FS_N;
}

// ---- optical flow (upstream stage; HIP build only) ---------------------------------------------
#include "dofs_flow.h"

namespace {
dofs::flow::Engine* flow_engine(dofs_ctx* ctx) {
    if (!ctx->flow_engine) ctx->flow_engine = std::make_shared<dofs::flow::Engine>();
    return static_cast<dofs::flow::Engine*>(ctx->flow_engine.get());
}

// main1's loop (segment.cpp:209-269) over a device-resident clip: gray, Farneback, segment and overlay
// of consecutive frame pairs, in chunks of `batch` pairs. Chunk c runs its Farneback on flow stream
// sf[c % 2] (own Farneback workspace and flow buffer), submits the chunk to the context's two-stage
// segment pipeline from that stream, and its overlay + box-record copy run on stream so once the
// chunk's segmentation is done — so chunk c+1's Farneback overlaps chunk c's graph stage, and the
// overlay of chunk c overlaps chunk c+1's stages.
struct VideoState {
    unsigned char* gray = nullptr;
    size_t gray_bytes = 0;
    float* flow[2] = {nullptr, nullptr};
    size_t flow_bytes = 0;
    dofs::flow::Engine eng[2];
    hipStream_t sf[2] = {nullptr, nullptr};
    hipStream_t so = nullptr;
    hipEvent_t ev_in = nullptr, ev_gray = nullptr, ev_end[3] = {nullptr, nullptr, nullptr};
    hipEvent_t ev_ov[dofs::Context<DofsBackend>::kSlots] = {};
    bool ok = true;
    explicit VideoState(int device) {
        (void)hipSetDevice(device);
        for (auto* st : {&sf[0], &sf[1], &so}) ok = ok && hipStreamCreateWithFlags(st, hipStreamNonBlocking) == hipSuccess;
        for (auto* e : {&ev_in, &ev_gray, &ev_end[0], &ev_end[1], &ev_end[2]})
            ok = ok && hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess;
        for (auto& e : ev_ov) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    }
    ~VideoState() {
        for (auto st : {sf[0], sf[1], so})
            if (st) (void)hipStreamSynchronize(st);
        if (gray) (void)hipFree(gray);
        for (auto f : flow)
            if (f) (void)hipFree(f);
        for (auto st : {sf[0], sf[1], so})
            if (st) (void)hipStreamDestroy(st);
        for (auto e : {ev_in, ev_gray, ev_end[0], ev_end[1], ev_end[2]})
            if (e) (void)hipEventDestroy(e);
        for (auto e : ev_ov)
            if (e) (void)hipEventDestroy(e);
    }
    bool reserve(size_t gb, size_t fb) {
        for (auto st : {sf[0], sf[1], so}) (void)hipStreamSynchronize(st);
        if (gb > gray_bytes) {
            if (gray) (void)hipFree(gray);
            gray = nullptr;
            gray_bytes = hipMalloc(&gray, gb) == hipSuccess ? gb : 0;
            if (!gray_bytes) return false;
        }
        if (fb > flow_bytes) {
            for (auto& f : flow) {
                if (f) (void)hipFree(f);
                f = nullptr;
            }
            flow_bytes = (hipMalloc(&flow[0], fb) == hipSuccess && hipMalloc(&flow[1], fb) == hipSuccess) ? fb : 0;
            if (!flow_bytes) return false;
        }
        return true;
    }
};

int video_clip(dofs_ctx* ctx, const unsigned char* d_bgr, int n, int H, int W, int batch, const float persp[9],
               const float inv[9], const float inv_upper[27], const dofs_params* params,
               const dofs_flow_params& fp, unsigned char* d_overlay, int* d_counts, dofs_box_record* d_records,
               int per_frame, hipStream_t caller) {
    if (!ctx->video) ctx->video = std::make_shared<VideoState>(ctx->be.device);
    VideoState& v = *static_cast<VideoState*>(ctx->video.get());
    if (!v.ok) return ctx->fail(DOFS_ERR_DEVICE, "video streams");
    const int64_t N = (int64_t)H * W;
    const int P = n - 1;  // frame pairs
    if (!v.reserve((size_t)n * N, sizeof(float) * 2 * (size_t)batch * N))
        return ctx->fail(DOFS_ERR_OOM, "video buffers");
    auto ck = [&](hipError_t e) { return e == hipSuccess; };
    bool ok = ck(hipEventRecord(v.ev_in, caller));
    for (auto st : {v.sf[0], v.sf[1], v.so}) ok = ok && ck(hipStreamWaitEvent(st, v.ev_in, 0));
    const int64_t px = (int64_t)n * N;
    hipLaunchKernelGGL(dofs::flow::k_bgr_gray, dim3((unsigned)std::min<int64_t>((px + 255) / 256, 16384)), dim3(256),
                       0, v.sf[0], d_bgr, px, v.gray);
    ok = ok && ck(hipGetLastError()) && ck(hipEventRecord(v.ev_gray, v.sf[0])) &&
         ck(hipStreamWaitEvent(v.sf[1], v.ev_gray, 0));
    if (!ok) return ctx->fail(DOFS_ERR_DEVICE, "video setup");
    const int nslots = ctx->nslots;
    std::vector<bool> ov_rec(nslots, false);
    for (int i = 0, c = 0; i < P; i += batch, ++c) {
        const int bc = std::min(batch, P - i);
        const int k = c & 1;
        hipStream_t st = v.sf[k];
        const int slot = ctx->slot_of(ctx->nbatch);
        // the workspace this chunk takes was last read by an overlay / record copy on v.so
        if (ov_rec[slot] && !ck(hipStreamWaitEvent(st, v.ev_ov[slot], 0))) return ctx->fail(DOFS_ERR_DEVICE, "wait");
        int rc = v.eng[k].run(v.gray + (int64_t)i * N, v.gray + (int64_t)(i + 1) * N, bc, H, W, fp, v.flow[k], st);
        if (rc != DOFS_OK) return ctx->fail(rc, v.eng[k].err);
        ctx->be.set_stream(st);  // api_run leaves st ordered after the chunk's graph stage (flow consumed)
        rc = dofs::api_run(ctx, (const dofs::F2*)v.flow[k], N, bc, H, W, persp, inv, inv_upper, params);
        if (rc != DOFS_OK) return rc;
        const int64_t id = ctx->nbatch - 1;
        ctx->be.set_stream(v.so);
        if (d_overlay) {
            rc = dofs::api_overlay(ctx, id, d_bgr + (int64_t)(i + 1) * N * 3, d_overlay + (int64_t)i * N * 3,
                                   false);
            if (rc != DOFS_OK) return rc;
        } else {
            ctx->join(id);
        }
        const dofs::Ws& w = ctx->pipe(slot).w;
        if (d_counts)
            ctx->be.copy2d(d_counts + i, sizeof(int), w.ctr + dofs::C_SNAP, sizeof(int) * dofs::kCounters, sizeof(int),
                           bc);
        const int kr = std::min(per_frame, w.snap_cap);
        if (d_records && kr > 0)
            ctx->be.copy2d(d_records + (int64_t)i * per_frame, sizeof(dofs_box_record) * per_frame, w.recs,
                           sizeof(dofs_box_record) * w.snap_cap, sizeof(dofs_box_record) * kr, bc);
        if (!ck(hipEventRecord(v.ev_ov[slot], v.so))) return ctx->fail(DOFS_ERR_DEVICE, "record");
        ov_rec[slot] = true;
    }
    ctx->be.set_stream(caller);
    hipStream_t all[3] = {v.sf[0], v.sf[1], v.so};
    for (int t = 0; t < 3; ++t)
        ok = ok && ck(hipEventRecord(v.ev_end[t], all[t])) && ck(hipStreamWaitEvent(caller, v.ev_end[t], 0));
    if (!ok) return ctx->fail(DOFS_ERR_DEVICE, "video join");
    return ctx->check();
}
}  // namespace

extern "C" {

void dofs_default_flow_params(dofs_flow_params* p) {
    if (!p) return;
    p->pyr_scale = 0.5;
    p->levels = 3;
    p->winsize = 15;
    p->iterations = 3;
    p->poly_n = 5;
    p->poly_sigma = 1.2;
    p->flags = 0;
}

int32_t dofs_farneback_batch_device(dofs_ctx* ctx, const uint8_t* d_prev, const uint8_t* d_next, int32_t B,
                                    int32_t H, int32_t W, const dofs_flow_params* params, float* d_flow,
                                    void* stream) {
    if (!ctx || !d_prev || !d_next || !d_flow || B <= 0 || H <= 0 || W <= 0) return DOFS_ERR_INVALID_ARG;
    dofs_flow_params p;
    dofs_default_flow_params(&p);
    if (params) p = *params;
    dofs::flow::Engine* e = flow_engine(ctx);
    const int rc = e->run(d_prev, d_next, B, H, W, p, d_flow, (hipStream_t)stream);
    if (rc != DOFS_OK) ctx->err = e->err;
    return rc;
}

int32_t dofs_farneback(dofs_ctx* ctx, const uint8_t* prev, const uint8_t* next, int32_t H, int32_t W,
                       size_t row_stride_bytes, const dofs_flow_params* params, float* flow_uv) {
    if (!ctx || !prev || !next || !flow_uv || H <= 0 || W <= 0) return DOFS_ERR_INVALID_ARG;
    const size_t st = row_stride_bytes ? row_stride_bytes : (size_t)W;
    const size_t n = (size_t)H * W;
    uint8_t* d = nullptr;
    float* df = nullptr;
    hipStream_t s = nullptr;
    int rc = DOFS_ERR_DEVICE;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess && hipMalloc(&d, 2 * n) == hipSuccess &&
        hipMalloc(&df, sizeof(float) * 2 * n) == hipSuccess &&
        hipMemcpy2DAsync(d, W, prev, st, W, H, hipMemcpyHostToDevice, s) == hipSuccess &&
        hipMemcpy2DAsync(d + n, W, next, st, W, H, hipMemcpyHostToDevice, s) == hipSuccess) {
        rc = dofs_farneback_batch_device(ctx, d, d + n, 1, H, W, params, df, s);
        if (rc == DOFS_OK &&
            (hipMemcpyAsync(flow_uv, df, sizeof(float) * 2 * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess))
            rc = DOFS_ERR_DEVICE;
    }
    if (rc == DOFS_ERR_DEVICE && ctx->err.empty()) ctx->err = "HIP error in dofs_farneback";
    if (s) (void)hipStreamSynchronize(s);
    if (d) (void)hipFree(d);
    if (df) (void)hipFree(df);
    if (s) (void)hipStreamDestroy(s);
    return rc;
}

int32_t dofs_video_clip_device(dofs_ctx* ctx, const uint8_t* d_bgr, int32_t n_frames, int32_t H, int32_t W,
                               int32_t batch, const float persp[9], const float inv[9], const float inv_upper[27],
                               const dofs_params* params, const dofs_flow_params* flow_params, uint8_t* d_overlay,
                               int32_t* d_counts, dofs_box_record* d_records, int32_t per_frame, void* stream) {
    if (!ctx || !d_bgr || n_frames < 1 || H <= 0 || W <= 0 || batch <= 0 || per_frame < 0 || !persp || !inv ||
        !inv_upper)
        return DOFS_ERR_INVALID_ARG;
    if (n_frames == 1) return DOFS_OK;  // no pair (main1 keeps the first frame as prev_frame)
    dofs_flow_params fp;
    dofs_default_flow_params(&fp);
    if (flow_params) fp = *flow_params;
    return video_clip(ctx, d_bgr, n_frames, H, W, batch, persp, inv, inv_upper, params, fp, d_overlay, d_counts,
                      d_records, per_frame, (hipStream_t)stream);
}

void dofs_bgr_to_gray(const uint8_t* bgr, int32_t H, int32_t W, size_t row_stride_bytes, uint8_t* gray) {
    const size_t st = row_stride_bytes ? row_stride_bytes : (size_t)W * 3;
    for (int32_t y = 0; y < H; ++y)
        for (int32_t x = 0; x < W; ++x) {
            const uint8_t* q = bgr + y * st + 3 * x;
            gray[(size_t)y * W + x] = (uint8_t)((q[0] * 1868 + q[1] * 9617 + q[2] * 4899 + (1 << 13)) >> 14);
        }
}

int32_t dofs_bgr_to_gray_device(const uint8_t* d_bgr, int64_t n_pixels, uint8_t* d_gray, void* stream) {
    if (!d_bgr || !d_gray || n_pixels < 0) return DOFS_ERR_INVALID_ARG;
    if (n_pixels == 0) return DOFS_OK;
    const unsigned gx = (unsigned)std::min<int64_t>((n_pixels + 255) / 256, 16384);
    hipLaunchKernelGGL(dofs::flow::k_bgr_gray, dim3(gx), dim3(256), 0, (hipStream_t)stream, d_bgr, n_pixels, d_gray);
    return hipGetLastError() == hipSuccess ? DOFS_OK : DOFS_ERR_DEVICE;
}

}  // extern "C"
