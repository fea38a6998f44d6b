// dofs_hip.hip — HIP/CDNA4 (gfx950) backend of the dense-optical-flow clustering + 3D-lifting path
// and the exported C-ABI (include/dofs.h). Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off.
//
// Every per-element body in dofs_kernels.h runs here as a grid-stride kernel over a 2-D grid
// (x: elements, y: frames of the batch), 256-thread workgroups (4 wave64s). Atomics are agent-scope
// (coherent across the 8 XCDs); union-find loads inside a launch use relaxed agent-scope atomic loads
// so a stale L1/L2 line can never be re-read forever (MI355X_MICROARCH.md §inter-workgroup visibility).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <array>
#include <string>
#include <vector>

#define DOFS_HD __device__
#define DOFS_HDM __host__ __device__

__device__ inline int dofs_ld(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline void dofs_st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline int dofs_cas(int* p, int expected, int v) {
    int old = expected;
    __hip_atomic_compare_exchange_strong(p, &old, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return old;
}
__device__ inline int dofs_exch(int* p, int v) { return atomicExch(p, v); }
__device__ inline void dofs_amin_u64(unsigned long long* p, unsigned long long v) { atomicMin(p, v); }
__device__ inline void dofs_amax_u64(unsigned long long* p, unsigned long long v) { atomicMax(p, v); }
__device__ inline void dofs_amin_u32(unsigned* p, unsigned v) { atomicMin(p, v); }
__device__ inline void dofs_amin(int* p, int v) { atomicMin(p, v); }
__device__ inline void dofs_amax(int* p, int v) { atomicMax(p, v); }
__device__ inline int dofs_aadd(int* p, int v) { return atomicAdd(p, v); }
__device__ inline void dofs_aor(int* p, int v) { atomicOr(p, v); }

#include "dofs_common.h"

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
__device__ inline void dofs_agg_min(int* base, int key, int val, bool act) { agg_minmax<false>(base, key, val, act); }

#include "dofs_kernels.h"

namespace dofs {

constexpr int kBlock = 256;

template <class F>
__global__ __launch_bounds__(kBlock) void k_generic(F f, int64_t n) {
    const int fr = blockIdx.y;
    const int64_t step = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += step) f(fr, i);
}


// ---------------------------------------------------------------------------------------------
// K5 (long heavy paths): two wave64s per path, one per mean channel (wave 0 also carries rank and
// root on the side). The float running mean of Forest::merge (graph.cpp:184-190) is a strictly
// sequential recurrence — mul, add (f32), cvt, mul (f64), cvt per merge — whose roundings must be
// replayed in Kruskal order; splitting the two channels over two SIMDs halves the issue load of the
// latency-bound chain (tools/replay_micro.hip: 41 vs 54 ns per step for one wave doing both).
// Per 64-step chunk every lane resolves one position's inputs (StepIn, plus the light child's
// replay output when it is a merge node) into LDS while the previous chunk is consumed; the chain
// reads step k with uniform LDS loads and writes step k's output to LDS; one coalesced store per
// chunk writes the outputs back by preorder position.
// ---------------------------------------------------------------------------------------------
struct LongStep {  // resolved inputs of one step for one wave (32 B)
    float fs;
    float wb;   // light child's weighted flow for this wave's channel
    int meta;   // StepIn meta | kLongOk (inputs ready)
    int pad;
    double r;
    int la;     // wave 0: light rank; wave 1: light bbox (x0 | y0 << 16)
    int lb;     // wave 0: light root; wave 1: light bbox (x1 | y1 << 16)
};
constexpr int kLongOk = 8;

__device__ inline int pack_xy(int x, int y) { return (x & 0xffff) | (y << 16); }

__device__ inline LongStep long_resolve(const Ws& w, int64_t lb, int p, int top, int round, int ch) {
    LongStep s;
    s.meta = 0;
    s.fs = 0.f;
    s.wb = 0.f;
    s.r = 0.0;
    s.la = 0;
    s.lb = 0;
    s.pad = 0;
    if (p < top) return s;
    const StepIn in = w.In[lb + p];
    s.fs = in.fs;
    s.r = in.r;
    s.meta = in.meta;
    if (in.meta & kStepDyn) {
        const int lq = in.lb;
        if (w.ready[lb + lq] >= round) return s;  // not ok: light child completes in a later round
        s.wb = (ch ? w.Rmy[lb + lq] : w.Rmx[lb + lq]) * (float)in.la;
        if (ch) {
            const B4 b = w.Rbb[lb + lq];
            s.la = pack_xy(b.x0, b.y0);
            s.lb = pack_xy(b.x1, b.y1);
        } else {
            s.la = w.Rrank[lb + lq];
            s.lb = w.Rroot[lb + lq];
        }
    } else {
        s.wb = ch ? in.wby : in.wbx;
        s.la = ch ? in.la : 0;     // pixel light child: rank 0 / bbox = its coordinates
        s.lb = ch ? in.la : in.lb;
    }
    s.meta |= kLongOk;
    return s;
}

__device__ void replay_long_path(const Ws& w, int f, int jj, int round, LongStep (*buf)[2][64], float (*res)[64],
                                 int (*resi)[64]) {
    const Dims& d = w.d;
    const int j = w.list_long[f * d.N + jj];
    int* curp = w.cur + f * d.N + j;
    const int wv = threadIdx.x >> 6;  // 0: mean x + rank + root, 1: mean y + bbox
    const int lane = threadIdx.x & 63;
    int q = *curp;
    const int top = w.ptop[f * d.N + j];
    __syncthreads();  // both waves have read the cursor before wave 0 may rewrite it
    if (q < 0) return;
    const int64_t lb = f * d.NL;
    float m = wv ? w.Rmy[lb + q + 1] : w.Rmx[lb + q + 1];
    int a0, a1, a2, a3;  // wave 0: rank, root; wave 1: bbox x0, y0, x1, y1
    if (wv == 0) {
        a0 = w.Rrank[lb + q + 1];
        a1 = w.Rroot[lb + q + 1];
        a2 = a3 = 0;
    } else {
        const B4 b = w.Rbb[lb + q + 1];
        a0 = b.x0;
        a1 = b.y0;
        a2 = b.x1;
        a3 = b.y1;
    }
    int cb = 0;
    LongStep mine = long_resolve(w, lb, q - lane, top, round, wv);
    buf[wv][cb][lane] = mine;
    for (;;) {
        const LongStep nx = long_resolve(w, lb, q - 64 - lane, top, round, wv);  // next chunk in flight
        // steps to run in this chunk: up to the first blocked position or through the path top
        const unsigned long long blocked = __ballot(!(mine.meta & kLongOk));
        const unsigned long long tops = __ballot((mine.meta & kLongOk) && (mine.meta & kStepTop));
        const int fb = blocked ? __ffsll((long long)blocked) - 1 : 64;
        const int ft = tops ? __ffsll((long long)tops) - 1 : 64;
        const int finished = ft < fb;
        const int n = finished ? ft + 1 : fb;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS staging has landed
        __builtin_amdgcn_wave_barrier();
        const LongStep* b = buf[wv][cb];
        if (wv == 0) {
#pragma unroll 8
            for (int k = 0; k < n; ++k) {
                const LongStep st = b[k];
                m = (float)((double)(m * st.fs + st.wb) * st.r);
                const int nroot = (st.meta & kStepB) ? (a0 > st.la ? a1 : st.lb) : (st.la > a0 ? st.lb : a1);
                a0 = (a0 == st.la) ? a0 + 1 : (a0 > st.la ? a0 : st.la);
                a1 = nroot;
                res[0][k] = m;
                resi[0][k] = a0;
                resi[1][k] = a1;
            }
        } else {
#pragma unroll 8
            for (int k = 0; k < n; ++k) {
                const LongStep st = b[k];
                m = (float)((double)(m * st.fs + st.wb) * st.r);
                const int lx0 = (int16_t)(st.la & 0xffff), ly0 = st.la >> 16;
                const int lx1 = (int16_t)(st.lb & 0xffff), ly1 = st.lb >> 16;
                a0 = lx0 < a0 ? lx0 : a0;
                a1 = ly0 < a1 ? ly0 : a1;
                a2 = lx1 > a2 ? lx1 : a2;
                a3 = ly1 > a3 ? ly1 : a3;
                res[1][k] = m;
                resi[2][k] = pack_xy(a0, a1);
                resi[3][k] = pack_xy(a2, a3);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        if (lane < n) {
            const int p = q - lane;
            if (wv) {
                w.Rmy[lb + p] = res[1][lane];
                const int lo = resi[2][lane], hi = resi[3][lane];
                B4 bb;
                bb.x0 = (int16_t)(lo & 0xffff);
                bb.y0 = (int16_t)(lo >> 16);
                bb.x1 = (int16_t)(hi & 0xffff);
                bb.y1 = (int16_t)(hi >> 16);
                w.Rbb[lb + p] = bb;
            } else {
                w.Rmx[lb + p] = res[0][lane];
                w.Rrank[lb + p] = resi[0][lane];
                w.Rroot[lb + p] = resi[1][lane];
            }
        }
        if (n < 64 || finished) {
            // both waves stop at the same step (same flags); the top's readiness is read only in
            // later rounds (kernel boundary), so either wave may publish it
            if (wv == 0 && lane == 0) {
                if (finished) {
                    w.ready[lb + q - n + 1] = round;
                    *curp = -1;
                } else {
                    *curp = q - n;
                }
            }
            __syncthreads();
            return;
        }
        q -= 64;
        cb ^= 1;
        mine = nx;
        buf[wv][cb][lane] = mine;
    }
}

__global__ __launch_bounds__(128) void k_replay_long(Ws w, int round) {
    __shared__ LongStep buf[2][2][64];
    __shared__ float res[2][64];
    __shared__ int resi[4][64];
    const int f = blockIdx.y;
    const int n = w.C(f)[C_LONG];
    for (int jj = blockIdx.x; jj < n; jj += gridDim.x) replay_long_path(w, f, jj, round, buf, res, resi);
}

struct HipBackend {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    hipError_t last = hipSuccess;
    std::string msg;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;

    static bool device_ok(int dev) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || dev >= n) return false;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
        return std::string(prop.gcnArchName).rfind("gfx950", 0) == 0;
    }

    explicit HipBackend(int dev) : device(dev) {
        note(hipSetDevice(dev), "hipSetDevice");
        note(hipStreamCreateWithFlags(&own, hipStreamNonBlocking), "hipStreamCreate");
        stream = own;
    }
    ~HipBackend() {
        for (auto e : pool) (void)hipEventDestroy(e);
        if (tmp) (void)hipFree(tmp);
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
    void set_stream(void* s) {
        (void)hipSetDevice(device);
        stream = s ? (hipStream_t)s : own;
    }

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
    void h2d(void* d, const void* h, size_t bytes) {
        note(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, stream), "hipMemcpyAsync H2D");
        sync();
    }
    void d2h(void* h, const void* d, size_t bytes) {
        note(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, stream), "hipMemcpyAsync D2H");
    }
    void sync() { note(hipStreamSynchronize(stream), "hipStreamSynchronize"); }
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

    template <class F>
    static int launch_on(hipStream_t s, int nf, int64_t n, const F& f) {
        if (n <= 0 || nf <= 0) return DOFS_OK;
        int64_t gx = (n + kBlock - 1) / kBlock;
        if (gx > 8192) gx = 8192;
        hipLaunchKernelGGL(k_generic<F>, dim3((unsigned)gx, (unsigned)nf), dim3(kBlock), 0, s, f, n);
        return hipGetLastError() == hipSuccess ? DOFS_OK : DOFS_ERR_DEVICE;
    }
    template <class F>
    static int launch_static(void* s, int nf, int64_t n, const F& f) {
        return launch_on((hipStream_t)s, nf, n, f);
    }
    template <class F>
    void launch(int nf, int64_t n, const F& f) {
        if (launch_on(stream, nf, n, f) != DOFS_OK) note(hipErrorLaunchFailure, "kernel launch");
    }

    void replay_long(const Ws& w, int round) {
        hipLaunchKernelGGL(k_replay_long, dim3(256u, (unsigned)w.d.B), dim3(128), 0, stream, w, round);
        if (hipGetLastError() != hipSuccess) note(hipErrorLaunchFailure, "k_replay_long launch");
    }

    void* temp(size_t bytes) {
        if (bytes > tmp_bytes) {
            sync();
            if (tmp) (void)hipFree(tmp);
            tmp = alloc(bytes);
            tmp_bytes = tmp ? bytes : 0;
        }
        return tmp;
    }
    // exclusive prefix sum of each frame's segment [f*n, (f+1)*n)
    void scan_excl(const int* in, int* out, int64_t n, int nf) {
        for (int f = 0; f < nf; ++f) {
            size_t bytes = 0;
            note(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in + f * n, out + f * n, (int)n, stream), "scan size");
            void* t = temp(bytes);
            note(hipcub::DeviceScan::ExclusiveSum(t, bytes, in + f * n, out + f * n, (int)n, stream), "scan");
        }
    }
    // stable LSD radix sort of (key, value) pairs by the 64-bit key, per frame
    void sort_pairs(const unsigned long long* kin, unsigned long long* kout, const unsigned* vin, unsigned* vout,
                    int64_t n, int nf) {
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
};

}  // namespace dofs

using DofsBackend = dofs::HipBackend;
#include "dofs_cabi.inc.h"
