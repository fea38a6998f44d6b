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
template <class B4>
__device__ inline void dofs_agg_size_bbox(int* cs, B4* bb, int key, int val, const B4& b, bool act) {
    const unsigned long long present = __ballot(1);
    const unsigned long long on = __ballot(act);
    if (!on) return;
    bool done = false;
    if (present == ~0ull) {
        const int leader = __ffsll((long long)on) - 1;
        const int k0 = __shfl(key, leader, 64);
        const bool same = act && key == k0;
        const int s = wave_reduce(same ? val : 0, [](int a, int c) { return a + c; });
        const int x0 = wave_reduce(same ? b.x0 : 0x7fffffff, [](int a, int c) { return a < c ? a : c; });
        const int y0 = wave_reduce(same ? b.y0 : 0x7fffffff, [](int a, int c) { return a < c ? a : c; });
        const int x1 = wave_reduce(same ? b.x1 : -1, [](int a, int c) { return a > c ? a : c; });
        const int y1 = wave_reduce(same ? b.y1 : -1, [](int a, int c) { return a > c ? a : c; });
        if (wave_lane() == leader) {
            atomicAdd(cs + k0, s);
            B4* a = bb + k0;
            if (__hip_atomic_load(&a->x0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > x0) atomicMin(&a->x0, x0);
            if (__hip_atomic_load(&a->y0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > y0) atomicMin(&a->y0, y0);
            if (__hip_atomic_load(&a->x1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < x1) atomicMax(&a->x1, x1);
            if (__hip_atomic_load(&a->y1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < y1) atomicMax(&a->y1, y1);
        }
        done = same;
    }
    if (act && !done) {
        atomicAdd(cs + key, val);
        B4* a = bb + key;
        atomicMin(&a->x0, b.x0);
        atomicMin(&a->y0, b.y0);
        atomicMax(&a->x1, b.x1);
        atomicMax(&a->y1, b.y1);
    }
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
// K5 (long heavy paths): one wave64 per path. The running union-find state (float mean x/y,
// rank, root) is a strictly sequential recurrence (Forest::merge, graph.cpp:184-190): its float
// roundings must be replayed in Kruskal order. Lane l gathers the inputs of position q-l (light
// child value, node size/bbox) for a 64-step chunk while the previous chunk is being consumed;
// every lane then runs the same 64 dependent steps, reading step k's inputs with v_readlane
// (wave-uniform scalars), and lane k keeps step k's result for one coalesced store.
// ---------------------------------------------------------------------------------------------
struct LongIn {
    int x;        // node at this position
    int ok;       // position on the path and its light child completed in an earlier round
    int top;      // this position is the path top
    int lside;    // light child is the end side (B)
    int lrank, lroot;
    float fs;     // (float) heavy-child size
    float wbx, wby;  // light child's weighted flow, float(m * (float)size)
    double r;     // 1 / (double)(size of the merged set)
    int sz;
    I4 bb;
};

__device__ inline LongIn long_load(const Ws& w, int64_t lb, int p, int top, int round) {
    LongIn in;
    in.ok = 0;
    in.top = 0;
    in.x = 0;
    in.sz = 0;
    if (p < top) return in;
    const int x = w.ord[lb + p];
    const int info = w.linfo[lb + p];
    const int lt = info & kLinfoId;
    const int rd = w.ready[lb + lt];
    const NodeVal lv = w.V[lb + lt];
    const int sz = w.SZ[lb + x];
    in.x = x;
    in.ok = rd < round;
    in.top = (info & kLinfoTop) ? 1 : 0;
    in.lside = (info & kLinfoB) ? 1 : 0;
    in.lrank = lv.rank;
    in.lroot = lv.root;
    in.fs = (float)(sz - lv.size);
    in.wbx = lv.mx * (float)lv.size;
    in.wby = lv.my * (float)lv.size;
    in.r = 1. / (double)sz;
    in.sz = sz;
    in.bb = w.BB[lb + x];
    return in;
}

__device__ inline int rl_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ inline float rl_f(float v, int k) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k)); }
__device__ inline double rl_d(double v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ void replay_long_path(const Ws& w, int f, int jj, int round) {
    const Dims& d = w.d;
    const int j = w.list_long[f * d.N + jj];
    int* curp = w.cur + f * d.N + j;
    int q = *curp;
    if (q < 0) return;
    const int top = w.ptop[f * d.N + j];
    const int lane = threadIdx.x;
    const int64_t lb = f * d.NL;
    const NodeVal run = w.V[lb + w.ord[lb + q + 1]];
    float mx = run.mx, my = run.my;
    int rank = run.rank, root = run.root;
    LongIn in = long_load(w, lb, q - lane, top, round);
    for (;;) {
        const LongIn nx = long_load(w, lb, q - 64 - lane, top, round);  // prefetch the next chunk
        float rx = 0.f, ry = 0.f;
        int rrank = 0, rroot = 0;
        int done = 64, finished = 0;
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            if (!rl_i(in.ok, k)) {
                done = k;
                break;
            }
            const float fs = rl_f(in.fs, k);
            const float tx = mx * fs, ty = my * fs;
            const float ux = tx + rl_f(in.wbx, k), uy = ty + rl_f(in.wby, k);
            const double r = rl_d(in.r, k);
            mx = (float)((double)ux * r);
            my = (float)((double)uy * r);
            const int lrank = rl_i(in.lrank, k), lroot = rl_i(in.lroot, k);
            // root = rank(A) > rank(B) ? root(A) : root(B); A = start side (graph.cpp:177-182)
            const int nroot = rl_i(in.lside, k) ? (rank > lrank ? root : lroot) : (lrank > rank ? lroot : root);
            rank = (rank == lrank) ? rank + 1 : (rank > lrank ? rank : lrank);
            root = nroot;
            if (lane == k) {
                rx = mx;
                ry = my;
                rrank = rank;
                rroot = root;
            }
            if (rl_i(in.top, k)) {
                done = k + 1;
                finished = 1;
                break;
            }
        }
        if (lane < done) {
            NodeVal v;
            v.mx = rx;
            v.my = ry;
            v.size = in.sz;
            v.root = rroot;
            v.x0 = (int16_t)in.bb.x0;
            v.y0 = (int16_t)in.bb.y0;
            v.x1 = (int16_t)in.bb.x1;
            v.y1 = (int16_t)in.bb.y1;
            v.rank = rrank;
            v.pad = 0;
            w.V[lb + in.x] = v;
            if (finished && lane == done - 1) w.ready[lb + in.x] = round;
        }
        if (finished) {
            if (lane == 0) *curp = -1;
            return;
        }
        if (done < 64) {
            if (lane == 0) *curp = q - done;
            return;
        }
        q -= 64;
        in = nx;
    }
}

__global__ __launch_bounds__(64) void k_replay_long(Ws w, int round) {
    const int f = blockIdx.y;
    const int n = w.C(f)[C_LONG];
    for (int jj = blockIdx.x; jj < n; jj += gridDim.x) replay_long_path(w, f, jj, round);
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
        hipLaunchKernelGGL(k_replay_long, dim3(1024u, (unsigned)w.d.B), dim3(64), 0, stream, w, round);
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
