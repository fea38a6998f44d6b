// Random 16-byte and 8-byte gathers from a buffer far larger than the L2s (the KRT sweep's union-find
// hops, KPathInit's pixel-flow reads): does the load's cache policy change the size of the L2's memory
// requests (TCC_EA0_RDREQ_{32B,64B,128B}) and the gather rate? Flavours: plain, nt (__builtin_nontemporal_load),
// sc1 (agent scope), sc0 sc1 (system scope). Two forms per flavour: independent loads (throughput, 2^26 lanes,
// one load each) and dependent hops (latency: each lane follows 16 hops of a random permutation cycle).
// Prints one line per kernel (ms, and the kernel's name for the rocprofv3 --pmc pass that counts requests).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/gather_micro tools/gather_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr unsigned long long kRecs = (4ull << 30) / 16;  // 4 GiB of 16-byte records

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

template <int F>
__device__ __forceinline__ int4 ld16(const int4* p) {
    if constexpr (F == 0) return *p;
    if constexpr (F == 1) {
        typedef int i4 __attribute__((ext_vector_type(4)));
        const i4 v = __builtin_nontemporal_load(reinterpret_cast<const i4*>(p));
        return make_int4(v.x, v.y, v.z, v.w);
    }
    if constexpr (F == 2) {  // agent scope: two 8-byte sc1 loads (no 16-byte atomic load)
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_int4((int)a, (int)(a >> 32), (int)b, (int)(b >> 32));
    }
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return make_int4((int)a, (int)(a >> 32), (int)b, (int)(b >> 32));
}

// independent random loads: one 16-byte record per lane
template <int F>
__global__ void gather16(const int4* buf, int* out, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const int4 v = ld16<F>(buf + mix(i ^ ((unsigned long long)seed << 40)) % kRecs);
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x7fffffff) out[0] = 1;  // (never: keeps the load)
}
// independent random 8-byte loads (a pixel's blurred flow)
template <int F>
__global__ void gather8(const int2* buf, int* out, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const int2* p = buf + mix(i ^ ((unsigned long long)seed << 40)) % (2 * kRecs);
    int2 v;
    if constexpr (F == 0) v = *p;
    if constexpr (F == 1) {
        typedef int i2 __attribute__((ext_vector_type(2)));
        const i2 u = __builtin_nontemporal_load(reinterpret_cast<const i2*>(p));
        v = make_int2(u.x, u.y);
    }
    if constexpr (F >= 2) {
        const unsigned long long a = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                                       F == 2 ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_SYSTEM);
        v = make_int2((int)a, (int)(a >> 32));
    }
    if ((v.x ^ v.y) == 0x7fffffff) out[0] = 1;
}
// dependent hops: x = rec[x].x, 16 times (the records hold a random successor)
template <int F>
__global__ void chase16(const int4* buf, int* out, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    unsigned x = (unsigned)(mix(i ^ ((unsigned long long)seed << 40)) % kRecs);
    int acc = 0;
    for (int h = 0; h < 16; ++h) {
        const int4 v = ld16<F>(buf + x);
        acc ^= v.y;
        x = (unsigned)v.x;
    }
    if (acc == 0x7fffffff) out[0] = (int)x;
}

__global__ void init(int4* buf) {
    for (unsigned long long r = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; r < kRecs;
         r += (unsigned long long)gridDim.x * blockDim.x)
        buf[r] = make_int4((int)(mix(r * 7 + 3) % kRecs), (int)r, 0, 1);
}

int main() {
    int4* buf = nullptr;
    int* out = nullptr;
    if (hipMalloc(&buf, kRecs * 16) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipLaunchKernelGGL(init, dim3(8192), dim3(256), 0, 0, buf);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const unsigned n = 1u << 26, T = 256, nc = 1u << 20;
    const char* fl[4] = {"plain", "nt", "sc1", "sc0sc1"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int f = 0; f < 4; ++f) {
            float ms[3];
            for (int k = 0; k < 3; ++k) {
                (void)hipEventRecord(a, 0);
                if (k == 0) {
                    if (f == 0) hipLaunchKernelGGL(gather16<0>, dim3(n / T), dim3(T), 0, 0, buf, out, rep);
                    if (f == 1) hipLaunchKernelGGL(gather16<1>, dim3(n / T), dim3(T), 0, 0, buf, out, rep);
                    if (f == 2) hipLaunchKernelGGL(gather16<2>, dim3(n / T), dim3(T), 0, 0, buf, out, rep);
                    if (f == 3) hipLaunchKernelGGL(gather16<3>, dim3(n / T), dim3(T), 0, 0, buf, out, rep);
                } else if (k == 1) {
                    const int2* b2 = reinterpret_cast<const int2*>(buf);
                    if (f == 0) hipLaunchKernelGGL(gather8<0>, dim3(n / T), dim3(T), 0, 0, b2, out, rep);
                    if (f == 1) hipLaunchKernelGGL(gather8<1>, dim3(n / T), dim3(T), 0, 0, b2, out, rep);
                    if (f == 2) hipLaunchKernelGGL(gather8<2>, dim3(n / T), dim3(T), 0, 0, b2, out, rep);
                    if (f == 3) hipLaunchKernelGGL(gather8<3>, dim3(n / T), dim3(T), 0, 0, b2, out, rep);
                } else {
                    if (f == 0) hipLaunchKernelGGL(chase16<0>, dim3(nc / T), dim3(T), 0, 0, buf, out, rep);
                    if (f == 1) hipLaunchKernelGGL(chase16<1>, dim3(nc / T), dim3(T), 0, 0, buf, out, rep);
                    if (f == 2) hipLaunchKernelGGL(chase16<2>, dim3(nc / T), dim3(T), 0, 0, buf, out, rep);
                    if (f == 3) hipLaunchKernelGGL(chase16<3>, dim3(nc / T), dim3(T), 0, 0, buf, out, rep);
                }
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                (void)hipEventElapsedTime(&ms[k], a, b);
            }
            printf("rep %d %-7s 2^26 random 16-B loads %.3f ms (%.2f G/s), 2^26 random 8-B loads %.3f ms (%.2f G/s), "
                   "2^20 lanes x 16 dependent 16-B hops %.3f ms (%.2f G hops/s)\n",
                   rep, fl[f], ms[0], n / ms[0] / 1e6, ms[1], n / ms[1] / 1e6, ms[2], 16.0 * nc / ms[2] / 1e6);
        }
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
