// Random 16-byte stores confined to a moving window (KPathInit's StepIn scatter, KLeafPos' position scatter):
// lane i of 2^26 stores to a random record of window i / (window / 16), so consecutive workgroups write the
// same window and the grid sweeps the buffer window by window. Does a window that fits the L2s or the
// memory-side cache turn the ~23 G random stores/s of a 4 GiB spread (partial_store_micro) into full-line
// writes? Windows 64 KiB ... 4 GiB; plain and nontemporal stores; and the same pattern as loads.
// Prints ms and G stores/s per case. Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/window_store_micro
// tools/window_store_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

constexpr unsigned long long kBytes = 4ull << 30;

template <int F>
__global__ void stw(int4* p, unsigned long long wrec, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const unsigned long long base = (i / wrec) * wrec;
    const unsigned long long r = base + mix(i ^ ((unsigned long long)seed << 40)) % wrec;
    const int4 v = make_int4((int)i, 1, 2, 3);
    if constexpr (F == 0) p[r] = v;
    if constexpr (F == 1) {
        typedef int i4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(i4{v.x, v.y, v.z, v.w}, reinterpret_cast<i4*>(p + r));
    }
}
__global__ void ldw(const int4* p, int* out, unsigned long long wrec, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const unsigned long long base = (i / wrec) * wrec;
    const int4 v = p[base + mix(i ^ ((unsigned long long)seed << 40)) % wrec];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x7fffffff) out[0] = 1;
}

int main() {
    int4* buf = nullptr;
    int* out = nullptr;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, kBytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const unsigned n = 1u << 26, T = 256;  // 2^26 lanes x 16 B = 1 GiB of records: every window written once
    const unsigned long long wins[] = {64ull << 10, 1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20, 256ull << 20,
                                       1ull << 30};
    for (int rep = 0; rep < 2; ++rep)
        for (unsigned long long wb : wins) {
            const unsigned long long wrec = wb / 16;
            float ms[3];
            for (int k = 0; k < 3; ++k) {
                (void)hipEventRecord(a, 0);
                if (k == 0) hipLaunchKernelGGL(stw<0>, dim3(n / T), dim3(T), 0, 0, buf, wrec, (unsigned)rep);
                if (k == 1) hipLaunchKernelGGL(stw<1>, dim3(n / T), dim3(T), 0, 0, buf, wrec, (unsigned)rep);
                if (k == 2) hipLaunchKernelGGL(ldw, dim3(n / T), dim3(T), 0, 0, buf, out, wrec, (unsigned)rep);
                (void)hipEventRecord(b, 0);
                (void)hipEventSynchronize(b);
                (void)hipEventElapsedTime(&ms[k], a, b);
            }
            printf("rep %d window %8llu KiB: store %.3f ms (%.1f G/s), nt store %.3f ms (%.1f G/s), load %.3f ms "
                   "(%.1f G/s)\n",
                   rep, wb >> 10, ms[0], n / ms[0] / 1e6, ms[1], n / ms[1] / 1e6, ms[2], n / ms[2] / 1e6);
        }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
