// Does a random store smaller than a 32-byte sector make the L2 read the rest of the sector? Three kernels
// store to random sectors of a 4 GiB buffer (one store per lane, 2^26 lanes): 4 bytes, 16 bytes, and the
// whole 32 bytes (two 16-byte stores of one lane to one sector). Run under rocprofv3 --pmc FETCH_SIZE (then
// WRITE_SIZE): a partial-sector store that fills shows FETCH ≈ 32-64 B per store, a full-sector store none.
// Prints each kernel's time. Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/partial_store_micro
// tools/partial_store_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

constexpr unsigned long long kSectors = (4ull << 30) / 32;  // 4 GiB of 32-byte sectors

__global__ void st4(int* p, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const unsigned long long s = mix(i ^ ((unsigned long long)seed << 40)) % kSectors;
    p[s * 8] = (int)i;
}
__global__ void st16(int4* p, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const unsigned long long s = mix(i ^ ((unsigned long long)seed << 40)) % kSectors;
    p[s * 2] = make_int4((int)i, 1, 2, 3);
}
__global__ void st32(int4* p, unsigned seed) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const unsigned long long s = mix(i ^ ((unsigned long long)seed << 40)) % kSectors;
    p[s * 2] = make_int4((int)i, 1, 2, 3);
    p[s * 2 + 1] = make_int4(4, 5, 6, 7);
}

int main() {
    void* buf = nullptr;
    if (hipMalloc(&buf, 4ull << 30) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, 4ull << 30);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const unsigned n = 1u << 26, T = 256;
    for (int rep = 0; rep < 3; ++rep) {
        float ms[3];
        for (int k = 0; k < 3; ++k) {
            (void)hipEventRecord(a, 0);
            if (k == 0) hipLaunchKernelGGL(st4, dim3(n / T), dim3(T), 0, 0, (int*)buf, (unsigned)rep);
            if (k == 1) hipLaunchKernelGGL(st16, dim3(n / T), dim3(T), 0, 0, (int4*)buf, (unsigned)rep);
            if (k == 2) hipLaunchKernelGGL(st32, dim3(n / T), dim3(T), 0, 0, (int4*)buf, (unsigned)rep);
            (void)hipEventRecord(b, 0);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&ms[k], a, b);
        }
        printf("rep %d: 2^26 random stores: 4 B %.3f ms, 16 B %.3f ms, 32 B (two 16 B) %.3f ms\n", rep, ms[0], ms[1],
               ms[2]);
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
