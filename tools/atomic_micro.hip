// Micro-benchmark: cost of random 4-byte atomics vs random loads at the KRT's access scale.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/atomic_micro tools/atomic_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ inline unsigned hsh(unsigned x) {
    x *= 0x9E3779B1u; x ^= x >> 16; x *= 0x85EBCA6Bu; x ^= x >> 13; return x;
}
// mode 0: load P[k]; 1: atomicAdd CS[k]; 2: atomicAdd CS[k] + atomicMax MX[k] (SoA);
// 3: same two atomics on one 16-B record (AoS); 4: atomicMax with read-before (skip if not larger);
// 5: two loads (P[k], SZ[k]) SoA; 6: CAS on P[k] (expected k)
__global__ void k(int mode, int* A, int* B, int4* R, int n, int span, int* sink) {
    int acc = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int key = (int)(hsh((unsigned)i) % (unsigned)span);
        switch (mode) {
            case 0: acc += __hip_atomic_load(A + key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break;
            case 1: atomicAdd(A + key, 1); break;
            case 2: atomicAdd(A + key, 1); atomicMax(B + key, i); break;
            case 3: atomicAdd(&R[key].z, 1); atomicMax(&R[key].w, i); break;
            case 4: { int c = __hip_atomic_load(B + key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); if (c < i) atomicMax(B + key, i); } break;
            case 5: acc += A[key] + B[key]; break;
            case 6: { int old = key; __hip_atomic_compare_exchange_strong(A + key, &old, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); acc += old; } break;
            case 7: acc += A[key]; break;
        }
    }
    if (acc == 0x7fffffff) *sink = acc;
}
int main() {
    const int n = 32 << 20;
    int spans[] = {1 << 20, 4 << 20, 16 << 20, 64 << 20};
    int *A, *B, *sink; int4* R;
    hipMalloc(&A, sizeof(int) * (64 << 20)); hipMalloc(&B, sizeof(int) * (64 << 20));
    hipMalloc(&R, sizeof(int4) * (64 << 20)); hipMalloc(&sink, 4);
    hipMemset(A, 0, sizeof(int) * (64 << 20)); hipMemset(B, 0, sizeof(int) * (64 << 20));
    hipMemset(R, 0, sizeof(int4) * (64 << 20));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const char* names[] = {"sc1 load", "atomicAdd", "add+max SoA", "add+max AoS", "max read-first", "2 loads SoA", "CAS", "plain load"};
    for (int s = 0; s < 4; ++s)
        for (int m = 0; m < 8; ++m) {
            hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, m, A, B, R, n, spans[s], sink);
            hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, m, A, B, R, n, spans[s], sink);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
            printf("span %3dM ints  %-16s %7.3f ms  %6.1f G lane-ops/s\n", spans[s] >> 20, names[m], ms, n / ms / 1e6);
        }
    return 0;
}
