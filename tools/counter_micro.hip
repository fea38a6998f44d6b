// Micro-benchmark: per-frame list counters (one int per frame, bumped by every element that appends),
// as KPathInit / KFilter / KLift use them. 32 frames x 2M elements, every element appends.
// mode 0: wave-aggregated atomicAdd with return (the compiler's atomic optimizer, uniform address);
// mode 1: block-aggregated (LDS count, one global atomic per block iteration, base broadcast);
// mode 2: like 0 but with 1 element in 8 appending.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/counter_micro tools/counter_micro.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void k(int mode, int* ctr, int* out, long n) {
    __shared__ int cnt, base;
    const int f = blockIdx.y;
    int* c = ctr + f * 64;
    for (long i0 = (long)blockIdx.x * 256; i0 < n; i0 += (long)gridDim.x * 256) {
        const long i = i0 + threadIdx.x;
        const bool want = i < n && (mode != 2 || (i & 7) == 0);
        if (mode == 1) {
            if (threadIdx.x == 0) cnt = 0;
            __syncthreads();
            int my = want ? atomicAdd(&cnt, 1) : 0;
            __syncthreads();
            if (threadIdx.x == 0) base = atomicAdd(c, cnt);
            __syncthreads();
            if (want) out[f * n + i] = base + my;
            __syncthreads();
        } else if (want) {
            out[f * n + i] = atomicAdd(c, 1);
        }
    }
}
int main() {
    const long n = 2 << 20;
    const int F = 32;
    int *ctr, *out;
    hipMalloc(&ctr, sizeof(int) * 64 * F);
    hipMalloc(&out, sizeof(int) * n * F);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"wave-aggregated", "block-aggregated", "wave-agg 1/8"};
    for (int m = 0; m < 3; ++m) {
        hipMemset(ctr, 0, sizeof(int) * 64 * F);
        hipLaunchKernelGGL(k, dim3(512, F), dim3(256), 0, 0, m, ctr, out, n);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(512, F), dim3(256), 0, 0, m, ctr, out, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-18s %8.3f ms per launch (32 frames x 2M elements)\n", names[m], ms / 5);
    }
    return 0;
}
