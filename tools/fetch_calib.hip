// fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// pipeline's kernels use (MI355X_MICROARCH.md §HBM: only 16-B-per-lane streaming reads are calibrated
// there). Each kernel moves a known byte count over 1 GiB buffers (past the 256 MiB Infinity Cache):
//   rd4 / rd8 / rd16     coalesced streaming reads, 4 / 8 / 16 B per lane
//   wr4 / wr8 / wr16     coalesced streaming stores, 4 / 8 / 16 B per lane
//   gather16             random 16-B record reads (the KRT sweep's union-find records)
//   gather4              random 4-B reads
//   scatter8             random 8-B stores
// Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// (tools/calib.py prints counter bytes / known bytes per kernel).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

template <class T>
__global__ __launch_bounds__(256) void rd(const T* __restrict__ a, int64_t n, int* sink) {
    int acc = 0;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        const T v = a[i];
        acc ^= reinterpret_cast<const int*>(&v)[0];
    }
    if (acc == 0x7A5C3E1F) sink[0] = acc;  // never true for the zero-filled input; keeps the loads
}
template <class T>
__global__ __launch_bounds__(256) void wr(T* __restrict__ a, int64_t n) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
        T v;
        memset(&v, (int)(i & 0x7F), sizeof(T));
        a[i] = v;
    }
}
__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return x;
}
template <class T>
__global__ __launch_bounds__(256) void gather(const T* __restrict__ a, int64_t n, int64_t count, int* sink) {
    int acc = 0;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step) {
        const T v = a[mix((uint64_t)i) % (uint64_t)n];
        acc ^= reinterpret_cast<const int*>(&v)[0];
    }
    if (acc == 0x7A5C3E1F) sink[0] = acc;
}
__global__ __launch_bounds__(256) void scatter8(uint64_t* a, int64_t n, int64_t count) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += step)
        a[mix((uint64_t)i + 77) % (uint64_t)n] = (uint64_t)i;
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    char* a = nullptr;
    int* sink = nullptr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0, bytes));
    const int grid = 256 * 16;
    const int64_t cnt = (int64_t)1 << 24;  // random accesses per gather / scatter launch
    for (int rep = 0; rep < 3; ++rep) {
        rd<int><<<grid, 256>>>((const int*)a, (int64_t)(bytes / 4), sink);
        rd<uint64_t><<<grid, 256>>>((const uint64_t*)a, (int64_t)(bytes / 8), sink);
        rd<int4><<<grid, 256>>>((const int4*)a, (int64_t)(bytes / 16), sink);
        wr<int><<<grid, 256>>>((int*)a, (int64_t)(bytes / 4));
        wr<uint64_t><<<grid, 256>>>((uint64_t*)a, (int64_t)(bytes / 8));
        wr<int4><<<grid, 256>>>((int4*)a, (int64_t)(bytes / 16));
        gather<int4><<<grid, 256>>>((const int4*)a, (int64_t)(bytes / 16), cnt, sink);
        gather<int><<<grid, 256>>>((const int*)a, (int64_t)(bytes / 4), cnt, sink);
        scatter8<<<grid, 256>>>((uint64_t*)a, (int64_t)(bytes / 8), cnt);
    }
    CK(hipDeviceSynchronize());
    printf("{\"buffer_bytes\": %zu, \"random_accesses\": %lld}\n", bytes, (long long)cnt);
    CK(hipFree(a));
    CK(hipFree(sink));
    return 0;
}
