// sort32_micro.hip — radix-sort configurations for the packed MST sort on 32-bit keys (dofs_sortfix.h,
// key32_of): n = 112 frames x (1920*1080 - 1) (u32 key, u32 frame|index) pairs. Keys: key32_of of
// weight-like doubles (30 % exact zeros, the rest sqrt of small uniforms) with the window top of the
// largest weight. Times (hipEvents, median of 5):
//   hip32      hipcub SortPairs over 32 bits (the library's default onesweep)
//   ros<R>_<T> rocprim onesweep, R bits per pass, T threads x 16 items per block
//   fkeys      the frame pass (keys-only, 7 bits), for reference
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o sort32_micro tools/sort32_micro.hip
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ inline unsigned long long mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ inline unsigned key32(unsigned long long k, int etop, int m) {  // dofs_kernels.h key32_of
    if (k >> 63) return 0xFFFFFFFFu;
    const int e = (int)((k >> 52) & 0x7FF), lo = etop - ((1 << (32 - m)) - 1);
    if (e > etop) return 0xFFFFFFFFu;
    if (e < lo) return 0u;
    return ((unsigned)(e - lo) << m) | (unsigned)((k >> (52 - m)) & ((1ull << m) - 1));
}
__global__ void k_fill(unsigned* k, unsigned* v, long n, long per, int vb) {
    const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long h = mix((unsigned long long)i);
    double w = 0.0;
    if ((h & 3) != 0) w = sqrt((double)((h >> 11) & 0xFFFFF) * (0.05 / 1048576.0));
    unsigned long long b;
    memcpy(&b, &w, 8);
    k[i] = key32(b, 1023 + 1, 27);  // weights < 0.23: the window's top at 2^1
    const long f = i / per;
    v[i] = (unsigned)(i % per) | ((unsigned)f << vb);
}

template <unsigned R, unsigned T>
using OsCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                         rocprim::radix_sort_onesweep_config<rocprim::kernel_config<T, 16>,
                                                                             rocprim::kernel_config<T, 16>, R,
                                                                             rocprim::block_radix_rank_algorithm::match>>;

int main() {
    const long per = 1920L * 1080 - 1, F = 112, n = per * F;
    const int vb = 23;
    unsigned *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, 4 * n));
    CK(hipMalloc(&k1, 4 * n));
    CK(hipMalloc(&v0, 4 * n));
    CK(hipMalloc(&v1, 4 * n));
    void* tmp = nullptr;
    size_t tb = 0;
    auto need = [&](size_t b) {
        if (b > tb) {
            if (tmp) CK(hipFree(tmp));
            CK(hipMalloc(&tmp, b));
            tb = b;
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto&& fn) {
        std::vector<float> t;
        for (int it = 0; it < 6; ++it) {
            k_fill<<<(unsigned)((n + 255) / 256), 256>>>(k0, v0, n, per, vb);
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (it) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("{\"sort\": \"%s\", \"n\": %ld, \"ms_median\": %.3f, \"ms_min\": %.3f}\n", name, n, t[t.size() / 2], t[0]);
        fflush(stdout);
    };
    size_t b = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, b, k0, k1, v0, v1, (int)n, 0, 32));
    need(b);
    timeit("hip32", [&] { CK(hipcub::DeviceRadixSort::SortPairs(tmp, b, k0, k1, v0, v1, (int)n, 0, 32)); });
#define ROS(R, T)                                                                                     \
    {                                                                                                 \
        using Cfg = OsCfg<R, T>;                                                                      \
        size_t bb = 0;                                                                                \
        CK(rocprim::radix_sort_pairs<Cfg>(nullptr, bb, k0, k1, v0, v1, (size_t)n, 0, 32));            \
        need(bb);                                                                                     \
        timeit("ros" #R "_" #T,                                                                       \
               [&] { CK(rocprim::radix_sort_pairs<Cfg>(tmp, bb, k0, k1, v0, v1, (size_t)n, 0, 32)); }); \
    }
    ROS(8, 512)
    ROS(8, 256)
    ROS(11, 512)
    ROS(11, 256)
    ROS(11, 1024)
    b = 0;
    CK(hipcub::DeviceRadixSort::SortKeys(nullptr, b, v0, v1, (int)n, vb, vb + 7));
    need(b);
    timeit("fkeys", [&] { CK(hipcub::DeviceRadixSort::SortKeys(tmp, b, v0, v1, (int)n, vb, vb + 7)); });
    return 0;
}
