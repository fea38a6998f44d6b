// sort_check.hip — hipcub SortPairs over a bit range [cut, 64) of u64 weight-like keys: the output must be
// the stable order of the truncated keys (a permutation of the input values). usage: sort_check n cut [end_bit]
// Measured (ROCm 7.2 image): [cut, 64) with cut > 0 is wrong for 2000 <= n <= 1M (the merge-sort path),
// right from 1.5M (onesweep) and for [0, 64).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <numeric>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 230396;
    const int cut = argc > 2 ? atoi(argv[2]) : 24;
    const int endb = argc > 3 ? atoi(argv[3]) : 64;
    std::vector<unsigned long long> k(n);
    std::vector<unsigned> v(n);
    unsigned long long s = 88172645463325252ull;
    for (long i = 0; i < n; ++i) {
        s ^= s << 13, s ^= s >> 7, s ^= s << 17;
        double w = (s & 3) ? sqrt((double)((s >> 11) & 0xFFFFF) * (0.05 / 1048576.0)) : 0.0;
        memcpy(&k[i], &w, 8);
        v[i] = (unsigned)i;
    }
    unsigned long long *k0, *k1;
    unsigned *v0, *v1;
    CK(hipMalloc(&k0, 8 * n));
    CK(hipMalloc(&k1, 8 * n));
    CK(hipMalloc(&v0, 4 * n));
    CK(hipMalloc(&v1, 4 * n));
    CK(hipMemcpy(k0, k.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, v.data(), 4 * n, hipMemcpyHostToDevice));
    size_t b = 0;
    CK(hipcub::DeviceRadixSort::SortPairs(nullptr, b, k0, k1, v0, v1, (int)n, cut, endb));
    void* t;
    CK(hipMalloc(&t, b));
    CK(hipcub::DeviceRadixSort::SortPairs(t, b, k0, k1, v0, v1, (int)n, cut, endb));
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> ko(n);
    std::vector<unsigned> vo(n);
    CK(hipMemcpy(ko.data(), k1, 8 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(vo.data(), v1, 4 * n, hipMemcpyDeviceToHost));
    const unsigned long long mask = endb >= 64 ? ~0ull : (1ull << endb) - 1ull;
    std::vector<unsigned> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](unsigned a, unsigned c) { return ((k[a] & mask) >> cut) < ((k[c] & mask) >> cut); });
    long bad = 0, badk = 0;
    for (long i = 0; i < n; ++i) {
        bad += vo[i] != idx[i];
        badk += ko[i] != k[idx[i]];
    }
    printf("n %ld bits [%d, %d) temp %zu: values off %ld, keys off %ld\n", n, cut, endb, b, bad, badk);
    return bad || badk;
}
