// Dependent-latency microbenchmark of the replay's mean-chain ops on one wave64 (tools/, not product
// code): cycles (s_memtime) per step of a chain of dependent instructions, for each op alone and for
// the full step f32 mul -> f32 add -> cvt f64 -> f64 mul -> cvt f32 (Forest::merge's running mean).
// usage: hipcc --offload-arch=gfx950 -O3 -o chain_lat tools/chain_lat.hip && ./chain_lat
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kSteps = 4096;

template <int V>
__global__ __launch_bounds__(64) void chain(const float* in, float* out, long long* cyc) {
    float v = in[threadIdx.x];
    const float a = in[64 + threadIdx.x], b = in[128 + threadIdx.x];
    const double r = 1.0 / ((double)in[192 + threadIdx.x] + 3.0);  // a genuine double (not a widened float)
    double dv = v;
    unsigned K = (unsigned)threadIdx.x, kl = (unsigned)(in[64] * 1000.0f);
    __shared__ float lds[64 * 64 + 1024];
    __shared__ float lds2[64 * 8];
    for (int i = threadIdx.x; i < 64 * 8; i += 64) lds2[i] = 1.0f + 1e-3f * (float)(i % 5);
    __syncthreads();
    const long long t0 = clock64();
#pragma unroll 16
    for (int k = 0; k < kSteps; ++k) {
        if (V == 0) v = v * a;                                  // f32 mul
        if (V == 1) dv = dv * r;                                // f64 mul
        if (V == 2) v = (float)(double)(v);                     // placeholder (optimised out)
        if (V == 3) v = (float)((double)v * r);                 // cvt f64, f64 mul, cvt f32
        if (V == 4) v = (float)((double)(v * a + b) * r);       // the full step (5 ops)
        if (V == 5) {                                           // cvt pair forced by asm
            double t;
            asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(t) : "v"(v));
            asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(v) : "v"(t));
        }
        if (V == 6) v = v + a;                                  // f32 add
        if (V == 7 || V == 8) {                                 // rank/root key step (union by rank)
            const unsigned lk = kl ^ (unsigned)k, bm = (k & 1) ? ~0u : 0u, lkp = lk + (1u << 27);
            unsigned eq = (bm & lkp) | (~bm & (K + (1u << 27)));
            unsigned ne = K > lk ? K : lk;
            asm volatile("" : "+v"(eq), "+v"(ne));
            K = (K ^ lk) < (1u << 27) ? eq : ne;
        }
        if (V == 8) v = (float)((double)(v * a + b) * r);       // both chains interleaved
        if (V == 9) {                                           // the full step plus an LDS store per step
            v = (float)((double)(v * a + b) * r);
            lds[(k & 63) * 64 + threadIdx.x] = v;
        }
        if (V == 10) {  // the full step plus an LDS store to one of two addresses (lanes by parity)
            v = (float)((double)(v * a + b) * r);
            lds[(k & 63) * 2 + (threadIdx.x & 1)] = v;
        }
        if (V == 11) {  // as 10, but only lanes 0 and 1 store (the rest to distinct dummy words)
            v = (float)((double)(v * a + b) * r);
            lds[threadIdx.x < 2 ? (k & 63) * 2 + threadIdx.x : 128 + (k & 15) * 64 + threadIdx.x] = v;
        }
        if (V == 12) {  // step inputs read from LDS (all lanes one of two addresses) + store as 10
            const float* q = lds2 + (k & 63) * 8 + (threadIdx.x & 1) * 4;
            const float fa = q[0], fb = q[1];
            v = (float)((double)(v * fa + fb) * r);
            lds[(k & 63) * 2 + (threadIdx.x & 1)] = v;
        }
    }
    const long long t1 = clock64();
    out[threadIdx.x] = v + (float)dv + (float)K + lds[threadIdx.x];
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int V>
void run(const char* name, const float* in, float* out, long long* cyc) {
    hipLaunchKernelGGL(chain<V>, dim3(1), dim3(64), 0, 0, in, out, cyc);
    hipLaunchKernelGGL(chain<V>, dim3(1), dim3(64), 0, 0, in, out, cyc);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-34s %7.2f cycles per step\n", name, (double)c / kSteps);
}

int main() {
    float h[256];
    for (int i = 0; i < 256; ++i) h[i] = 1.0f + 1e-3f * (float)(i % 7);
    float *in, *out;
    long long* cyc;
    hipMalloc(&in, sizeof(h));
    hipMalloc(&out, 256 * sizeof(float));
    hipMalloc(&cyc, 8);
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>("f32 mul", in, out, cyc);
    run<6>("f32 add", in, out, cyc);
    run<1>("f64 mul", in, out, cyc);
    run<5>("cvt f64 + cvt f32", in, out, cyc);
    run<3>("cvt f64, f64 mul, cvt f32", in, out, cyc);
    run<4>("full step (mul, add, cvt, mul, cvt)", in, out, cyc);
    run<7>("rank/root key step", in, out, cyc);
    run<8>("full step + key step", in, out, cyc);
    run<9>("full step + LDS store", in, out, cyc);
    run<10>("full step + same-address LDS store", in, out, cyc);
    run<11>("full step + 2-lane store (dummies)", in, out, cyc);
    run<12>("LDS inputs + step + same-addr store", in, out, cyc);
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    printf("clock rate attribute: %d kHz (clock64 counts shader cycles)\n", clk);
    return 0;
}
