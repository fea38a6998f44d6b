// Microbenchmark of the sequential Forest::merge running-mean step (tools/, not product code).
// Each variant walks a chain of L precomputed steps with one (or two) wave64s and reports ns/step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

struct In {  // per step inputs (32 B)
    float fs, wbx, wby;
    int flags;
    double r;
    int lrank, lroot;
};

__device__ __forceinline__ float rlf(float v, int k) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k)); }
__device__ __forceinline__ int rli(int v, int k) { return __builtin_amdgcn_readlane(v, k); }
__device__ __forceinline__ double rld(double v, int k) {
    long long b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)b, k), hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// V1: lane l holds step (c*64+l) inputs in registers; sequential loop reads them with readlane.
__global__ __launch_bounds__(64) void v1(const In* in, float4* out, int L) {
    const int lane = threadIdx.x;
    float mx = 1.5f, my = 0.25f;
    int rank = 3, root = 7;
    In cur = in[lane];
    for (int c = 0; c < L / 64; ++c) {
        In nx = in[((c + 1) % (L / 64)) * 64 + lane];
        float rx = 0, ry = 0; int rr = 0, ro = 0;
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            const float fs = rlf(cur.fs, k);
            const float ux = mx * fs, uy = my * fs;
            const float vx = ux + rlf(cur.wbx, k), vy = uy + rlf(cur.wby, k);
            const double r = rld(cur.r, k);
            mx = (float)((double)vx * r);
            my = (float)((double)vy * r);
            const int lr = rli(cur.lrank, k), lo = rli(cur.lroot, k), fl = rli(cur.flags, k);
            const int nroot = (fl & 1) ? (rank > lr ? root : lo) : (lr > rank ? lo : root);
            rank = rank == lr ? rank + 1 : (rank > lr ? rank : lr);
            root = nroot;
            if (lane == k) { rx = mx; ry = my; rr = rank; ro = root; }
        }
        out[c * 64 + lane] = make_float4(rx, ry, __int_as_float(rr), __int_as_float(ro));
        cur = nx;
    }
}

// V2: chunk staged in LDS (coalesced), sequential loop reads step k with uniform LDS loads.
__global__ __launch_bounds__(64) void v2(const In* in, float4* out, int L) {
    __shared__ In buf[2][64];
    const int lane = threadIdx.x;
    float mx = 1.5f, my = 0.25f;
    int rank = 3, root = 7;
    buf[0][lane] = in[lane];
    __syncthreads();
    for (int c = 0; c < L / 64; ++c) {
        const In nx = in[((c + 1) % (L / 64)) * 64 + lane];
        const In* b = buf[c & 1];
        float rx = 0, ry = 0; int rr = 0, ro = 0;
#pragma unroll 16
        for (int k = 0; k < 64; ++k) {
            const In s = b[k];
            const float vx = mx * s.fs + s.wbx, vy = my * s.fs + s.wby;
            mx = (float)((double)vx * s.r);
            my = (float)((double)vy * s.r);
            const int nroot = (s.flags & 1) ? (rank > s.lrank ? root : s.lroot) : (s.lrank > rank ? s.lroot : root);
            rank = rank == s.lrank ? rank + 1 : (rank > s.lrank ? rank : s.lrank);
            root = nroot;
            if (lane == k) { rx = mx; ry = my; rr = rank; ro = root; }
        }
        out[c * 64 + lane] = make_float4(rx, ry, __int_as_float(rr), __int_as_float(ro));
        buf[(c + 1) & 1][lane] = nx;
        __syncthreads();
    }
}

// V3: float chain only (x and y), inputs via LDS, results via LDS (lane 0 writes) — lower bound.
__global__ __launch_bounds__(64) void v3(const In* in, float4* out, int L) {
    __shared__ In buf[2][64];
    __shared__ float2 res[64];
    const int lane = threadIdx.x;
    float mx = 1.5f, my = 0.25f;
    buf[0][lane] = in[lane];
    __syncthreads();
    for (int c = 0; c < L / 64; ++c) {
        const In nx = in[((c + 1) % (L / 64)) * 64 + lane];
        const In* b = buf[c & 1];
#pragma unroll 16
        for (int k = 0; k < 64; ++k) {
            const In s = b[k];
            const float vx = mx * s.fs + s.wbx, vy = my * s.fs + s.wby;
            mx = (float)((double)vx * s.r);
            my = (float)((double)vy * s.r);
            res[k] = make_float2(mx, my);
        }
        __syncthreads();
        out[c * 64 + lane] = make_float4(res[lane].x, res[lane].y, 0.f, 0.f);
        buf[(c + 1) & 1][lane] = nx;
        __syncthreads();
    }
}

// V4: like V3 but the two channels run in two waves (one per SIMD).
__global__ __launch_bounds__(128) void v4(const In* in, float4* out, int L) {
    __shared__ In buf[2][64];
    __shared__ float res[2][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float m = wv ? 0.25f : 1.5f;
    if (wv == 0) buf[0][lane] = in[lane];
    __syncthreads();
    for (int c = 0; c < L / 64; ++c) {
        In nx;
        if (wv == 0) nx = in[((c + 1) % (L / 64)) * 64 + lane];
        const In* b = buf[c & 1];
#pragma unroll 16
        for (int k = 0; k < 64; ++k) {
            const In s = b[k];
            const float wb = wv ? s.wby : s.wbx;
            const float v = m * s.fs + wb;
            m = (float)((double)v * s.r);
            res[wv][k] = m;
        }
        __syncthreads();
        if (wv == 0) {
            out[c * 64 + lane] = make_float4(res[0][lane], res[1][lane], 0.f, 0.f);
            buf[(c + 1) & 1][lane] = nx;
        }
        __syncthreads();
    }
}

int main() {
    const int L = 1 << 20;
    std::vector<In> h(L);
    for (int i = 0; i < L; ++i) {
        h[i].fs = (float)(1000 + i);
        h[i].wbx = 1.5f; h[i].wby = 0.25f; h[i].flags = i & 1;
        h[i].r = 1.0 / (1001.0 + i); h[i].lrank = 0; h[i].lroot = i;
    }
    In* d; float4* o;
    hipMalloc(&d, sizeof(In) * L);
    hipMalloc(&o, sizeof(float4) * L);
    hipMemcpy(d, h.data(), sizeof(In) * L, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int v = 1; v <= 4; ++v) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (v == 1) v1<<<1, 64>>>(d, o, L);
            if (v == 2) v2<<<1, 64>>>(d, o, L);
            if (v == 3) v3<<<1, 64>>>(d, o, L);
            if (v == 4) v4<<<1, 128>>>(d, o, L);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep) printf("V%d: %.3f ms for %d steps = %.2f ns/step\n", v, ms, L, ms * 1e6 / L);
        }
    }
    return 0;
}
