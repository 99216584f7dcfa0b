// Microbenchmark: throughput of 64-bit modular-multiply variants on gfx950 (dev tool).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef uint64_t u64;
#define CK(x) do { hipError_t e = (x); if (e) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ u64 fix2(u64 r, u64 q) { int64_t s=(int64_t)r; s = s<0? s+(int64_t)q : s; s = s>=(int64_t)q ? s-(int64_t)q : s; return (u64)s; }
// A: current (compiler u64<->f64 conversions)
__device__ __forceinline__ u64 mm_a(u64 a, u64 w, double wq, u64 q) { u64 qh = (u64)((double)a * wq); return fix2(a * w - qh * q, q); }
// B: magic-number conversions, round-to-nearest quotient, one-sided correction
__device__ __forceinline__ u64 mm_b(u64 a, u64 w, double wq, u64 q) {
    double ad = __longlong_as_double((long long)(a | 0x4330000000000000ULL)) - 4503599627370496.0;
    double y = fma(ad, wq, 4503599627370496.0);
    u64 qh = (u64)__double_as_longlong(y) & 0xFFFFFFFFFFFFFULL;
    int64_t r = (int64_t)(a * w - qh * q);
    r += (r >> 63) & (int64_t)q;
    return (u64)r;
}
// C: Shoup with umulhi
__device__ __forceinline__ u64 mm_c(u64 a, u64 w, u64 wp, u64 q) { u64 qh = __umul64hi(a, wp); u64 r = a * w - qh * q; return r >= q ? r - q : r; }

// D: all-fp64 exact remainder (values carried as doubles < 2^52):
//   p + pl = a*w exactly (fma split), qh = rint(a*w/q) (magic fma), t + tl = qh*q exactly,
//   r = (p - t) + (pl - tl) is exact (Sterbenz: p, t within a factor 2 once qh >= 1).
__device__ __forceinline__ double mm_d(double a, double w, double wq, double qd) {
    const double M = 4503599627370496.0;
    double p = a * w;
    double pl = fma(a, w, -p);
    double qh = fma(a, wq, M) - M;
    double t = qh * qd;
    double tl = fma(qh, qd, -t);
    double r = (p - t) + (pl - tl);
    return r < 0.0 ? r + qd : r;
}

template <int V>
__global__ void kern(u64* out, u64 q, u64 w, u64 wp, double wq, int iters) {
    u64 x0 = threadIdx.x + blockIdx.x, x1 = x0 + 7, x2 = x0 + 13, x3 = x0 + 29;
    for (int i = 0; i < iters; i++) {
        if (V == 0) { x0 = mm_a(x0, w, wq, q); x1 = mm_a(x1, w, wq, q); x2 = mm_a(x2, w, wq, q); x3 = mm_a(x3, w, wq, q); }
        if (V == 1) { x0 = mm_b(x0, w, wq, q); x1 = mm_b(x1, w, wq, q); x2 = mm_b(x2, w, wq, q); x3 = mm_b(x3, w, wq, q); }
        if (V == 2) { x0 = mm_c(x0, w, wp, q); x1 = mm_c(x1, w, wp, q); x2 = mm_c(x2, w, wp, q); x3 = mm_c(x3, w, wp, q); }
        if (V == 3) {
            double d0 = (double)x0, d1 = (double)x1, d2 = (double)x2, d3 = (double)x3;
            const double wd = (double)w, qd = (double)q;
            for (int k = 0; k < 16; k++) { d0 = mm_d(d0, wd, wq, qd); d1 = mm_d(d1, wd, wq, qd); d2 = mm_d(d2, wd, wq, qd); d3 = mm_d(d3, wd, wq, qd); }
            x0 = (u64)d0; x1 = (u64)d1; x2 = (u64)d2; x3 = (u64)d3;
            i += 15;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3;
}

int main() {
    const u64 q = 1125899906826241ULL;  // 2^50-ish prime, == 1 mod 2^17
    const u64 w = 123456789012345ULL % q;
    const u64 wp = (u64)(((unsigned __int128)w << 64) / q);
    const double wq = (double)w / (double)q;
    u64* out; CK(hipMalloc(&out, 8 << 20));
    const int blocks = 256 * 8, threads = 256, iters = 4096;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const char* names[] = {"fp64 (compiler cvt)", "fp64 magic + fma", "shoup umulhi", "all-fp64 exact rem"};
    u64 ref = 0;
    // host check of the all-fp64 remainder against u128 arithmetic
    {
        unsigned long long bad = 0, s = 88172645463325252ULL;
        for (int it = 0; it < 2000000; it++) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            u64 a = s % q, ww = (s >> 11) % q;
            double wq2 = (double)ww / (double)q;
            const double M = 4503599627370496.0;
            double ad = (double)a, wd = (double)ww, qd = (double)q;
            double p = ad * wd, pl = fma(ad, wd, -p), qh = fma(ad, wq2, M) - M, t = qh * qd, tl = fma(qh, qd, -t);
            double r = (p - t) + (pl - tl); r = r < 0 ? r + qd : r;
            if ((u64)r != (u64)(((unsigned __int128)a * ww) % q)) bad++;
        }
        printf("host check all-fp64 remainder: %llu mismatches / 2e6\n", bad);
    }
    for (int v = 0; v < 4; v++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            if (v == 0) kern<0><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            if (v == 1) kern<1><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            if (v == 2) kern<2><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            if (v == 3) kern<3><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            u64 h; hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
            if (rep == 1) printf("%-22s %8.3f ms  %7.1f Gmulmod/s  check %llx\n", names[v], ms, 4.0 * blocks * threads * iters / (ms * 1e6), (unsigned long long)h);
        }
    }
    return 0;
}
