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

template <int V>
__global__ void kern(u64* out, u64 q, u64 w, u64 wp, double wq, int iters) {
    u64 x0 = threadIdx.x + blockIdx.x, x1 = x0 + 7, x2 = x0 + 13, x3 = x0 + 29;
    for (int i = 0; i < iters; i++) {
        if (V == 0) { x0 = mm_a(x0, w, wq, q); x1 = mm_a(x1, w, wq, q); x2 = mm_a(x2, w, wq, q); x3 = mm_a(x3, w, wq, q); }
        if (V == 1) { x0 = mm_b(x0, w, wq, q); x1 = mm_b(x1, w, wq, q); x2 = mm_b(x2, w, wq, q); x3 = mm_b(x3, w, wq, q); }
        if (V == 2) { x0 = mm_c(x0, w, wp, q); x1 = mm_c(x1, w, wp, q); x2 = mm_c(x2, w, wp, q); x3 = mm_c(x3, w, wp, q); }
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
    const char* names[] = {"fp64 (compiler cvt)", "fp64 magic + fma", "shoup umulhi"};
    u64 ref = 0;
    for (int v = 0; v < 3; v++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(a);
            if (v == 0) kern<0><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            if (v == 1) kern<1><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            if (v == 2) kern<2><<<blocks, threads>>>(out, q, w, wp, wq, iters);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            u64 h; hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost);
            if (rep == 1) printf("%-22s %8.3f ms  %7.1f Gmulmod/s  check %llx\n", names[v], ms, 4.0 * blocks * threads * iters / (ms * 1e6), (unsigned long long)h);
        }
    }
    return 0;
}
